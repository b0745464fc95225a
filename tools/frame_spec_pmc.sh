#!/bin/bash
# Counters of the speculative record-mark walk on the bench's framed streams
# (tools/frame_spec_probe.py, config $1): SQ instruction passes
# (tools/sq_counters.sh) and the HBM byte passes FETCH_SIZE / WRITE_SIZE, each
# in a run of its own (MI355X_MICROARCH.md: per-pass block limits).
#   tools/frame_spec_pmc.sh CONFIG -> gpurun_out/sq_fspec$CONFIG.json, gpurun_out/fspec$CONFIG_{fetch,write}/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
C=${1:-2}
SQ_SCRIPT=tools/frame_spec_probe.py bash $R/tools/sq_counters.sh fspec$C "2 $C" && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fspec${C}_fetch -o run \
    -- python3 $R/tools/frame_spec_probe.py 2 $C > $O/fspec${C}_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/fspec${C}_write -o run \
    -- python3 $R/tools/frame_spec_probe.py 2 $C > $O/fspec${C}_write.log 2>&1
