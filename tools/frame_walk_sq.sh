#!/bin/bash
# k_fs_walk A/B: frame_spec_probe timing, then one SQ pass (VALU / SALU / LDS
# instructions) over framed configs 2 and 4: gpurun_out/fwsq/
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/fwsq
rm -rf $O; mkdir -p $O
timeout -k 10 200 python3 $R/tools/frame_spec_probe.py 10 2 4 > $O/probe.jsonl 2> $O/probe.err && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/p1 -o run -- python3 $R/tools/frame_spec_probe.py 2 2 4 > $O/p1.log 2>&1
