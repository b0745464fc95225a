#!/bin/bash
# Instruction / wait / LDS-conflict counters of one bench.py workload's
# kernels, two rocprofv3 --pmc passes of 8 SQ counters each (the per-pass
# block limits of MI355X_MICROARCH.md), then one JSON summary per kernel:
#   tools/sq_counters.sh TAG "bench args" [library]
# (SQ_SCRIPT=tools/frame_bench.py: that script with those args instead of bench.py)
# -> gpurun_out/sq_TAG/{p1,p2}/..., gpurun_out/sq_TAG.json
# (python tools/sq_summary.py gpurun_out/sq_TAG > profiles/.../sq_counters_summary.json)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/sq_$1
LIB=${3:-$R/oncrpc4j_amd/libxdrgpu.so}
S=$R/${SQ_SCRIPT:-bench.py}
rm -rf "$O"
P1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVES"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
XDRG_LIBRARY=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P1 --output-format csv -d "$O/p1" -o run \
    -- python3 "$S" $2 > "$O.p1.log" 2>&1 && \
XDRG_LIBRARY=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P2 --output-format csv -d "$O/p2" -o run \
    -- python3 "$S" $2 > "$O.p2.log" 2>&1 && \
python3 "$R/tools/sq_summary.py" "$O" > "$O.json"
