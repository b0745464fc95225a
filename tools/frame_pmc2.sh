#!/bin/bash
# SQ counter passes over tools/frame_bench.py (frame walk kernels), one
# rocprofv3 --pmc run per group (MI355X_MICROARCH.md: per-block limits).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-frpmc}
mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU --output-format csv -d $O/sq1 -o run -- python3 $R/tools/frame_bench.py > $O/sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM --output-format csv -d $O/sq2 -o run -- python3 $R/tools/frame_bench.py > $O/sq2.log 2>&1
