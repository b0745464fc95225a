#!/bin/bash
# Counter passes over tools/frame_bench.py (the record-mark walk kernels):
# kernel trace + stats, then SQ instruction / wait counters and HBM bytes in
# separate passes (MI355X_MICROARCH.md: one block's counters per pass).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fr_trace -o run -- python3 $R/tools/frame_bench.py > $O/fr_trace.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/fr_sq1 -o run -- python3 $R/tools/frame_bench.py > $O/fr_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/fr_sq2 -o run -- python3 $R/tools/frame_bench.py > $O/fr_sq2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fr_fetch -o run -- python3 $R/tools/frame_bench.py > $O/fr_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/fr_write -o run -- python3 $R/tools/frame_bench.py > $O/fr_write.log 2>&1
