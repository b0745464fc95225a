#!/bin/bash
# Counter passes over the record-path place kernels of one bench config
# (default 4): kernel trace, FETCH_SIZE, WRITE_SIZE, an SQ pass and an L2
# pass, each its own rocprofv3 run (MI355X_MICROARCH.md HBM section).
#   tools/prof_rec.sh [config] [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
CFG=${1:-4}
TAG=${2:-c$CFG}
B="python3 $R/bench.py --config $CFG --steps 3 --warmup 1 --cpu-seconds 0 --no-host-inclusive"
P="cd /tmp && TMPDIR=/tmp timeout -s KILL 120 rocprofv3 --output-format csv"
exec tools/gpu_session.sh \
  "trace_$TAG:150:$P --kernel-trace --stats -d $R/gpurun_out/p_${TAG}_trace -o run -- $B" \
  "fetch_$TAG:150:$P --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/p_${TAG}_fetch -o run -- $B" \
  "write_$TAG:150:$P --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/p_${TAG}_write -o run -- $B" \
  "sq_$TAG:150:$P --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $R/gpurun_out/p_${TAG}_sq -o run -- $B" \
  "sq2_$TAG:150:$P --kernel-trace --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY -d $R/gpurun_out/p_${TAG}_sq2 -o run -- $B" \
  "l2_$TAG:150:$P --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum -d $R/gpurun_out/p_${TAG}_l2 -o run -- $B"
