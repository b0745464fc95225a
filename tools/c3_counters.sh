#!/bin/bash
# Config 3's payload kernels (k_enc_payload vs k_dec_payload): the two SQ passes
# of sq_counters.sh plus one TCC pass of memory-side write requests (all vs
# 64-byte: partial-line writes show as the rest), summaries under gpurun_out/.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
A="--config 3 --steps 2 --warmup 1 --extra 0 --cpu-seconds 0 --no-host-inclusive --no-check"
bash $R/tools/sq_counters.sh c3 "$A" || exit 1
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv \
    -d $R/gpurun_out/c3_tcc -o run -- python3 $R/bench.py $A > $R/gpurun_out/c3_tcc.log 2>&1
