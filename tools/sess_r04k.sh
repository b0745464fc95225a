#!/bin/bash
# round-4 session k: group decode with tile-relative positions (no pointer below
# the LDS tile) under the group tests, the whole GPU suite, config-3 decode head
# words (trace) and the payload kernels' block order (key 37 A/B), the
# element-parallel place's phase probes, config-4 SQ counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
B3="python3 $R/bench.py --config 3 --extra 0 --cpu-seconds 0 --no-host-inclusive"
B4="python3 $R/bench.py --config 4 --steps 4 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0"
exec tools/gpu_session.sh \
 "t_grp:300:python -u -m pytest tests/test_chunk_map.py tests/test_volume_index.py tests/test_groups.py tests/test_group_cond.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "t_all:700:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
 "tr_3:300:$PROF --kernel-trace --stats -d $R/gpurun_out/k_c3/trace -o run -- $B3 --steps 10 --warmup 3" \
 "b3_x1:200:$B3 --steps 10 --warmup 3" \
 "b3_x0:200:XDRG_TUNE=37=0 $B3 --steps 10 --warmup 3" \
 "gb_def:200:python -u tools/group_bench.py readdir dump" \
 "gb_p1:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp1.so python -u tools/group_bench.py readdir dump" \
 "gb_p3:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp3.so python -u tools/group_bench.py readdir dump" \
 "cb:300:python -u tools/cond_bench.py" \
 "c4_sq1:120:$PROF --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/c4_sq1 -o run -- $B4" \
 "c4_sq2:120:$PROF --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/c4_sq2 -o run -- $B4"
