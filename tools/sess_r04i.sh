#!/bin/bash
# round-4 session i: where the element-parallel place spends its time (experiment
# builds skipping one phase each: 1 element decode, 2 record walk, 4 staging, 3 both decode phases)
tools/gpu_session.sh \
 "gb_def:200:python -u tools/group_bench.py readdir dump" \
 "gb_p1:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp1.so python -u tools/group_bench.py readdir dump" \
 "gb_p2:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp2.so python -u tools/group_bench.py readdir dump" \
 "gb_p4:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp4.so python -u tools/group_bench.py readdir dump" \
 "gb_p3:200:GB_NOCHECK=1 XDRG_LIBRARY=exp/lib_elp3.so python -u tools/group_bench.py readdir dump" \
 "t_vix:200:python -u -m pytest tests/test_volume_index.py tests/test_groups.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "cb:300:python -u tools/cond_bench.py"
R=$GRAFT_REPO_ROOT
B4="python3 $R/bench.py --config 4 --steps 4 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0"
tools/gpu_session.sh \
 "c4_sq1:120:cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/c4_sq1 -o run -- $B4" \
 "c4_sq2:120:cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/c4_sq2 -o run -- $B4"
