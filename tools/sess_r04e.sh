#!/bin/bash
# round-4 session e: tile-block one-pass decode (key 31 = 3) parity and config-4 A/B;
# element-parallel group place without scratch + SQ counters; config-3 XCD A/B; frame split
P="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
R=$GRAFT_REPO_ROOT
B3="python -u bench.py --config 3 --steps 5 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0"
B4="python -u bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-host-inclusive --extra 0"
GE="cd /tmp && XDRG_TUNE=38=1024 TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace"
tools/gpu_session.sh \
 "t_spec:300:python -u -m pytest tests/test_spec_counts.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "t_par:500:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py -x -q --timeout 120 --timeout-method thread -m gpu -k 'tile or cfg4 or cfg3'" \
 "c4_def:200:$B4" \
 "c4_t32:200:XDRG_TUNE=31=3 $B4" \
 "c4_t24:200:XDRG_TUNE=31=3,40=24576 $B4" \
 "c4_t16:200:XDRG_TUNE=31=3,40=16384 $B4" \
 "t_grp:300:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_chunk_map.py tests/test_volume_index.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "gb_el1k:200:XDRG_TUNE=38=1024 python -u tools/group_bench.py" \
 "gb_el512:200:XDRG_TUNE=38=512 python -u tools/group_bench.py" \
 "gb_sq1:120:$GE --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $R/gpurun_out/gb_sq1 -o run -- python3 $R/tools/group_bench.py readdir" \
 "gb_sq2:120:$GE --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT -d $R/gpurun_out/gb_sq2 -o run -- python3 $R/tools/group_bench.py readdir" \
 "c3_x0:200:XDRG_TUNE=37=0 $B3" \
 "c3_x1:200:$B3" \
 "fb_tr:200:$P --kernel-trace --stats -d $R/gpurun_out/prof_fb -o run -- python3 $R/tools/frame_bench.py"
