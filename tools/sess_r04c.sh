#!/bin/bash
# round-4 session c: LDS-DMA group staging + element-parallel place, config-3 heads A/B (key 39)
P="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
R=$GRAFT_REPO_ROOT
B3="python -u bench.py --config 3 --steps 5 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0"
tools/gpu_session.sh \
 "t_grp:400:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_chunk_map.py tests/test_volume_index.py tests/test_gpu_baseline_shapes.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "t_par:400:python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k 'payload or dyn or group'" \
 "gb_def:200:python -u tools/group_bench.py" \
 "gb_el1k:200:XDRG_TUNE=38=1024 python -u tools/group_bench.py" \
 "gb_el2k:200:XDRG_TUNE=38=2048 python -u tools/group_bench.py" \
 "gb_el1k_t16:200:XDRG_TUNE=38=1024,33=16384 python -u tools/group_bench.py" \
 "c3_h0:200:$B3" \
 "c3_h1:200:XDRG_TUNE=39=1 $B3" \
 "gb_tr_el:200:cd /tmp && XDRG_TUNE=38=1024 TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats -d $R/gpurun_out/prof_grp_el -o run -- python3 $R/tools/group_bench.py readdir"
