#!/bin/bash
# round-4 GPU session: group tests (nested groups, element-parallel place),
# group throughput A/B, the full GPU suite, config-3/4 kernel traces, the bench line
P="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
R=$GRAFT_REPO_ROOT
tools/gpu_session.sh \
 "t_grp:400:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_chunk_map.py tests/test_volume_index.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "gb_def:200:python -u tools/group_bench.py" \
 "gb_el1k:200:XDRG_TUNE=38=1024 python -u tools/group_bench.py" \
 "gb_el512_t16:200:XDRG_TUNE=38=512,33=16384 python -u tools/group_bench.py" \
 "t_all:700:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
 "prof_c3:200:$P --kernel-trace --stats -d $R/gpurun_out/prof_c3 -o run -- python3 $R/bench.py --config 3 --steps 3 --warmup 1 --cpu-seconds 0 --no-host-inclusive --extra 0" \
 "prof_c4:200:$P --kernel-trace --stats -d $R/gpurun_out/prof_c4 -o run -- python3 $R/bench.py --config 4 --steps 5 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0" \
 "bench_a:600:python -u bench.py > gpurun_out/bench_a.json"
