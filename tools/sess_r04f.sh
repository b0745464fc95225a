#!/bin/bash
# round-4 session f: element-parallel place with the fixed-size element path; conditional / nested shapes A/B
tools/gpu_session.sh \
 "t_grp:300:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_chunk_map.py tests/test_volume_index.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "gb_el0:200:python -u tools/group_bench.py" \
 "gb_el1k:200:XDRG_TUNE=38=1024 python -u tools/group_bench.py" \
 "gb_el512:200:XDRG_TUNE=38=512 python -u tools/group_bench.py" \
 "gb_el768:200:XDRG_TUNE=38=768 python -u tools/group_bench.py" \
 "cb_el0:300:python -u tools/cond_bench.py" \
 "cb_el1k:300:XDRG_TUNE=38=1024 python -u tools/cond_bench.py" \
 "cb_el512:300:XDRG_TUNE=38=512 python -u tools/cond_bench.py"
