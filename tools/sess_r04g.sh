#!/bin/bash
# round-4 session g: element-parallel place with the block's metadata prefetched into LDS
tools/gpu_session.sh \
 "t_grp:300:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_chunk_map.py tests/test_volume_index.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "gb_el1k:200:XDRG_TUNE=38=1024 python -u tools/group_bench.py" \
 "gb_el768:200:XDRG_TUNE=38=768 python -u tools/group_bench.py" \
 "gb_el1k_t24:200:XDRG_TUNE=38=1024,33=24576 python -u tools/group_bench.py" \
 "gb_el512_t16:200:XDRG_TUNE=38=512,33=16384 python -u tools/group_bench.py" \
 "cb_el1k:300:XDRG_TUNE=38=1024 python -u tools/cond_bench.py"
