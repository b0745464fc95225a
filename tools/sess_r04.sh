#!/bin/bash
# round-4 GPU session: full GPU suite, the bench line, config-3/4 kernel traces
tools/gpu_session.sh \
 "t_all:600:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
 "prof_c3:200:cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 3 --warmup 1 --cpu-seconds 0 --no-host-inclusive --extra 0" \
 "prof_c4:200:cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 5 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0" \
 "bench_a:600:python -u bench.py > gpurun_out/bench_a.json"
