#!/bin/bash
# Round-3 checkpoint on the GPU: the whole -m gpu suite and the default bench
# line.  Each step has its own limit; a crash, abort or time-out ends the
# session (tools/gpu_session.sh).  Per-config rocprofv3 evidence:
# tools/profile_configs.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
exec tools/gpu_session.sh \
  "gputest:700:python -u -m pytest tests -q -m gpu $T" \
  "bench:400:python -u bench.py > gpurun_out/bench_r03e.json" \
  "cond:200:python -u tools/cond_bench.py > gpurun_out/cond_bench.jsonl" \
  "groups:200:python -u tools/group_bench.py > gpurun_out/group_bench.jsonl"
