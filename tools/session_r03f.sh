#!/bin/bash
# Extent-derived decode counts (key 31 = 1 two passes, 2 one pass): their
# tests, the record-path parity suite, the config-4 A/B and a config-4 trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
B="python3 $R/bench.py --config 4 --extra 0 --cpu-seconds 0 --no-host-inclusive"
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
exec tools/gpu_session.sh \
  "t_spec:300:python -u -m pytest tests/test_spec_counts.py -x -q -m gpu $T" \
  "t_par:500:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py tests/test_host_ptrs.py -x -q -m gpu $T" \
  "ab_spec:300:python -u tools/ab_knob.py --config 4 --key 31 --values 0,1,2 --rounds 5" \
  "cond:300:python -u tools/cond_bench.py" \
  "tr4:300:$PROF --kernel-trace --stats -d $R/gpurun_out/c4spec2/trace -o run -- $B --steps 10 --warmup 3"
