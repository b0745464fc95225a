#!/bin/bash
# Round-3 checkpoint on the GPU: the extent-derived count tests (key 31), its
# A/B on config 4, the whole -m gpu suite and the default bench line.  Each
# step has its own limit; a crash, abort or time-out ends the session
# (tools/gpu_session.sh).  Per-config rocprofv3 evidence: tools/profile_configs.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread"
exec tools/gpu_session.sh \
  "t_spec:300:python -u -m pytest tests/test_spec_counts.py -x -q -m gpu $T -p no:cacheprovider" \
  "ab_spec:300:python -u tools/ab_knob.py --config 4 --key 31 --values 0,1 --rounds 5" \
  "gputest:700:python -u -m pytest tests -q -m gpu $T -p no:cacheprovider" \
  "bench:400:python -u bench.py > gpurun_out/bench_r03e.json"
