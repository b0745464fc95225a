#!/bin/bash
# emit_per default 4 (adaptive): frame tests, then the default bench (the
# framed config-2 receive leg is one of its extra configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
exec tools/gpu_session.sh \
  "t_fr:300:python -u -m pytest tests/test_gpu_frame.py tests/test_rpc.py tests/test_zerocopy.py -x -q -m gpu $T" \
  "bench:400:python -u bench.py --cpu-seconds 0 --no-host-inclusive > gpurun_out/bench_q.json"
