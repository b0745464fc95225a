#!/bin/bash
# Frame scan: k_fr_emit issues its loads before its tests, the entry
# initialisation folded into k_fr_exits.  Frame tests, the bench (receive
# legs of the framed configs), a kernel trace of framed config 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
B="python3 $R/bench.py --config 2 --framed --extra 0 --cpu-seconds 0 --no-host-inclusive"
exec tools/gpu_session.sh \
  "t_fr:300:python -u -m pytest tests/test_gpu_frame.py tests/test_rpc.py tests/test_zerocopy.py -x -q -m gpu $T" \
  "bench:400:python -u bench.py --cpu-seconds 0 --no-host-inclusive > gpurun_out/bench_o.json" \
  "tr_2f:300:$PROF --kernel-trace --stats -d $R/gpurun_out/prof_o/c2f -o run -- $B --steps 10 --warmup 3"
