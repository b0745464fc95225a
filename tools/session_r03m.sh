#!/bin/bash
# Lane-per-record decode through an LDS tile (tuning key 35): conditional
# tape tests, the record-path parity suite, then the conditional bench at
# tiles 0 / 8 / 16 / 32 KiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
steps=("t_cond:400:python -u -m pytest tests/test_cond.py tests/test_rpcgen.py tests/test_zerocopy.py tests/test_gpu_parity.py -x -q -m gpu $T")
for t in 0 8192 16384 32768; do
  steps+=("cb$t:200:XDRG_TUNE=35=$t python -u tools/cond_bench.py")
done
exec tools/gpu_session.sh "${steps[@]}"
