#!/bin/bash
# Staged repeated-group decode (tuning key 33): group parity tests, then the
# group / conditional-tape benches at decode tiles 0 (HBM), 16, 32, 64 KiB.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
steps=("t_grp:300:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_rpcgen.py -x -q -m gpu $T")
for t in 0 16384 32768 65536; do
  steps+=("gd$t:200:XDRG_TUNE=33=$t python -u tools/group_bench.py && XDRG_TUNE=33=$t python -u tools/cond_bench.py")
done
exec tools/gpu_session.sh "${steps[@]}"
