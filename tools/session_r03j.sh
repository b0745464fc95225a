#!/bin/bash
# Group encode with G lanes per record (tuning key 32): group parity tests,
# then the group / conditional-tape benches at G = 64, 16, 8, 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
steps=("t_grp:300:python -u -m pytest tests/test_groups.py tests/test_group_cond.py tests/test_rpcgen.py -x -q -m gpu $T")
for g in 64 16 8 4; do
  steps+=("gb$g:200:XDRG_TUNE=32=$g python -u tools/group_bench.py && XDRG_TUNE=32=$g python -u tools/cond_bench.py")
done
exec tools/gpu_session.sh "${steps[@]}"
