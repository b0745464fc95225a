#!/bin/bash
# Truncated framed streams (HEAD library vs this tree), then config-4 traces
# under each extent-derived count mode (key 31 = 0 / 1 / 2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
B="python3 $R/bench.py --config 4 --extra 0 --cpu-seconds 0 --no-host-inclusive --steps 10 --warmup 3"
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats"
steps=("diag_head:120:env XDRG_LIBRARY=$R/exp/head/oncrpc4j_amd/libxdrgpu.so python -u tools/diag_trunc.py"
       "diag_now:120:python -u tools/diag_trunc.py")
for m in 0 1 2; do
  steps+=("tr_m$m:300:export XDRG_TUNE=31=$m && $PROF -d $R/gpurun_out/c4modes/m$m -o run -- $B")
done
exec tools/gpu_session.sh "${steps[@]}"
