#!/bin/bash
# Config 4 under each extent-derived count mode (key 31 = 0 / 1 / 2): bench
# lines (wall clock), and FETCH / WRITE counter passes of modes 1 and 2.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
B="python3 $R/bench.py --config 4 --extra 0 --cpu-seconds 0 --no-host-inclusive"
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace"
steps=()
for m in 0 1 2; do
  steps+=("b_m$m:200:XDRG_TUNE=31=$m python -u bench.py --config 4 --extra 0 --cpu-seconds 0 --no-host-inclusive > gpurun_out/c4m$m.json")
done
for m in 1 2; do
  steps+=("fe_m$m:200:export XDRG_TUNE=31=$m && $PROF --pmc FETCH_SIZE -d $R/gpurun_out/c4pmc/m$m/fetch -o run -- $B --steps 4 --warmup 2")
  steps+=("wr_m$m:200:export XDRG_TUNE=31=$m && $PROF --pmc WRITE_SIZE -d $R/gpurun_out/c4pmc/m$m/write -o run -- $B --steps 4 --warmup 2")
done
exec tools/gpu_session.sh "${steps[@]}"
