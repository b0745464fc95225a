#!/bin/bash
# Per-config rocprofv3 evidence (round 3): for each bench.py workload alone
# (configs 2, 2 framed, 3, 4, 4 framed; no extra configs, no host leg, no CPU
# baseline) a --kernel-trace --stats run and separate --pmc FETCH_SIZE /
# WRITE_SIZE passes (MI355X_MICROARCH.md HBM section), so each config's
# dominant-kernel average comes from its own launches.  Then
#   python tools/pmc_summary.py --per-config r03 gpurun_out/prof_cfg
# writes profiles/r03_configs/<cfg>_kernel_stats.csv and pmc_traffic.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
steps=()
for c in 2 2f 3 4 4f; do
  cfg=${c%f}; fr=""; [ "$c" != "$cfg" ] && fr="--framed"
  B="python3 $R/bench.py --config $cfg $fr --extra 0 --cpu-seconds 0 --no-host-inclusive"
  D=$R/gpurun_out/prof_cfg/c$c
  steps+=("tr_$c:300:$PROF --kernel-trace --stats -d $D/trace -o run -- $B --steps 10 --warmup 3")
  steps+=("fe_$c:300:$PROF --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o run -- $B --steps 4 --warmup 2")
  steps+=("wr_$c:300:$PROF --kernel-trace --pmc WRITE_SIZE -d $D/write -o run -- $B --steps 4 --warmup 2")
done
exec tools/gpu_session.sh "${steps[@]}"
