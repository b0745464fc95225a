#!/bin/bash
# round-4 session h: full GPU suite at the new defaults, per-config rocprofv3
# evidence (trace + FETCH_SIZE + WRITE_SIZE passes, as tools/profile_configs.sh),
# the bench line, group / conditional throughput at the defaults
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
steps=("t_all:700:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu")
for c in 2 2f 3 4 4f; do
  cfg=${c%f}; fr=""; [ "$c" != "$cfg" ] && fr="--framed"
  B="python3 $R/bench.py --config $cfg $fr --extra 0 --cpu-seconds 0 --no-host-inclusive"
  D=$R/gpurun_out/prof_cfg/c$c
  steps+=("tr_$c:300:$PROF --kernel-trace --stats -d $D/trace -o run -- $B --steps 10 --warmup 3")
  steps+=("fe_$c:300:$PROF --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o run -- $B --steps 4 --warmup 2")
  steps+=("wr_$c:300:$PROF --kernel-trace --pmc WRITE_SIZE -d $D/write -o run -- $B --steps 4 --warmup 2")
done
steps+=("gb:200:python -u tools/group_bench.py" "cb:300:python -u tools/cond_bench.py")
steps+=("bench_b:600:python -u bench.py > gpurun_out/bench_b.json")
exec tools/gpu_session.sh "${steps[@]}"
