#!/bin/bash
# Closing GPU session of a round: the whole GPU suite and smoke() at HEAD, the
# per-config rocprofv3 evidence (tools/profile_configs.sh's steps), the
# driver-shaped bench line, group / conditional throughput.  Then, here:
#   python tools/pmc_summary.py --per-config rNN gpurun_out/prof_cfg
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
rm -rf gpurun_out/prof_cfg gpurun_out/close_*.log gpurun_out/bench_close.json
steps=("close_tests:800:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu"
       "close_smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'")
for c in 2 2f 3 4 4f; do
  cfg=${c%f}; fr=""; [ "$c" != "$cfg" ] && fr="--framed"
  B="python3 $R/bench.py --config $cfg $fr --extra 0 --cpu-seconds 0 --no-host-inclusive"
  D=$R/gpurun_out/prof_cfg/c$c
  steps+=("close_tr_$c:300:$PROF --kernel-trace --stats -d $D/trace -o run -- $B --steps 10 --warmup 3")
  steps+=("close_fe_$c:300:$PROF --kernel-trace --pmc FETCH_SIZE -d $D/fetch -o run -- $B --steps 4 --warmup 2")
  steps+=("close_wr_$c:300:$PROF --kernel-trace --pmc WRITE_SIZE -d $D/write -o run -- $B --steps 4 --warmup 2")
done
steps+=("close_gb:200:python -u tools/group_bench.py" "close_cb:300:python -u tools/cond_bench.py"
        "close_bench:600:python -u bench.py > gpurun_out/bench_close.json")
exec tools/gpu_session.sh "${steps[@]}"
