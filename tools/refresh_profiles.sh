#!/bin/bash
# GPU-box session that regenerates the measured evidence under gpurun_out/:
# bench lines (configs 2, 2 framed, 3, 4), a rocprofv3 kernel-trace --stats
# summary of the default bench, and separate FETCH_SIZE / WRITE_SIZE passes
# (MI355X_MICROARCH.md HBM section).  tools/pmc_summary.py then writes the
# committed profiles/ files.  Each step runs under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
PROF="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
exec tools/gpu_session.sh \
  "bench:300:python bench.py > gpurun_out/bench.json" \
  "b2f:300:python bench.py --framed --cpu-seconds 0 --no-host-inclusive > gpurun_out/b2f.json" \
  "b3:300:python bench.py --config 3 --steps 10 --warmup 3 --cpu-seconds 0 --no-host-inclusive > gpurun_out/b3.json" \
  "b4:300:python bench.py --config 4 --steps 10 --warmup 3 --cpu-seconds 0 --no-host-inclusive > gpurun_out/b4.json" \
  "trace:300:$PROF --kernel-trace --stats -d $R/gpurun_out/prof_trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-seconds 0 --no-host-inclusive" \
  "fetch:300:$PROF --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/prof_fetch -o run -- python3 $R/bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-host-inclusive" \
  "write:300:$PROF --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/prof_write -o run -- python3 $R/bench.py --steps 4 --warmup 2 --cpu-seconds 0 --no-host-inclusive"
