#!/bin/bash
# Round-3 closing check: the whole GPU suite, smoke(), the default bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
exec tools/gpu_session.sh \
  "t_all:900:python -u -m pytest tests -x -q -m gpu $T" \
  "smoke:200:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "bench:600:python -u bench.py > gpurun_out/bench_r.json"
