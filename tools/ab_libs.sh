#!/bin/bash
# Interleaved A/B of library builds on one bench.py workload: every round runs
# each library once (a process each, XDRG_LIBRARY), one JSON line per run with
# the library and bench.py's kernel_ms_per_step.
#   tools/ab_libs.sh ROUNDS "bench args" lib_a.so lib_b.so ...
# (the product library is oncrpc4j_amd/libxdrgpu.so; experiment builds: tools/mkexp.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
rounds=$1; args=$2; shift 2
for r in $(seq 1 "$rounds"); do
    for lib in "$@"; do
        out=$(XDRG_LIBRARY=$PWD/$lib timeout -k 10 300 python bench.py $args) || { echo "run failed: $lib" >&2; exit 3; }
        echo "$out" | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(json.dumps({'round': $r, 'lib': '$lib', 'ms_per_step': d['ms_per_step'], 'kernel_ms_per_step': d.get('kernel_ms_per_step')}))"
    done
done
