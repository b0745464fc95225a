#!/bin/bash
# Interleaved A/B of library builds on tools/frame_spec_probe.py (framed
# configs 2 and 4): tools/frame_ab.sh ROUNDS lib_a.so lib_b.so ... -> JSON lines
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
rounds=$1; shift
for r in $(seq 1 "$rounds"); do
    for lib in "$@"; do
        XDRG_LIBRARY=$PWD/$lib timeout -k 10 200 python3 tools/frame_spec_probe.py 10 2 4 | \
            python3 -c "import json,sys; [print(json.dumps({'round': $r, 'lib': '$lib', 'config': d['config'], 'spec_ms': d['spec']['frame_scan_ms']})) for d in map(json.loads, sys.stdin)]" || exit 3
    done
done
