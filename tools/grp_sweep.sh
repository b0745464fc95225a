#!/bin/bash
# Sweep of the group decode's LDS tile (key 33) and element descriptors per
# sub-batch (key 38) on the READDIRPLUS and volume_index shapes
# (tools/cond_bench.py, XDRG_SHAPES=plus,volume): one line per setting.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for t in "" "33=16384" "33=24576" "33=49152" "38=512" "38=2048" "33=16384,38=512" "33=49152,38=2048"; do
  XDRG_TUNE="$t" XDRG_SHAPES=plus,volume timeout -k 10 120 python3 tools/cond_bench.py 2>/dev/null | \
    python3 -c "import json,sys; [print(json.dumps({'tune': '$t', 'shape': d['shape'][:24], 'decode_ms': d['decode_ms'], 'encode_ms': d['encode_ms']})) for d in map(json.loads, sys.stdin) if not d.get('skipped')]" || exit 3
done
