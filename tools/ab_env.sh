#!/bin/bash
# Interleaved A/B of XDRG_TUNE settings through bench.py itself (one process
# per run, ROUNDS rounds): tools/ab_env.sh OUT "bench args" ROUNDS "tune A" "tune B" ...
# ("" = the defaults).  One JSON line per run: {"tune": ..., "round": ..., "line": bench line}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
out=$1; args=$2; rounds=$3; shift 3
for r in $(seq 1 "$rounds"); do
  for t in "$@"; do
    line=$(XDRG_TUNE="$t" timeout -k 10 300 python bench.py $args --cpu-seconds 0 --no-host-inclusive 2>/dev/null | grep '^{') || exit 3
    echo "{\"tune\": \"$t\", \"round\": $r, \"line\": $line}" >> "$out"
  done
done
