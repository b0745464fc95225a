#!/bin/bash
# Runs named GPU steps on the gpurun box, each under its own time limit, logs
# under gpurun_out/.  Test failures (exit 1) do not stop the session; a crash,
# abort, fault or time-out (any other non-zero status, or a GPU fault printed
# in the step's log) ends it at once.
#   tools/gpu_session.sh "name:seconds:command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; secs=${rest%%:*}; cmd=${rest#*:}
    echo "== $name (limit ${secs}s): $cmd"
    start=$(date +%s)
    timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
    rc=$?
    echo "== $name rc=$rc ($(( $(date +%s) - start ))s)"
    tail -n 12 "gpurun_out/$name.log"
    if grep -q -E "HSA_STATUS_ERROR|illegal memory access|MEMORY_APERTURE|hipErrorIllegalAddress" "gpurun_out/$name.log"; then
        echo "== STOP: $name left a GPU fault in its log"
        exit 3
    fi
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
        echo "== STOP: $name ended with status $rc"
        exit "$rc"
    fi
done
