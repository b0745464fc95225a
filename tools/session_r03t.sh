#!/bin/bash
# chunk_map tapes incl. nested unrolled arrays inside union arms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
exec tools/gpu_session.sh "t_cm:300:python -u -m pytest tests/test_chunk_map.py -x -q -m gpu $T"
