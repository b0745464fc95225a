#!/bin/bash
# round-4 session j: group decode place fix (generic-pointer tile offset) checked by the
# group tests, then the whole GPU suite, then session i's phase probes and counters
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
tools/gpu_session.sh \
 "t_grp:300:python -u -m pytest tests/test_chunk_map.py tests/test_volume_index.py tests/test_groups.py tests/test_group_cond.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "t_all:700:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" || exit $?
exec tools/sess_r04i.sh
