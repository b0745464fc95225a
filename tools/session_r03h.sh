#!/bin/bash
# Truncated framed streams under every decode mode, the extent-derived count
# tests, the record-path parity suite and the config-4 A/B of key 31.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
exec tools/gpu_session.sh \
  "diag:120:python -u tools/diag_trunc.py" \
  "t_spec:300:python -u -m pytest tests/test_spec_counts.py -x -q -m gpu $T" \
  "t_par:500:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py tests/test_host_ptrs.py -x -q -m gpu $T" \
  "ab_spec:300:python -u tools/ab_knob.py --config 4 --key 31 --values 0,1,2 --rounds 5"
