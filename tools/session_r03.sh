#!/bin/bash
# Round-3 GPU session: the new parity tests (host memory, conditional groups,
# output-staged encode) and the A/Bs of the new kernel choices.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread"
exec tools/gpu_session.sh \
  "t_new:480:python -u -m pytest tests/test_host_ptrs.py tests/test_group_cond.py tests/test_groups.py tests/test_cond.py tests/test_rpcgen.py -x -q $T -m gpu" \
  "t_out:480:python -u -m pytest tests/test_gpu_parity.py -q $T -m gpu -k 'staged_out or enc_out'" \
  "ab_c4_out:300:python -u tools/ab_knob.py --config 4 --key 27 --values 0,1 --rounds 5" \
  "ab_c3_nts:300:python -u tools/ab_knob.py --config 3 --key 28 --values 1,0 --rounds 5"
