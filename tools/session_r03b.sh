#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread"
exec tools/gpu_session.sh \
  "t_io:480:python -u -m pytest tests/test_gpu_parity.py -q $T -m gpu -k 'staged_io or enc_io'" \
  "ab_c4_io:300:python -u tools/ab_knob.py --config 4 --key 27 --values 0,2,0,2 --rounds 5" \
  "ab_c4_iotile:300:python -u tools/ab_knob.py --config 4 --key 12 --values 8192,12288,16384 --base 27=2 --rounds 5" \
  "bench:600:python -u bench.py > gpurun_out/bench_full.json"
