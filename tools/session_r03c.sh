#!/bin/bash
# iostage re-check after the barrier fix: stop at the first failure
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q $T -m gpu -k 'staged_io and cfg4' > gpurun_out/t_io1.log 2>&1 || { echo "t_io1 failed"; tail -20 gpurun_out/t_io1.log; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q $T -m gpu -k 'staged_io or enc_io' > gpurun_out/t_io.log 2>&1 || { echo "t_io failed"; tail -20 gpurun_out/t_io.log; exit 1; }
tail -2 gpurun_out/t_io.log
timeout -k 10 300 python -u tools/ab_knob.py --config 4 --key 27 --values 0,2,0,2 --rounds 5 > gpurun_out/ab_c4_io.log 2>&1 || { echo "ab failed"; tail -5 gpurun_out/ab_c4_io.log; exit 1; }
timeout -k 10 300 python -u tools/ab_knob.py --config 4 --key 12 --values 8192,12288,16384 --base 27=2 --rounds 5 > gpurun_out/ab_c4_iotile.log 2>&1
grep enc_place gpurun_out/ab_c4_io.log gpurun_out/ab_c4_iotile.log
