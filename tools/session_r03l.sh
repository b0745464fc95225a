#!/bin/bash
# Record-major encode with marks written per record: record-path parity
# (raw and record-marked), then the per-config rocprofv3 session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py tests/test_spec_counts.py -x -q -m gpu $T > gpurun_out/t_rm.log 2>&1 || { echo "parity failed"; tail -30 gpurun_out/t_rm.log; exit 1; }
tail -2 gpurun_out/t_rm.log
exec bash tools/profile_configs.sh
