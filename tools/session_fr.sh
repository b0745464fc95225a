#!/bin/bash
# Frame walk iteration: parity (stop at the first failure), bench, per-kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
TAG=${1:-fr}
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py -x -q $T -m gpu > gpurun_out/${TAG}_tests.log 2>&1 || { echo "frame tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python -u tools/frame_bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { echo "frame_bench failed"; tail -20 gpurun_out/${TAG}_bench.log; exit 1; }
cat gpurun_out/${TAG}_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace -o run -- python3 $GRAFT_REPO_ROOT/tools/frame_bench.py > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace.log 2>&1 || { echo "trace failed"; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/trace_split.py $(find $GRAFT_REPO_ROOT/gpurun_out/${TAG}_trace -name "*kernel_trace.csv" | head -1) k_fr_
