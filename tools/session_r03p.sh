#!/bin/bash
# k_fr_emit with several sub-chunks per block (tuning key 36): frame tests at
# 1 / 4 / 7, then the framed config-2 receive leg traced at 1, 2, 4, 8.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
R=$PWD
T="--timeout 120 --timeout-method thread -p no:cacheprovider"
steps=("t_fr:300:python -u -m pytest tests/test_gpu_frame.py tests/test_rpc.py -x -q -m gpu $T")
for e in 1 2 4 8; do
  steps+=("ep$e:300:cd /tmp && XDRG_TUNE=36=$e TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats -d $R/gpurun_out/prof_p/e$e -o run -- python3 $R/bench.py --config 2 --framed --extra 1 --extra-steps 5 --cpu-seconds 0 --no-host-inclusive --steps 3 --warmup 2 > $R/gpurun_out/ep$e.json")
done
exec tools/gpu_session.sh "${steps[@]}"
