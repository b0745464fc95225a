#!/bin/bash
# Receive pipeline after the stride check (tuning key 29): parity of fixed-size
# decode at explicit extents, the fixed-schema parity suite, frame walk bench
# (serial cliff), then the full bench.  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_stride_offsets.py -x -q $T -m gpu > gpurun_out/t_stride.log 2>&1 || { echo "t_stride failed"; tail -30 gpurun_out/t_stride.log; exit 1; }
tail -2 gpurun_out/t_stride.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q $T -m gpu -k 'random_parity and (staged-) ' > gpurun_out/t_fixed.log 2>&1 || { echo "t_fixed failed"; tail -30 gpurun_out/t_fixed.log; exit 1; }
tail -2 gpurun_out/t_fixed.log
timeout -k 10 300 python -u tools/frame_bench.py > gpurun_out/frame_bench.log 2>&1 || { echo "frame_bench failed"; tail -20 gpurun_out/frame_bench.log; exit 1; }
tail -12 gpurun_out/frame_bench.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r03d.json 2> gpurun_out/bench_r03d.err || { echo "bench failed"; tail -20 gpurun_out/bench_r03d.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_r03d.json").read().strip().splitlines()[-1])
print(d["value"], d["ms_per_step"], d["roofline"]["frac"])
for e in d.get("extra_configs", []):
    print({k: e.get(k) for k in ("config", "framed", "GiB_s", "ms_per_step")}, (e.get("receive") or {}).get("ms_per_step"), (e.get("receive") or {}).get("kernel_ms_per_step"))
PY
