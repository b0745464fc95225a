#!/bin/bash
# Closing GPU session of round 6: the full GPU suite and smoke() at HEAD, the
# group / conditional throughput, the host receive windows (READDIR and
# volume_index shapes), the frame walk alone, and the driver-shaped bench
# line; per-config rocprofv3 evidence is tools/profile_configs.sh's own call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
rm -f gpurun_out/close_*.log gpurun_out/bench_close.json
exec tools/gpu_session.sh \
  "close_tests:800:python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu" \
  "close_smoke:300:python -u -c 'import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")'" \
  "close_gb:200:python -u tools/group_bench.py" "close_cb:300:python -u tools/cond_bench.py" \
  "close_recv:300:python -u tools/recv_group_bench.py --schema volume_index --replies 131072 && python -u tools/recv_group_bench.py" \
  "close_frame:200:python -u tools/frame_spec_probe.py 10 2 4" \
  "close_bench:500:python -u bench.py > gpurun_out/bench_close.json"
