#!/bin/bash
# round-4 GPU session: receive / host tests, the branchy record-mark check
# experiment, a config-3 kernel trace, the full bench
tools/gpu_session.sh \
 "t_hr:400:python -u -m pytest tests/test_host_ptrs.py tests/test_receive.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "diag_def:120:python -u tools/diag_trunc.py" \
 "diag_br:120:XDRG_LIBRARY=exp/lib_branchy.so python -u tools/diag_trunc.py" \
 "diag_pr:120:XDRG_LIBRARY=exp/lib_branchy_printf.so python -u tools/diag_trunc.py" \
 "prof_c3:200:cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c3 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config 3 --steps 3 --warmup 1 --cpu-seconds 0 --no-host-inclusive" \
 "bench_b:600:python -u bench.py"
