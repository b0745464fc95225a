#!/bin/bash
# rocprofv3 kernel trace + stats of tools/frame_bench.py (record-mark walk).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/fr_trace -o run -- python3 $R/tools/frame_bench.py > $R/gpurun_out/fr_trace.log 2>&1
