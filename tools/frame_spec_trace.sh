#!/bin/bash
# rocprofv3 kernel trace + stats of tools/frame_spec_probe.py (framed configs 2 and 4)
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-fst}
rm -rf $O; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/frame_spec_probe.py 5 ${2:-2 4} > $O/probe.jsonl 2> $O/probe.err
