#!/bin/bash
# framed config 2 and 4 receive legs, speculative walk vs exact kernels, with kernel stats
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/spec_b1
mkdir -p $O
B="python3 $R/bench.py --steps 10 --warmup 2 --extra 0 --extra-steps 5 --cpu-seconds 0 --no-host-inclusive --framed"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2f -o run -- $B --config 2 > $O/c2f.json 2> $O/c2f.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c4f -o run -- $B --config 4 > $O/c4f.json 2> $O/c4f.err || exit 1
XDRG_TUNE=47=0 timeout -k 10 300 $B --config 2 > $O/c2f_exact.json 2> $O/c2f_exact.err || exit 1
XDRG_TUNE=47=0 timeout -k 10 300 $B --config 4 > $O/c4f_exact.json 2> $O/c4f_exact.err || exit 1
