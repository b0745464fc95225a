#!/bin/bash
# frame_spec_probe.py (config 2 and 4 framed) under rocprofv3 for the product
# library and exp/lib_<name>.so builds: frame_spec_ab.sh tag name...
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=$1; shift
for n in prod "$@"; do
    O=$R/gpurun_out/ab_$T/$n; rm -rf $O; mkdir -p $O
    L=$R/oncrpc4j_amd/libxdrgpu.so; [ "$n" = prod ] || L=$R/exp/lib_$n.so
    XDRG_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- python3 $R/tools/frame_spec_probe.py 5 2 4 > $O/probe.jsonl 2> $O/probe.err || exit 1
done
