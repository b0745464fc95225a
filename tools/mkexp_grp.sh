#!/bin/bash
# experiment builds of kernels_group.hip with -D flags: mkexp_grp.sh name "flags"
set -e
cd "$(dirname "$0")/../oncrpc4j_amd/csrc"
mkdir -p ../../exp
B=build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $2 -c kernels_group.hip -o /tmp/expg_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/lib_$1.so $B/kernels_fixed.o $B/kernels_rec.o $B/kernels_multi.o $B/kernels_frame.o /tmp/expg_$1.o $B/xdrg_abi.o
