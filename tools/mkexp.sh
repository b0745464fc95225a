#!/bin/bash
# experiment builds of kernels_rec.hip with -D flags: mkexp.sh name "flags"
set -e
cd "$(dirname "$0")/../oncrpc4j_amd/csrc"
mkdir -p ../../exp
B=build
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $2 -c kernels_rec.hip -o /tmp/exp_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/lib_$1.so $B/kernels_fixed.o /tmp/exp_$1.o $B/kernels_multi.o $B/kernels_frame.o $B/kernels_group.o $B/xdrg_abi.o
