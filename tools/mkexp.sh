#!/bin/bash
# experiment builds of one kernel source with -D flags, linked with the regular
# objects of the others: mkexp.sh name kernels_rec|kernels_group|kernels_frame "flags"
set -e
cd "$(dirname "$0")/../oncrpc4j_amd/csrc"
mkdir -p ../../exp
B=build
objs=""
for k in kernels_fixed kernels_rec kernels_multi kernels_frame kernels_group xdrg_abi; do
    if [ "$k" = "$2" ]; then objs="$objs /tmp/exp_$1.o"; else objs="$objs $B/$k.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics $3 -c $2.hip -o /tmp/exp_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/lib_$1.so $objs
