#!/bin/bash
# experiment builds of one kernel source with -D flags, linked with the regular
# objects of the others: mkexp.sh name kernels_rec|kernels_group|kernels_frame "flags"
#
# The attribution switches (XDRG_ENC_PROBE / XDRG_SW_PROBE in kernels_rec,
# XDRG_EL_PROBE in kernels_group: parts of a kernel switched off, wrong output)
# are not in the product sources: when the flags name one, the source is
# compiled from a temporary copy with tools/probes/patches/<rec|group>_probes.patch
# applied.  Occupancy knobs (XDRG_*_OCC) and XDRG_BRANCHY_MARK need no patch.
set -e
T=$(cd "$(dirname "$0")" && pwd)
cd "$T/../oncrpc4j_amd/csrc"
mkdir -p ../../exp
B=build
objs=""
for k in kernels_fixed kernels_rec kernels_multi kernels_frame kernels_group xdrg_abi; do
    if [ "$k" = "$2" ]; then objs="$objs /tmp/exp_$1.o"; else objs="$objs $B/$k.o"; fi
done
src=$2.hip
if [[ "$3" == *_PROBE* ]]; then
    P=$T/probes/patches/${2#kernels_}_probes.patch
    [ -f "$P" ] || { echo "mkexp: no probe patch for $2" >&2; exit 1; }
    W=$(mktemp -d /tmp/mkexp.XXXXXX)
    cp ./*.h "$W"/ && cp "$src" "$W"/
    patch -s -p1 -d "$W" < "$P"
    src=$W/$2.hip
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -I. $3 -c "$src" -o /tmp/exp_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../exp/lib_$1.so $objs
[ -z "${W:-}" ] || rm -rf "$W"
