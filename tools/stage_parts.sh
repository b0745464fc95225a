#!/bin/bash
# Config-4 staged-kernel attribution (GPU box): the product library beside probe
# builds made HERE beforehand with tools/mkexp.sh, which applies
# tools/probes/patches/rec_probes.patch to a temporary copy of kernels_rec.hip:
#   for p in 1 2 16 32; do tools/mkexp.sh swp$p kernels_rec -DXDRG_SW_PROBE=$p; done
#   for p in 1 2 4 8 16; do tools/mkexp.sh enp$p kernels_rec -DXDRG_ENC_PROBE=$p; done
cd $GRAFT_REPO_ROOT
for lib in oncrpc4j_amd/libxdrgpu.so exp/lib_swp1.so exp/lib_swp2.so exp/lib_swp16.so exp/lib_swp32.so; do
  XDRG_LIBRARY=$PWD/$lib XDRG_PARTS=decode timeout -k 10 120 python tools/ab_stage_parts.py || exit 3
done
for lib in oncrpc4j_amd/libxdrgpu.so exp/lib_enp1.so exp/lib_enp2.so exp/lib_enp4.so exp/lib_enp8.so exp/lib_enp16.so; do
  XDRG_LIBRARY=$PWD/$lib XDRG_PARTS=encode timeout -k 10 120 python tools/ab_stage_parts.py || exit 3
done
