cd $GRAFT_REPO_ROOT
for r in 1 2; do
for lib in oncrpc4j_amd/libxdrgpu.so exp/lib_swp512.so; do
  XDRG_LIBRARY=$PWD/$lib XDRG_PARTS=decode timeout -k 10 120 python tools/ab_stage_parts.py >> gpurun_out/r5_lb.log 2>&1 || exit 3
done
done
