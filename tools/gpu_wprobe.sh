cd $GRAFT_REPO_ROOT
for lib in oncrpc4j_amd/libxdrgpu.so exp/lib_swp32.so exp/lib_swp64.so exp/lib_swp192.so oncrpc4j_amd/libxdrgpu.so; do
  XDRG_LIBRARY=$PWD/$lib XDRG_PARTS=decode timeout -k 10 120 python tools/ab_stage_parts.py >> gpurun_out/r5_wprobe.log 2>&1 || exit 3
done
SQ_SCRIPT=tools/frame_bench.py bash tools/sq_counters.sh fr "" || exit 4
