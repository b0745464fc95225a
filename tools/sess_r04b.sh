#!/bin/bash
# round-4 session b: gather/FETCH calibration probe, config-3 decode A/B
# (heads in the payload kernel vs round 3's lib, XCD order), frame tests +
# frame bench after the k_fr_mark gmark prefetch, group kernel split
P="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
R=$GRAFT_REPO_ROOT
B3="python -u bench.py --config 3 --steps 5 --warmup 2 --cpu-seconds 0 --no-host-inclusive --extra 0"
tools/gpu_session.sh \
 "probe:120:tools/probes/build/gather_fetch" \
 "probe_fe:120:$P --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/probe_fe -o run -- $R/tools/probes/build/gather_fetch" \
 "t_frame:300:python -u -m pytest tests/test_gpu_frame.py tests/test_receive.py -x -q --timeout 120 --timeout-method thread -m gpu" \
 "fb:200:python -u tools/frame_bench.py" \
 "fb_r03:200:XDRG_LIBRARY=exp/lib_r03.so python -u tools/frame_bench.py" \
 "c3_def:200:$B3" \
 "c3_x0:200:XDRG_TUNE=37=0 $B3" \
 "c3_r03:200:XDRG_LIBRARY=exp/lib_r03.so $B3" \
 "gb_tr:200:$P --kernel-trace --stats -d $R/gpurun_out/prof_grp -o run -- python3 $R/tools/group_bench.py readdir" \
 "gb_tr_el:200:XDRG_TUNE=38=1024 $P --kernel-trace --stats -d $R/gpurun_out/prof_grp_el -o run -- python3 $R/tools/group_bench.py readdir"
