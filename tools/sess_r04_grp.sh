#!/bin/bash
# round-4 group-decode study: kernel split of READDIR / DUMP / READDIRPLUS and SQ counters of the place kernel
P="cd /tmp && TMPDIR=/tmp rocprofv3 --output-format csv"
R=$GRAFT_REPO_ROOT
tools/gpu_session.sh \
 "gb:200:python -u tools/group_bench.py" \
 "gb_tr:200:$P --kernel-trace --stats -d $R/gpurun_out/prof_grp -o run -- python3 $R/tools/group_bench.py readdir" \
 "gb_sq:120:$P --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY -d $R/gpurun_out/prof_grp_sq -o run -- python3 $R/tools/group_bench.py readdir" \
 "gb_sq2:120:$P --kernel-trace --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_BUSY_CYCLES -d $R/gpurun_out/prof_grp_sq2 -o run -- python3 $R/tools/group_bench.py readdir"
