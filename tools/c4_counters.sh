#!/bin/bash
# Instruction counters of config 4's staged kernels per variant (library via
# XDRG_LIBRARY, kernel choices via XDRG_TUNE): one rocprofv3 --pmc pass each
# (8 SQ counters, MI355X_MICROARCH.md limits), summaries under gpurun_out/c4i_*.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
run() {   # tag lib tune
    XDRG_LIBRARY=$2 XDRG_TUNE=$3 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C --output-format csv \
        -d $O/c4i_$1 -o run -- python3 $R/tools/ab_stage_parts.py 8388608 > $O/c4i_$1.log 2>&1
}
run base "" "21=0" && run runs0 "" "20=0,21=0" && run pipe "" "21=1" && \
run nobytes $R/exp/lib_NOBYTES.so "" && run nowords $R/exp/lib_NOWORDS.so "" && run nofixed $R/exp/lib_NOFIXED.so ""
