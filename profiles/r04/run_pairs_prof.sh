#!/bin/bash
# per-kernel times and VALU counts of the paired accumulation (KGS_ACC_PAIRS=1) at 2^20 points
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/pairs_prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
KGS_ACC_PAIRS=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/profiles/msm_loop.py 20 5 > $OUT/trace.log 2>&1
KGS_ACC_PAIRS=1 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- python3 $R/profiles/msm_loop.py 20 3 > $OUT/pmc.log 2>&1
KGS_ACC_PAIRS=0 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc0 -o run -- python3 $R/profiles/msm_loop.py 20 3 > $OUT/pmc0.log 2>&1
ls -R $OUT | head -30
