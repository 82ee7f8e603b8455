# Stall breakdown (SQ wave-cycle counters) of k_accumulate alone and of the register-resident add ubench;
# build the ubench first: hipcc --offload-arch=gfx950 -O3 profiles/ubench/madd29.hip -o profiles/ubench/madd29_bin
set -e
OUT=gpurun_out/stall
mkdir -p $OUT
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/acc -o run -- python3 profiles/msm_loop.py 20 5 > $OUT/acc.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/ub -o run -- profiles/ubench/madd29_bin > $OUT/ub.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM --output-format csv -d $OUT/acc2 -o run -- python3 profiles/msm_loop.py 20 5 > $OUT/acc2.log 2>&1
