# k_accumulate alone (one MSM of 2^20 points): the default launch (2 blocks per CU of the build compiled
# for 3) against -DKGS_ACC_WAVES=3 (3 blocks per CU): phase times, then one stall-counter pass each
# usage: bash profiles/acc_balance_ab.sh   (needs kzg-grandsums-study_amd/lib_ab/w3/libkgs.so:
#   make -C kzg-grandsums-study_amd EXTRA=-DKGS_ACC_WAVES=3 BUILD=build_w3 LIBOUT=lib_ab/w3/libkgs.so lib_ab/w3/libkgs.so)
set -e
OUT=gpurun_out/acc_balance
mkdir -p $OUT
W3=$PWD/kzg-grandsums-study_amd/lib_ab/w3/libkgs.so
for rep in 1 2; do
  timeout -k 10 90 python3 -u profiles/msm_loop.py 20 20
  KGS_LIB=$W3 timeout -k 10 90 python3 -u profiles/msm_loop.py 20 20
done
C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/w2 -o run -- python3 profiles/msm_loop.py 20 5 > $OUT/w2.log 2>&1
KGS_LIB=$W3 timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/w3 -o run -- python3 profiles/msm_loop.py 20 5 > $OUT/w3.log 2>&1
python3 profiles/summarize_stall.py $OUT/w2/run_counter_collection.csv
python3 profiles/summarize_stall.py $OUT/w3/run_counter_collection.csv
