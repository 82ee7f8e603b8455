#!/bin/bash
# NTT: twiddles of the next butterfly step loaded ahead (lib) vs the round's-start tree (base):
# NTT / proof parity of lib, pair timing interleaved x3, headline bench x2, counters of lib at 2^21.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=gpurun_out/ntt6
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "ntt or golden or mid_size or large_proof" -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=kzg-grandsums-study_amd/lib_ab/base/libkgs.so
N=kzg-grandsums-study_amd/lib/libkgs.so
for rep in 1 2 3; do
  for L in $B $N; do
    for m in 20 21 22; do
      KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 2>/dev/null >> $OUT/times.txt
    done
  done
done
cat $OUT/times.txt
timeout -k 10 600 python3 profiles/ab_bench.py 2 $B $N > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/$OUT/p1 -o run -- python3 $R/profiles/ntt_ab.py 21 4 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/$OUT/p2 -o run -- python3 $R/profiles/ntt_ab.py 21 4 > /dev/null 2>&1
python3 $R/profiles/summarize_counters.py k_ntt_lds_pass $R/$OUT/p1/run_counter_collection.csv $R/$OUT/p2/run_counter_collection.csv > $R/$OUT/summary.txt
cat $R/$OUT/summary.txt
