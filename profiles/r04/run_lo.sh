#!/bin/bash
# Round 4, VERDICT r3 Next #4: k_lo_scatter's 1024-thread / 70 KB-LDS blocks vs smaller blocks.
# Parity of each variant on the MSM tests, the lo pass alone (MSM phases at 2^20 / 2^21 / 2^24 and a
# skewed 2^20), then the headline leg interleaved x3 (profiles/ab_bench.py).
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/lo
mkdir -p $OUT
V="kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/sl_256_8k/libkgs.so kzg-grandsums-study_amd/lib_ab/sl_512_16k/libkgs.so kzg-grandsums-study_amd/lib_ab/sl_256_16k/libkgs.so"
for L in $V; do
  KGS_LIB=$R/$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "msm or golden" -q -x --timeout 200 --timeout-method thread > $OUT/parity_$(basename $(dirname $L)).log 2>&1 || { tail -20 $OUT/parity_$(basename $(dirname $L)).log; exit 1; }
  echo "$L: $(tail -1 $OUT/parity_$(basename $(dirname $L)).log)"
done
for L in $V; do
  for a in "20 10" "21 10" "20 10 skew"; do
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py $a >> $OUT/msm_phases.txt 2>&1
  done
done
cat $OUT/msm_phases.txt
timeout -k 10 1000 python3 profiles/ab_bench.py 3 $V > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
