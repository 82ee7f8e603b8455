#!/bin/bash
# Round 4, VERDICT r3 Next #4: co-residency of the 1024-thread single-block / lo-pass kernels with the
# in-flight proofs' accumulate waves (two per SIMD at 168 VGPRs leave 176 per SIMD: a 1024-thread block
# of > 44 VGPRs per wave cannot start on a CU until an accumulate block there drains).
# Variants: sl_* (k_lo_scatter threads / tile), scan256 (k_tile_inverse, k_tile_carry, k_div_carries at
# 256 threads), both256 (scan256 + 256-thread lo scatter). Parity of each variant on the MSM / golden /
# division tests, the MSM phases alone, then the headline leg interleaved x2. ntt3w: the NTT LDS passes
# built for 3 waves per SIMD (<= 168 VGPRs; see run_ntt.sh).
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/lo
mkdir -p $OUT
V="kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/sl_256_16k/libkgs.so kzg-grandsums-study_amd/lib_ab/sl_256_8k/libkgs.so kzg-grandsums-study_amd/lib_ab/scan256/libkgs.so kzg-grandsums-study_amd/lib_ab/both256/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so"
for L in $V; do
  n=$(basename $(dirname $L))
  KGS_LIB=$R/$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "msm or ntt or golden or builder or eval_and_division" -q -x --timeout 200 --timeout-method thread > $OUT/parity_$n.log 2>&1 || { tail -20 $OUT/parity_$n.log; exit 1; }
  echo "$L: $(tail -1 $OUT/parity_$n.log)"
done
for L in $V; do
  for a in "20 10" "20 10 skew"; do
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py $a >> $OUT/msm_phases.txt 2>&1
  done
done
cat $OUT/msm_phases.txt
for L in kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so; do
  KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/ntt_ab.py 21 50 >> $OUT/ntt_alone.txt 2>&1
done
cat $OUT/ntt_alone.txt
timeout -k 10 800 python3 profiles/ab_bench.py 2 $V > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
