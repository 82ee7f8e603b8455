#!/bin/bash
# 32-bit-m CIOS rows (fq29::reduce_row32) vs the all-29-bit-m build: MSM / proof parity on the new
# build, then interleaved MSM phase times (2^20, 2^21 points) and headline bench legs x3.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/m32
REPS=${REPS:-1 2 3}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "msm or golden or mid_size or large_proof or skew or pairing" -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
  tail -1 $OUT/parity.log
fi
B=kzg-grandsums-study_amd/lib_ab/m29/libkgs.so
C=kzg-grandsums-study_amd/lib/libkgs.so
for rep in $REPS; do
  for L in $B $C; do
    t=$(basename $(dirname $(dirname $L)))_$(basename $(dirname $L))
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 10 | sed "s|^|$t: |" >> $OUT/msm_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 21 10 | sed "s|^|$t: |" >> $OUT/msm_ab.txt
  done
done
cat $OUT/msm_ab.txt
timeout -k 10 900 python3 profiles/ab_bench.py 3 $B $C > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
