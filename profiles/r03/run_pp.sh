#!/bin/bash
# accumulate loop: ping-pong point buffers + prefetched bucket ends (lib = 168-VGPR shared build,
# pp176 = 176-VGPR shared build) vs the previous loop (m32): MSM / proof parity on lib, then
# interleaved MSM phase times and headline bench x3.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/pp
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  for L in ${TEST_LIBS:-kzg-grandsums-study_amd/lib/libkgs.so}; do
    KGS_LIB=$R/$L timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "msm or golden or mid_size or large_proof or skew or pairing" -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
    echo "$L: $(tail -1 $OUT/parity.log)"
  done
fi
LIBS=${LIBS:-"kzg-grandsums-study_amd/lib_ab/m32/libkgs.so kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/pp176/libkgs.so"}
OUT=$R/gpurun_out/${TAG:-pp}; mkdir -p $OUT
for rep in 1 2; do
  for L in $LIBS; do
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 10 2>/dev/null | sed "s|^.*msm|$L msm|" >> $OUT/msm.txt
  done
done
cat $OUT/msm.txt
timeout -k 10 900 python3 profiles/ab_bench.py 3 $LIBS > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
