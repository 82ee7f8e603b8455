#!/bin/bash
# Round 4: the JS latency A/B (run_js.sh); NTT variants alone and in flight against the in-tree build
# (ntt3w: passes at 3 waves/SIMD, first A/B +0.75 % inside the noise; mac4: four column terms of both
# interleaved products per asm block, fewer s_nop pads); k_lo_scatter block residency alone / in flight
# (diagnostic build).
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js
mkdir -p $OUT
for L in lib lib_ab/ntt3w lib_ab/mac4 lib lib_ab/ntt3w lib_ab/mac4; do
  KGS_LIB=$R/kzg-grandsums-study_amd/$L/libkgs.so timeout -k 10 120 python3 profiles/ntt_ab.py 21 50 >> $OUT/ntt_alone.txt 2>&1
done
grep -v amdgpu.ids $OUT/ntt_alone.txt
KGS_LIB=$R/kzg-grandsums-study_amd/lib_ab/mac4/libkgs.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "ntt or golden or eval_and_division or builder" -q -x --timeout 200 --timeout-method thread > $OUT/parity_mac4.log 2>&1 || { tail -20 $OUT/parity_mac4.log; exit 1; }
echo "mac4 parity: $(tail -n 1 $OUT/parity_mac4.log)"
KGS_LIB=$R/kzg-grandsums-study_amd/lib_diag/libkgs.so timeout -k 10 300 python3 profiles/lo_residency.py > $OUT/lo_residency.txt 2>&1 || { cat $OUT/lo_residency.txt; exit 1; }
grep -v amdgpu.ids $OUT/lo_residency.txt
timeout -k 10 900 python3 profiles/ab_bench.py 3 kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so kzg-grandsums-study_amd/lib_ab/mac4/libkgs.so > $OUT/ntt_bench_ab.txt 2>&1 || { cat $OUT/ntt_bench_ab.txt; exit 1; }
cat $OUT/ntt_bench_ab.txt
bash profiles/r04/run_js.sh
