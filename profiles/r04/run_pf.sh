#!/bin/bash
# Round 4: the 3-wave (in-flight) NTT build without the twiddle prefetch (spills 20-72 B instead of
# 100-164 B in the DIF passes, none in the DIT passes) against the prefetching one (lib_ab/pf3):
# parity with one-lane contexts, the headline leg x3 interleaved.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/pf
mkdir -p $OUT
KGS_LIB=$R/kzg-grandsums-study_amd/lib/libkgs.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "mid_size or golden or ntt" -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -n 1 $OUT/parity.log)"
timeout -k 10 900 python3 profiles/ab_bench.py 3 kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/pf3/libkgs.so > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
