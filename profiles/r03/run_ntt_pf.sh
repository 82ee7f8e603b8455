#!/bin/bash
# NTT pass A/B: nopf = one tile per block (round-3 split planes); pf0 = persistent grid, no prefetch;
# pf2 / pf4 = persistent with 2 / 4 of a thread's 8 tile elements prefetched during the rounds.
# Parity of the NTT first (bit-exact vs the oracle), then interleaved timings.
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt_pf
mkdir -p $OUT
for v in nopf pf0 pf2 pf4; do
  KGS_LIB=$PWD/kzg-grandsums-study_amd/lib_ab/$v/libkgs.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q -x -k "ntt or golden" --timeout 120 --timeout-method thread > $OUT/parity_$v.log 2>&1 || { tail -20 $OUT/parity_$v.log; exit 1; }
  tail -1 $OUT/parity_$v.log
done
for rep in 1 2 3; do
  for v in nopf pf0 pf2 pf4; do
    for m in 20 21 22; do
      KGS_LIB=kzg-grandsums-study_amd/lib_ab/$v/libkgs.so timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 >> $OUT/times.txt
    done
  done
done
cat $OUT/times.txt
timeout -k 10 120 python3 profiles/hostreg_probe.py 32 5 > $OUT/hostreg.txt 2>&1
cat $OUT/hostreg.txt
