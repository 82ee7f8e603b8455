#!/bin/bash
# Three-round LDS passes (lds_plan): NTT parity (2^0..2^22 vs the oracles), golden proofs, then the
# 2^20/2^21/2^22 pair timing of base (6-stage passes + radix-8 tail) vs single (three-round plan, direct
# first/last rounds, one product at a time) vs new (+ two butterflies' products interleaved), interleaved x3,
# and a kernel trace of the new build at 2^21.
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt3
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "ntt or golden or mid_size or large_proof" -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B=kzg-grandsums-study_amd/lib_ab/base/libkgs.so
N=kzg-grandsums-study_amd/lib/libkgs.so
S=kzg-grandsums-study_amd/lib_ab/single/libkgs.so
for rep in 1 2 3; do
  for L in $B $S $N; do
    E=""
    for m in 20 21 22; do
      env $E KGS_LIB=$L timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 | sed "s|^|$E |" >> $OUT/times.txt
    done
  done
done
cat $OUT/times.txt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/kt21 -o run -- python3 $R/profiles/ntt_ab.py 21 20
python3 $R/profiles/summarize_trace.py $R/$OUT/kt21/run_kernel_trace.csv $R/$OUT/kt21.csv
cd $R
timeout -k 10 300 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
