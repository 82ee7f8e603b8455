#!/bin/bash
# accumulate schedule variants vs the production build: MSM phase times, interleaved
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/sched
mkdir -p $OUT
LIBS=${LIBS:-kzg-grandsums-study_amd/lib/libkgs.so}
for rep in 1 2; do
  for L in $LIBS; do
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 10 2>/dev/null | sed "s|^.*msm|$L msm|" >> $OUT/msm.txt
  done
done
cat $OUT/msm.txt
