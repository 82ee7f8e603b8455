#!/bin/bash
# kernel trace of the skewed (all-equal scalars) and uniform 2^20 MSM, lo12k vs in-tree
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/lo_skew
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for t in lo12k lib; do
  L=$R/kzg-grandsums-study_amd/lib_ab/$t/libkgs.so; [ $t = lib ] && L=$R/kzg-grandsums-study_amd/lib/libkgs.so
  KGS_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/skew_$t -o run -- python3 $R/profiles/msm_loop.py 20 3 skew
  KGS_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $OUT/uni_$t -o run -- python3 $R/profiles/msm_loop.py 20 10
done
