#!/bin/bash
# round-3 A/B session: parity of the changed kernels, NTT A/B + counters, lo-pass A/B + write bytes,
# host-boundary probe. Every GPU step under its own timeout; the script stops at the first failure.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/ab2
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py "tests/test_gpu_dist.py::test_slice_holds_one_wth_of_the_tables" -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
tail -2 $OUT/parity.log
bash profiles/r03/run_ntt_ab.sh > $OUT/ntt_ab.log 2>&1
grep "pair" $OUT/ntt_ab.log | tail -18
S=kzg-grandsums-study_amd/lib_ab/sl16/libkgs.so
C=kzg-grandsums-study_amd/lib/libkgs.so
for rep in 1 2 3; do
  for L in $S $C; do
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 10 >> $OUT/lo_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 21 10 >> $OUT/lo_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 3 skew >> $OUT/lo_ab.txt
  done
done
cat $OUT/lo_ab.txt
cd /tmp && export TMPDIR=/tmp
for tag in sl16 c; do
  L=$S; [ $tag = c ] && L=$C
  KGS_LIB=$R/$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$tag -o run -- python3 $R/profiles/msm_loop.py 20 3
  KGS_LIB=$R/$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$tag -o run -- python3 $R/profiles/msm_loop.py 20 5
done
cd $R
timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary.txt 2>&1
cat $OUT/boundary.txt
