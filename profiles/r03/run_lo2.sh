#!/bin/bash
# lo pass, second rewrite (16 K chunks in one LDS tile, vector count, scan fused into the scatter,
# wave-per-bucket runs) vs lo12k (first round-3 version; round 2's sl16 build predates the current
# C-ABI and is compared through profiles/r03/lo_pass_ab.txt): MSM parity, phase times
# interleaved x3, kernel trace + WRITE_SIZE per build.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/lo2
REPS=${REPS:-1 2 3}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "msm or golden or mid_size or large_proof or skew" -q --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
  tail -1 $OUT/parity.log
fi
S=kzg-grandsums-study_amd/lib_ab/sl16/libkgs.so
P=kzg-grandsums-study_amd/lib_ab/lo12k/libkgs.so
C=kzg-grandsums-study_amd/lib/libkgs.so
for rep in $REPS; do
  for L in $P $C; do
    t=$(basename $(dirname $L))
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 10 | sed "s|^|$t: |" >> $OUT/lo_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 21 10 | sed "s|^|$t: |" >> $OUT/lo_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/msm_loop.py 20 3 skew | sed "s|^|$t: |" >> $OUT/lo_ab.txt
  done
done
cat $OUT/lo_ab.txt
cd /tmp && export TMPDIR=/tmp
for L in $P $C; do
  t=$(basename $(dirname $L))
  KGS_LIB=$R/$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/w_$t -o run -- python3 $R/profiles/msm_loop.py 20 3
  KGS_LIB=$R/$L timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$t -o run -- python3 $R/profiles/msm_loop.py 20 5
done
