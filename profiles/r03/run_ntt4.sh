#!/bin/bash
# NTT products: x2 (in-tree: two butterflies' products interleaved) vs x4 (four, -DKGS_NTT_X4) vs base;
# parity of both builds, pair timing interleaved x3, then instruction-cache counters of x2 and x4.
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt4
mkdir -p $OUT
B=kzg-grandsums-study_amd/lib_ab/base/libkgs.so
N=kzg-grandsums-study_amd/lib/libkgs.so
X=kzg-grandsums-study_amd/lib_ab/x4/libkgs.so
for L in $N $X; do
  KGS_LIB=$R$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "ntt or golden" -q --timeout 200 --timeout-method thread > $OUT/tests_$(basename $(dirname $L)).log 2>&1 || { tail -30 $OUT/tests_$(basename $(dirname $L)).log; exit 1; }
  tail -1 $OUT/tests_$(basename $(dirname $L)).log
done
for rep in 1 2 3; do
  for L in $B $N $X; do
    for m in 20 21 22; do
      KGS_LIB=$L timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 >> $OUT/times.txt
    done
  done
done
cat $OUT/times.txt
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
for L in $N $X; do
  t=$(basename $(dirname $L))
  KGS_LIB=$R/$L timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU GRBM_GUI_ACTIVE --output-format csv -d $R/$OUT/ic_$t -o run -- python3 $R/profiles/ntt_ab.py 21 4
  python3 $R/profiles/summarize_counters.py k_ntt_lds_pass $R/$OUT/ic_$t/run_counter_collection.csv > $R/$OUT/ic_$t.txt
  cat $R/$OUT/ic_$t.txt
done
