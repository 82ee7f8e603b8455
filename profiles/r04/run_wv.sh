#!/bin/bash
# Round 4: the NTT pass build chosen per context mode (in flight: 3 waves/SIMD; one proof at a time: 2),
# and the JS addon's eager collection beside a lone proof (KGS_JS_EAGER_GC). Parity, the NTT alone, the
# headline leg against the all-3-wave build x2, the JS single-call latency (8 samples, x2 interleaved)
# and the 16-way JS rate with the collection on / off.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/wv
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_quirks.py -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -n 1 $OUT/parity.log)"
for L in lib lib; do
  KGS_LIB=$R/kzg-grandsums-study_amd/$L/libkgs.so timeout -k 10 120 python3 profiles/ntt_ab.py 21 50 >> $OUT/ntt_alone.txt 2>&1
done
grep -v amdgpu.ids $OUT/ntt_alone.txt
timeout -k 10 600 python3 profiles/ab_bench.py 2 kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
timeout -k 10 200 python3 profiles/boundary_probe.py 20 2 > /dev/null 2>&1
JS=kzg-grandsums-study_amd/js/test/time_prove.js
for rep in 1 2; do
  for v in eager noeager; do
    E="KGS_JS_EAGER_GC=1"
    [ $v = noeager ] && E="KGS_JS_EAGER_GC=0"
    env $E KGS_JS_CONTEXTS=8 KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 200 node $JS /tmp/kgs_bench_p20.ptau 20 8 0 > $OUT/js_${v}_$rep.out 2>&1
    echo "$v rep $rep: $(grep '^{' $OUT/js_${v}_$rep.out | tail -n 1 | cut -c1-200)"
  done
done
for v in eager noeager; do
  E="KGS_JS_EAGER_GC=1"
  [ $v = noeager ] && E="KGS_JS_EAGER_GC=0"
  env $E KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node $JS /tmp/kgs_bench_p20.ptau 20 3 16 > $OUT/js_conc_$v.out 2>&1
  echo "$v conc: $(grep '^{' $OUT/js_conc_$v.out | tail -n 1)"
done
