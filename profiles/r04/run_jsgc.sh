#!/bin/bash
# Round 4, VERDICT r3 Next #6: the JS module's eager collection beside a lone proof (a JS-level full GC
# started 5 or 9 ms after the proof is queued; KGS_JS_EAGER_GC=0 off), single-call latency x3 interleaved (8 samples
# each), the 16-way rate, and the JS drop-in GPU tests.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/jsgc
mkdir -p $OUT
timeout -k 10 200 python3 profiles/boundary_probe.py 20 2 > $OUT/boundary.txt 2>&1
grep -v amdgpu.ids $OUT/boundary.txt | tail -8
JS=kzg-grandsums-study_amd/js/test/time_prove.js
for rep in 1 2 3; do
  for v in d5 d9 noeager; do
    E="KGS_JS_EAGER_GC=5"
    [ $v = d9 ] && E="KGS_JS_EAGER_GC=9"
    [ $v = noeager ] && E="KGS_JS_EAGER_GC=0"
    env $E KGS_JS_CONTEXTS=8 KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 200 node $JS /tmp/kgs_bench_p20.ptau 20 8 0 > $OUT/js_${v}_$rep.out 2>&1
    echo "$v rep $rep: $(grep '^{' $OUT/js_${v}_$rep.out | tail -n 1 | cut -c1-120)"
  done
done
for v in eager noeager; do
  E="KGS_JS_EAGER_GC=5"
  [ $v = noeager ] && E="KGS_JS_EAGER_GC=0"
  env $E KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node $JS /tmp/kgs_bench_p20.ptau 20 3 16 > $OUT/js_conc_$v.out 2>&1
  echo "$v conc: $(grep '^{' $OUT/js_conc_$v.out | tail -n 1 | cut -c1-400)"
done
timeout -k 10 600 python3 -u -m pytest tests/test_js_dropin.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/js_tests.log 2>&1 || { tail -20 $OUT/js_tests.log; exit 1; }
echo "js tests: $(tail -n 1 $OUT/js_tests.log)"
