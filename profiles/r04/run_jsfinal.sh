#!/bin/bash
# Round 4, last JS check: the drop-in JS GPU tests and the single-call / 16-way timing (bench leg shape)
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/jsfinal
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_js_dropin.py tests/test_js_log.py tests/test_js_verifier_log.py -m gpu -q -x --timeout 300 --timeout-method thread > $OUT/js_tests.log 2>&1 || { tail -20 $OUT/js_tests.log; exit 1; }
echo "js tests: $(tail -n 1 $OUT/js_tests.log)"
timeout -k 10 200 python3 profiles/boundary_probe.py 20 2 > $OUT/boundary.txt 2>&1
for rep in 1 2; do
  KGS_JS_CONTEXTS=8 KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 5 16 > $OUT/js_$rep.out 2>&1
  echo "rep $rep: $(grep '^{' $OUT/js_$rep.out | tail -n 1 | cut -c1-160) ... $(grep '^{' $OUT/js_$rep.out | tail -n 1 | grep -o '"concurrent_proofs_per_s":[0-9.]*')"
done
