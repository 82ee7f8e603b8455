#!/bin/bash
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03c
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_js_dropin.py tests/test_gpu_configs.py -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary.txt 2>&1
cat $OUT/boundary.txt
P=/tmp/kgs_bench_p20.ptau
KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js $P 20 5 16 > $OUT/js.json
cat $OUT/js.json
