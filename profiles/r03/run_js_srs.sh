#!/bin/bash
# JS drop-in: SRS load hop skipped when the context already holds the file's tables. JS GPU tests,
# then the latency / concurrency probe x3 (same command as bench.py's javascript_module leg).
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js_srs
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_js_dropin.py tests/test_js_log.py -m gpu -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
test -f /tmp/kgs_bench_p20.ptau || timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, '.'); import bench
K = bench.load_pkg(); c = K.Context(0); c.write_synthetic_ptau('/tmp/kgs_bench_p20.ptau', 20, bench.bench_tau()); c.close()"
for i in 1 2 3; do
  KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 5 16 >> $OUT/js.json
done
cat $OUT/js.json
