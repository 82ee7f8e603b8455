#!/bin/bash
# Host-buffer boundary A/B: per-call registration of caller buffers (KGS_HOST_REGISTER=1) vs pinned
# staging (default) vs caller-pinned inputs (probe line host_prereg); JS output buffers registered
# for their life (KGS_JS_OUT_REGISTER=1; the default when this ran, opt-in since) vs not.
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03e
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "caller_pinned or golden or mid_size" -v --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary_staging.txt 2>&1
cat $OUT/boundary_staging.txt
KGS_HOST_REGISTER=1 timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary_percall.txt 2>&1
cat $OUT/boundary_percall.txt
P=/tmp/kgs_bench_p20.ptau
for v in outreg outnoreg outreg2 outnoreg2; do
  E="KGS_JS_NO_REG=0"; case $v in outreg*) E="KGS_JS_OUT_REGISTER=1";; esac
  env $E KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js $P 20 5 16 > $OUT/js_$v.json
  echo "$v $(cat $OUT/js_$v.json)"
done
