#!/bin/bash
# Round 4: host copies with non-temporal stores (KGS_COPY_NT, default on) against memcpy: the Python
# host-buffer path (copy / prove columns of boundary_probe.py) and the JS single call, x2 interleaved,
# then the host-path GPU tests (caller-pinned inputs, write-back) with the new copy.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/nt
mkdir -p $OUT
for rep in 1 2; do
  for v in 1 0; do
    KGS_COPY_NT=$v timeout -k 10 200 python3 profiles/boundary_probe.py 20 4 > $OUT/boundary_nt${v}_$rep.txt 2>&1
    echo "nt=$v rep $rep"; grep -E "^host " $OUT/boundary_nt${v}_$rep.txt
    KGS_COPY_NT=$v KGS_JS_CONTEXTS=8 KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 200 node kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 8 0 > $OUT/js_nt${v}_$rep.out 2>&1
    python3 -c "
import json
d=json.loads([l for l in open('$OUT/js_nt${v}_$rep.out') if l.startswith('{')][-1])
print('  js best', d['ms_per_proof'], 'walls', d['all_ms'], 'copy', [i[7] for i in d['all_inside_libkgs']])"
  done
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "caller_pinned or golden or to_mont" -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -n 1 $OUT/parity.log)"
