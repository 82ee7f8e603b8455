# JavaScript module latency with the library default (V8 collects on its own schedule) against the
# application's opt-in eager collection (node --expose-gc + KGS_JS_EAGER_GC=1: one full collection 5 ms
# after a lone proof is queued, beside its GPU work), same box, interleaved
# usage: bash profiles/js_gc_ab.sh [reps=3]
set -e
PTAU=/tmp/kgs_bench_p20.ptau
JS=kzg-grandsums-study_amd/js/test/time_prove.js
timeout -k 10 120 python -u profiles/hip_runtime_ab.py torch 20 9 | grep -E "median" | tail -1
summ() {
  python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
b = d['best_inside_libkgs']
print('best', d['latency_ms']['min'], 'median', d['latency_ms']['median'], 'max', d['latency_ms']['max'], '| exec', b['exec_ms'], '| 16-way', d.get('concurrent_proofs_per_s'))"
}
for rep in $(seq 1 ${1:-3}); do
  echo "== rep $rep default";  (unset KGS_JS_EAGER_GC; timeout -k 10 150 node --expose-gc $JS $PTAU 20 9 16 | summ)
  echo "== rep $rep eager";    KGS_JS_EAGER_GC=1 timeout -k 10 150 node --expose-gc $JS $PTAU 20 9 16 | summ
done
