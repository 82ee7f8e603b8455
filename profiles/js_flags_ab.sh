# JavaScript module latency (7 single proofs: best / median) and 16-way throughput under node / V8
# settings, same box, interleaved; the Python host-buffer path first as the same-box reference.
# The GPU box grants the process 16 CPUs (cgroup cpu.max): V8's parallel GC helper threads run beside
# the prover's proving, copy and feeder threads.
# usage: bash profiles/js_flags_ab.sh [reps=3]
set -e
PTAU=/tmp/kgs_bench_p20.ptau
JS=kzg-grandsums-study_amd/js/test/time_prove.js
timeout -k 10 120 python -u profiles/hip_runtime_ab.py torch 20 9 | grep -E "median" | tail -1
summ() {
  python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
b = d['best_inside_libkgs']['libkgs_timing_ms']
print('best', d['latency_ms']['min'], 'median', d['latency_ms']['median'], '| rounds', ' '.join(f'{x:5.2f}' for x in b[:5]), 'copy', b[6], 'prove', b[7], '| 16-way', d.get('concurrent_proofs_per_s'))"
}
for rep in $(seq 1 ${1:-3}); do
  echo "== rep $rep default";        timeout -k 10 150 node $JS $PTAU 20 7 16 | summ
  echo "== rep $rep single-threaded-gc"; timeout -k 10 150 node --single-threaded-gc $JS $PTAU 20 7 16 | summ
  echo "== rep $rep v8-pool-size=1"; timeout -k 10 150 node --v8-pool-size=1 $JS $PTAU 20 7 16 | summ
  echo "== rep $rep copy-threads=8"; KGS_COPY_THREADS=8 timeout -k 10 150 node $JS $PTAU 20 7 16 | summ
done
