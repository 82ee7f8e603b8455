#!/bin/bash
# round 6: the whole -m gpu suite (one process, per-test time limit), smoke, and one default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/${SUITE_DIR:-suite}
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=15 > $O/gpu_tests.log 2>&1 || { echo "gpu suite rc=$?"; tail -40 $O/gpu_tests.log; exit 1; }
tail -20 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench_default.json'))
h=d['host_buffer_boundary']; j=h.get('javascript_module',{})
print('value', d['value'], 'host inflight', d['host_buffer_inflight']['proofs_per_s'], d['host_buffer_inflight']['vs_device_resident'])
print('latency', d['latency_single_proof_ms'], 'host', h['latency_ms'])
print('js', j.get('ms_per_proof'), j.get('latency_ms'), 'js16', j.get('concurrent_proofs_per_s'))
print('roofline', d['roofline']['achieved'], d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
print('cpu', d['cpu_baseline'])
print('extra', {k: (v.get('proofs_per_s'), v.get('ms_per_proof'), v.get('proof_verified')) for k, v in d['extra_configs'].items() if isinstance(v, dict)})
"
