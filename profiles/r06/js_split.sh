#!/bin/bash
# round 6: where the JS single call's time goes beside libkgs (library default, no eager GC): every
# sample's [native call wall, queue -> worker, worker -> completion] and time inside libkgs
# (time_prove.js with KGS_JS_TIME_ALL=1), next to the Python host call of the same proofs
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/js_split
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 120 python3 -c "
import bench
K = bench.load_pkg()
c = K.Context(0)
c.write_synthetic_ptau('/tmp/kgs_js_p20.ptau', 20, bench.bench_tau())
" || exit 1
for rep in 1 2; do
  KGS_JS_TIME_ALL=1 KGS_JS_CONTEXTS=8 timeout -k 10 200 node kzg-grandsums-study_amd/js/test/time_prove.js \
    /tmp/kgs_js_p20.ptau 20 15 0 > $O/time_all_$rep.json 2> $O/time_all_$rep.err || { echo "node rc=$?"; tail -5 $O/time_all_$rep.err; exit 1; }
  KGS_JS_TIME_ALL=1 KGS_JS_CONTEXTS=8 timeout -k 10 200 node --trace-gc kzg-grandsums-study_amd/js/test/time_prove.js \
    /tmp/kgs_js_p20.ptau 20 15 0 > $O/time_all_gc_$rep.txt 2>&1 || { echo "node gc rc=$?"; exit 1; }
done
python3 - <<'EOF'
import json
O = "gpurun_out/r06/js_split"
for rep in (1, 2):
    d = json.loads(open(f"{O}/time_all_{rep}.json").read().strip().splitlines()[-1])
    print(f"rep {rep}: latency {d['latency_ms']}")
    for ms, lib, call in zip(d["all_ms"], d["all_inside_libkgs"], d["all_native_call"]):
        print(f"  total {ms:7.3f}  native call {call[0]:7.3f}  q->w {call[1]:6.3f}  w->done {call[2]:6.3f}  "
              f"exec {lib[0]:7.3f}  copy {lib[7]:6.3f} prover {lib[8]:7.3f}  outside-call {ms - call[0]:6.3f}")
EOF
