#!/bin/bash
# round 6: the JavaScript module's 16-way concurrency leg (time_prove.js, 16 chains x 7 proofs over the
# 8-context pool) and its single-proof latency, by staging-copy variant, interleaved x3 on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/js_lat_ab
mkdir -p $O
PT=/tmp/kgs_bench_p20.ptau
timeout -k 10 200 python -u profiles/boundary_probe.py 20 1 > /dev/null 2>&1 || { echo "ptau setup failed"; exit 1; }
for rep in 1 2 3 4; do
  for v in new r05 nt0; do
    case $v in
      new) E="" ;;
      r05) E="KGS_STREAM_COPY=0 KGS_COPY_NT=0" ;;
      nt0) E="KGS_COPY_NT=0" ;;
    esac
    echo "== rep $rep $v" >> $O/js.txt
    env $E KGS_JS_CONTEXTS=8 timeout -k 10 300 node --expose-gc kzg-grandsums-study_amd/js/test/time_prove.js $PT 20 15 0 >> $O/js.txt 2>&1 || { echo "js failed $v"; exit 1; }
  done
done
python3 - <<'PY'
import json, collections
O = "gpurun_out/r06/js_lat_ab"
v = None
res = collections.defaultdict(list)
for line in open(f"{O}/js.txt"):
    if line.startswith("=="): v = line.split()[3]
    elif line.startswith("{"):
        d = json.loads(line); res[v].append((d.get("concurrent_proofs_per_s"), d["ms_per_proof"], d["latency_ms"]["median"]))
for k, xs in res.items():
    print(k, "16-way", [x[0] for x in xs], "best", [x[1] for x in xs], "median", [x[2] for x in xs])
PY
