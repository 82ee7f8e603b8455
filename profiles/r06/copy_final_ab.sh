#!/bin/bash
# round 6: the staging copy's stores, final A/B (interleaved x3): memcpy (the new default), NT stores
# (KGS_COPY_NT=1), round 5's copy (KGS_STREAM_COPY=0) — Python single-proof latency, host path in
# flight, JS single-proof latency (15 samples)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/copy_final_ab
mkdir -p $O
PT=/tmp/kgs_bench_p20.ptau
for rep in 1 2 3; do
  for v in memcpy nt r05; do
    case $v in
      memcpy) E="" ;;
      nt) E="KGS_COPY_NT=1" ;;
      r05) E="KGS_STREAM_COPY=0" ;;
    esac
    for f in latency inflight js; do echo "== rep $rep $v" >> $O/$f.txt; done
    env $E timeout -k 10 300 python -u profiles/boundary_probe.py 20 7 2>&1 | grep -E "^(device|host) " >> $O/latency.txt || { echo "probe failed $v"; exit 1; }
    env $E timeout -k 10 300 python -u profiles/host_inflight.py 20 4 64 1 device,host >> $O/inflight.txt 2>&1 || { echo "inflight failed $v"; exit 1; }
    env $E KGS_JS_CONTEXTS=8 timeout -k 10 300 node --expose-gc kzg-grandsums-study_amd/js/test/time_prove.js $PT 20 15 0 >> $O/js.txt 2>&1 || { echo "js failed $v"; exit 1; }
  done
done
python3 - <<'PY'
import json, collections, statistics as st
O = "gpurun_out/r06/copy_final_ab"
def sect(fn):
    v = None
    for line in open(f"{O}/{fn}"):
        if line.startswith("=="): v = line.split()[3]; continue
        yield v, line
lat = collections.defaultdict(list)
for v, line in sect("latency.txt"):
    if line.startswith("host "): lat[v].append(float(line.split()[1]))
inf = collections.defaultdict(list)
for v, line in sect("inflight.txt"):
    if line.startswith("rep"):
        p = line.split(); inf[(v, p[2])].append(float(p[5]))
js = collections.defaultdict(list)
for v, line in sect("js.txt"):
    if line.startswith("{"):
        d = json.loads(line); js[v].append((d["ms_per_proof"], d["latency_ms"]["median"]))
for v in ("memcpy", "nt", "r05"):
    print(f"{v:7s} host latency median {st.median(lat[v]):.2f} ms | in flight host {st.mean(inf[(v,'host')]):.2f} device {st.mean(inf[(v,'device')]):.2f} | js best/median {js[v]}")
PY
