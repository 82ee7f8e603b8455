#!/bin/bash
# round 6: host path in flight (4 contexts, 32 steps as the bench) by staging-store mode, interleaved x6
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/inflight_store_ab
mkdir -p $O
for rep in 1 2 3 4 5 6; do
  for v in memcpy nt; do
    case $v in memcpy) E="" ;; nt) E="KGS_COPY_NT=1" ;; esac
    echo "== rep $rep $v" >> $O/inflight.txt
    env $E timeout -k 10 300 python -u profiles/host_inflight.py 20 4 32 2 device,host >> $O/inflight.txt 2>&1 || { echo "failed $v"; exit 1; }
  done
done
python3 - <<'PY'
import collections, statistics as st
v = None; d = collections.defaultdict(list)
for line in open("gpurun_out/r06/inflight_store_ab/inflight.txt"):
    if line.startswith("=="): v = line.split()[3]; continue
    if line.startswith("rep"):
        p = line.split(); d[(v, p[2])].append(float(p[5]))
for v in ("memcpy", "nt"):
    h, dv = d[(v, "host")], d[(v, "device")]
    print(f"{v:7s} host mean {st.mean(h):.2f} median {st.median(h):.2f} | device mean {st.mean(dv):.2f} | ratio {st.mean(h)/st.mean(dv):.4f} (n={len(h)})")
PY
