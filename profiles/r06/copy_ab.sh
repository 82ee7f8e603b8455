#!/bin/bash
# round 6: the host-boundary staging copy, A/B on one box (interleaved x2):
#   new     stream_copy (256 KiB pieces over 4 threads, in-order DMA spans) + NT stores
#   nt0     stream_copy + memcpy
#   r05     round 5: span-by-span par_copy + memcpy (KGS_STREAM_COPY=0 KGS_COPY_NT=0)
#   t2, t8  stream_copy + NT with 2 / 8 threads per copy
#   unord   stream_copy + NT, T_0's DMAs not ordered after F_0's (KGS_FEED_ORDER=0)
# VARIANTS / ABDIR select the variants and the output directory
# legs: single-proof latency (profiles/boundary_probe.py), in-flight throughput (profiles/host_inflight.py),
# the JS module's single-proof latency (time_prove.js)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/copy_ab
mkdir -p $O
PT=/tmp/kgs_bench_p20.ptau
VARIANTS=${VARIANTS:-"new nt0 r05 t2 t8"}
O=gpurun_out/r06/${ABDIR:-copy_ab}
mkdir -p $O
for rep in 1 2; do
  for v in $VARIANTS; do
    case $v in
      new) E="" ;;
      unord) E="KGS_FEED_ORDER=0" ;;
      nt0) E="KGS_COPY_NT=0" ;;
      r05) E="KGS_STREAM_COPY=0 KGS_COPY_NT=0" ;;
      t2) E="KGS_COPY_TASK_THREADS=2" ;;
      t8) E="KGS_COPY_TASK_THREADS=8" ;;
    esac
    echo "== rep $rep $v" | tee -a $O/latency.txt $O/inflight.txt $O/js.txt
    env $E timeout -k 10 300 python -u profiles/boundary_probe.py 20 5 2>&1 | grep -E "^(device|host) " >> $O/latency.txt || { echo "probe failed $v"; exit 1; }
    env $E timeout -k 10 300 python -u profiles/host_inflight.py 20 4 32 1 device,host >> $O/inflight.txt 2>&1 || { echo "inflight failed $v"; exit 1; }
    if [ -f $PT ]; then
      env $E KGS_JS_CONTEXTS=8 timeout -k 10 300 node --expose-gc kzg-grandsums-study_amd/js/test/time_prove.js $PT 20 7 0 >> $O/js.txt 2>&1 || { echo "js failed $v"; exit 1; }
    fi
  done
done
ABDIR=${ABDIR:-copy_ab} python3 - <<'PY'
import json, re, statistics as st
import os
O = "gpurun_out/r06/" + os.environ.get("ABDIR", "copy_ab")
for name in ("latency", "inflight"):
    print(open(f"{O}/{name}.txt").read()[-6000:])
for line in open(f"{O}/js.txt"):
    if line.startswith("=="): print(line.strip())
    elif line.startswith("{"):
        d = json.loads(line); print("  js best", d["ms_per_proof"], "median", d["latency_ms"]["median"], "inside", d["best_inside_libkgs"]["libkgs_timing_ms"][6:8])
PY
