#!/bin/bash
# round 6: where F_0's arrival goes (single-proof latency, profiles/boundary_probe.py, interleaved x3)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/f0_ab
mkdir -p $O
for rep in 1 2 3; do
  for v in r05 new span8 f0copy span8copy t2; do
    case $v in
      r05) E="KGS_STREAM_COPY=0 KGS_COPY_NT=0" ;;
      new) E="" ;;
      span8) E="KGS_F0_SPAN_MB=8" ;;
      f0copy) E="KGS_F0_STREAM=copy" ;;
      span8copy) E="KGS_F0_SPAN_MB=8 KGS_F0_STREAM=copy" ;;
      t2) E="KGS_COPY_TASK_THREADS=2" ;;
    esac
    echo "== rep $rep $v" >> $O/latency.txt
    env $E timeout -k 10 300 python -u profiles/boundary_probe.py 20 5 2>&1 | grep -E "^(device|host) " >> $O/latency.txt || { echo "probe failed $v"; exit 1; }
  done
done
awk '/^==/{v=$4} /^host /{r1[v]+=$6; c[v]+=$(NF-2); t[v]+=$2; n[v]++; if (!(v in mn) || $2 < mn[v]) mn[v]=$2} /^device/{d1[v]+=$6; dt[v]+=$2; dn[v]++} END{for (k in n) printf "%-9s host mean %.2f min %.2f (r1 %.2f copy %.2f) device %.2f (r1 %.2f)\n", k, t[k]/n[k], mn[k], r1[k]/n[k], c[k]/n[k], dt[k]/dn[k], d1[k]/dn[k]}' $O/latency.txt
