#!/bin/bash
# proofs in flight per GPU: 4 (default) vs 5 / 6 / 8, headline leg only, interleaved x2
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/inflight
mkdir -p $OUT
for rep in 1 2; do
  for k in 4 5 6 8; do
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --no-extra-legs --no-host-leg --steps 64 --msm-reps 3 --inflight $k 2>/dev/null | python3 -c "
import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('inflight $k rep $rep', d['value'], d['latency_ms_single_proof'])" >> $OUT/inflight.txt
  done
done
cat $OUT/inflight.txt
