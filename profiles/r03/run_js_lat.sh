#!/bin/bash
# JS drop-in latency (inputs prepared before the timed loop) x2, then the default bench
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js_lat
mkdir -p $OUT
timeout -k 10 200 python3 profiles/boundary_probe.py 20 3 > $OUT/boundary.txt 2>&1
grep -v amdgpu.ids $OUT/boundary.txt | tail -6
for i in 1 2; do
  KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 5 16 > $OUT/js_$i.json
  cat $OUT/js_$i.json
done
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
python3 -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['latency_ms_single_proof'], json.dumps(d['host_buffer_boundary'])[:700])"
