#!/bin/bash
# GPU suite + boundary probe + default bench (one call); stops at the first failing step
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03b
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary.txt 2>&1
cat $OUT/boundary.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
