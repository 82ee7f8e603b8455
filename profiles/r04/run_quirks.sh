#!/bin/bash
# Round 4: reference-quirks tests (tests/test_gpu_quirks.py) + the parity suite, then a default bench.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/quirks
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_quirks.py tests/test_gpu_parity.py -v -x --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/tests.log | head -40; tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
cat $OUT/bench_default.json
