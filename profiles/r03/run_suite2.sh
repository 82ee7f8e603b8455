#!/bin/bash
# full GPU suite, then single-proof timeline, boundary probe, JS timing and the default bench
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/suite2
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { grep -E "FAILED|Error|error" $OUT/tests.log | head -30; tail -5 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 200 python3 profiles/boundary_probe.py 20 5 > $OUT/boundary.txt 2>&1
grep -v amdgpu.ids $OUT/boundary.txt
KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 5 16 > $OUT/js.json
cat $OUT/js.json
timeout -k 10 400 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/profiles/prove_loop.py 20 1 > $OUT/prove_loop.txt 2>&1
python3 $R/profiles/timeline.py $OUT/kt/run_kernel_trace.csv > $OUT/timeline.txt
tail -26 $OUT/timeline.txt
