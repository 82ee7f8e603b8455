#!/bin/bash
# kernel trace of the JavaScript drop-in's single-proof path (time_prove.js, no concurrency) next to
# prove_loop.py (Python, device-resident inputs): is the JS prover phase slower on the GPU?
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js_timeline
mkdir -p $OUT
timeout -k 10 200 python3 profiles/boundary_probe.py 20 2 > /dev/null 2>&1  # writes /tmp/kgs_bench_p20.ptau
cd /tmp && export TMPDIR=/tmp
KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_js -o run -- node $R/kzg-grandsums-study_amd/js/test/time_prove.js /tmp/kgs_bench_p20.ptau 20 3 0 > $OUT/js.json 2>&1
python3 $R/profiles/timeline.py $OUT/kt_js/run_kernel_trace.csv > $OUT/timeline_js.txt
cat $OUT/js.json | tail -1
tail -26 $OUT/timeline_js.txt
