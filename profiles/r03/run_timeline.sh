#!/bin/bash
# kernel trace of single 2^20 grand-sum proofs (two MSM lanes, device-resident inputs): timeline
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/timeline
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt -o run -- python3 $R/profiles/prove_loop.py 20 1 > $OUT/prove_loop.txt 2>&1
python3 $R/profiles/timeline.py $OUT/kt/run_kernel_trace.csv > $OUT/timeline.txt
tail -28 $OUT/timeline.txt
