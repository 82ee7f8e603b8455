#!/bin/bash
# Per-kernel durations of the NTT pair at 2^20 / 2^21 (kernel trace), in-tree build
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt_trace
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
for m in 20 21; do
  timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 >> $OUT/times.txt
done
cat $OUT/times.txt
cd /tmp && export TMPDIR=/tmp
for m in 20 21; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $R/$OUT/kt$m -o run -- python3 $R/profiles/ntt_ab.py $m 20
  f=$(ls $R/$OUT/kt$m/*/run_kernel_trace.csv 2>/dev/null || ls $R/$OUT/kt$m/run_kernel_trace.csv)
  python3 $R/profiles/summarize_trace.py $f $R/$OUT/kt$m.csv
done
