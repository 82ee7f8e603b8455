#!/bin/bash
# Instruction-issue and field-arithmetic micro-benchmarks behind DESIGN.md §3 (run on the MI355X box
# from the repo root: bash profiles/ubench/run.sh > profiles/ubench/ubench_<round>.txt; optional
# arguments select benchmarks, default all).
set -e
D=$(dirname "$0")
mkdir -p gpurun_out/ubench
LIST=${*:-issue_rates mont29 madd29 batch_affine29}
for b in $LIST; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result -mllvm -pragma-unroll-threshold=1000000 \
    "$D/$b.hip" -o gpurun_out/ubench/$b 2>/dev/null
done
for b in $LIST; do
  echo "== $b"
  timeout -k 10 120 gpurun_out/ubench/$b
  if [ "$b" = mont29 ]; then python3 "$D/mont29_check.py"; fi
done
