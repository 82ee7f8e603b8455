#!/bin/bash
# Instruction-issue and field-arithmetic micro-benchmarks behind DESIGN.md §3 (run on the MI355X box
# from the repo root: bash profiles/ubench/run.sh > profiles/ubench/ubench_<round>.txt).
set -e
D=$(dirname "$0")
mkdir -p gpurun_out/ubench
for b in issue_rates mont29 madd29; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-result "$D/$b.hip" -o gpurun_out/ubench/$b
done
echo "== issue_rates"; timeout -k 10 120 gpurun_out/ubench/issue_rates
echo "== mont29";      timeout -k 10 120 gpurun_out/ubench/mont29 && python3 "$D/mont29_check.py"
echo "== madd29";      timeout -k 10 120 gpurun_out/ubench/madd29
