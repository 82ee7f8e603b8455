#!/bin/bash
# Round 4: the JS latency A/B (run_js.sh), then the ntt3w variant against the in-tree build x4 more
# (first A/B: +0.75 % in flight, inside the noise; profiles/r04/coresidency/).
set -e
cd "$(dirname "$0")/../.."
R=$PWD
bash profiles/r04/run_js.sh
timeout -k 10 900 python3 profiles/ab_bench.py 4 kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/ntt3w/libkgs.so > gpurun_out/js/ntt3w_bench_ab.txt 2>&1 || { cat gpurun_out/js/ntt3w_bench_ab.txt; exit 1; }
cat gpurun_out/js/ntt3w_bench_ab.txt
