#!/bin/bash
# Round 4: the clock held under k_accumulate alone / one proof at a time / four in flight, and the
# whole pipeline's SIMD cycles per VALU instruction in flight (diagnostic build; profiles/inflight_clock.py)
set -e
cd "$(dirname "$0")/../.."
R=$PWD
mkdir -p gpurun_out/ic
KGS_LIB=$R/kzg-grandsums-study_amd/lib_diag/libkgs.so timeout -k 10 300 python3 profiles/inflight_clock.py > gpurun_out/ic/inflight_clock.txt 2>&1 || { cat gpurun_out/ic/inflight_clock.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/ic/inflight_clock.txt
