#!/bin/bash
# Round 4: the MSM row / column sums with 16 lanes per line in in-flight contexts (k_rowcol16, in-tree)
# against the block-tree k_rowcol (lib_ab/rc0); both with the Horner tile tree on contiguous threads:
# parity (MSM, golden, division), MSM phases, the headline leg x3 interleaved, and the per-proof VALU
# counter pass of the in-tree build.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/rc
mkdir -p $OUT
for L in lib lib_ab/rc0; do
  n=$(basename $L)
  KGS_LIB=$R/kzg-grandsums-study_amd/$L/libkgs.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -k "msm or golden or from_mont or mid_size or large_proof or eval_and_division" -q -x --timeout 200 --timeout-method thread > $OUT/parity_$n.log 2>&1 || { tail -20 $OUT/parity_$n.log; exit 1; }
  echo "$L: $(tail -n 1 $OUT/parity_$n.log)"
done
for L in lib lib_ab/rc0 lib lib_ab/rc0; do
  for a in "20 10" "20 10 skew"; do
    KGS_LIB=$R/kzg-grandsums-study_amd/$L/libkgs.so timeout -k 10 120 python3 profiles/msm_loop.py $a >> $OUT/msm_phases.txt 2>&1
  done
done
grep -v amdgpu.ids $OUT/msm_phases.txt
timeout -k 10 900 python3 profiles/ab_bench.py 3 kzg-grandsums-study_amd/lib/libkgs.so kzg-grandsums-study_amd/lib_ab/rc0/libkgs.so > $OUT/bench_ab.txt 2>&1 || { cat $OUT/bench_ab.txt; exit 1; }
cat $OUT/bench_ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $R/profiles/prove_loop.py 20 1 lanes1 > /dev/null 2>&1
python3 $R/profiles/summarize_valu.py $OUT/pmc_valu > $OUT/valu_share.txt
head -14 $OUT/valu_share.txt
