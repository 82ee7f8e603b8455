#!/bin/bash
# NTT: base vs x2 (interleaved products) vs in-tree (x2 + LDS slot swizzle + 32-bit index math):
# parity of the in-tree build, pair timing interleaved x3, counters of the in-tree build at 2^21.
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt5
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "ntt or golden or mid_size" -q --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
B=kzg-grandsums-study_amd/lib_ab/base/libkgs.so
X=kzg-grandsums-study_amd/lib_ab/x2/libkgs.so
N=kzg-grandsums-study_amd/lib/libkgs.so
for rep in 1 2 3; do
  for L in $B $X $N; do
    for m in 20 21 22; do
      KGS_LIB=$L timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 >> $OUT/times.txt
    done
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/$OUT/p1 -o run -- python3 $R/profiles/ntt_ab.py 21 4
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/$OUT/p2 -o run -- python3 $R/profiles/ntt_ab.py 21 4
python3 $R/profiles/summarize_counters.py k_ntt_lds_pass $R/$OUT/p1/run_counter_collection.csv $R/$OUT/p2/run_counter_collection.csv > $R/$OUT/summary.txt
