#!/bin/bash
# NTT A/B (2^21 forward+inverse pairs, kgs_bench_ntt) of three builds, interleaved, on one box:
#   a = round-2 layout (64 KiB tiles, 32-byte element slots in LDS)
#   b = 64 KiB tiles, split 16-byte planes (bank-conflict free)
#   c = in-tree: 32 KiB tiles (128 threads) + split planes
# then one counter pass per build (SQ stall / LDS counters of the LDS passes).
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt_ab
mkdir -p $OUT
A=kzg-grandsums-study_amd/lib_ab/a/libkgs.so
B=kzg-grandsums-study_amd/lib_ab/b/libkgs.so
C=kzg-grandsums-study_amd/lib/libkgs.so
for rep in 1 2 3; do
  for L in $A $B $C; do
    for m in 21 22; do
      KGS_LIB=$L timeout -k 10 120 python3 profiles/ntt_ab.py $m 20 >> $OUT/times.txt
    done
  done
done
cat $OUT/times.txt
cd /tmp && export TMPDIR=/tmp
for tag in a c; do
  L=$A; [ $tag = c ] && L=$C
  KGS_LIB=$GRAFT_REPO_ROOT/$L timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc1_$tag -o run -- python3 $GRAFT_REPO_ROOT/profiles/ntt_ab.py 21 4
  KGS_LIB=$GRAFT_REPO_ROOT/$L timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $GRAFT_REPO_ROOT/$OUT/pmc2_$tag -o run -- python3 $GRAFT_REPO_ROOT/profiles/ntt_ab.py 21 4
done
