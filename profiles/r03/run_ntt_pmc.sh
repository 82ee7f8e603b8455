#!/bin/bash
# Counter passes of the NTT pair at 2^21 (in-tree build): issue rate (cpi), stall shares, LDS
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/ntt_pmc
mkdir -p $OUT
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES --output-format csv -d $R/$OUT/p1 -o run -- python3 $R/profiles/ntt_ab.py 21 4
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU --output-format csv -d $R/$OUT/p2 -o run -- python3 $R/profiles/ntt_ab.py 21 4
python3 $R/profiles/summarize_counters.py k_ntt_lds_pass $R/$OUT/p1/run_counter_collection.csv $R/$OUT/p2/run_counter_collection.csv > $R/$OUT/summary.txt
cat $R/$OUT/summary.txt
