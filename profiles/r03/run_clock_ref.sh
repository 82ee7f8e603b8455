#!/bin/bash
# register-resident reference of the (round-3, 32-bit-m) fq29 add under the clock / VALU counters,
# then the default bench with the full-rate mad peak
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/clockref
mkdir -p $OUT
bash profiles/ubench/run.sh madd29 > $OUT/madd29.txt 2>&1
cat $OUT/madd29.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc -o run -- $R/gpurun_out/ubench/madd29 > /dev/null 2>&1
python3 $R/profiles/summarize_clock.py $OUT/pmc/run_counter_collection.csv 50 > $OUT/clock_madd29.txt
cat $OUT/clock_madd29.txt
cd $R
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
cat $OUT/bench_default.json
