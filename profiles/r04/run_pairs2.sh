#!/bin/bash
# paired accumulation v2 (flat loops): parity, per-kernel counters, MSM phases, headline A/B x3
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/${PAIRS_OUT:-pairs2}
mkdir -p $OUT
KGS_ACC_PAIRS=1 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "(msm or golden or large_proof or mid_size or skew or twelve) and not 2p24" -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { grep -E "FAILED|Error" $OUT/parity.log | head; tail -20 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
cd /tmp && export TMPDIR=/tmp
KGS_ACC_PAIRS=1 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES --output-format csv -d $OUT/pmc -o run -- python3 $R/profiles/msm_loop.py 20 3 > $OUT/pmc.log 2>&1
cd $R
for P in 0 1; do
  for a in "20 10" "21 10" "20 10 skew"; do
    KGS_ACC_PAIRS=$P timeout -k 10 120 python3 profiles/msm_loop.py $a | sed "s|^|pairs=$P: |" >> $OUT/msm_phases.txt 2>&1
  done
done
cat $OUT/msm_phases.txt
ARGS="--no-cpu-baseline --no-extra-legs --no-host-leg --steps 64 --msm-reps 10"
for rep in 1 2 3; do
  for P in 0 1; do
    KGS_ACC_PAIRS=$P timeout -k 10 180 python3 bench.py $ARGS > $OUT/b.json 2> $OUT/b.err
    python3 -c "import json;d=json.load(open('$OUT/b.json'));print('pairs=$P rep $rep:', d['value'], 'lat', d['latency_ms_single_proof'], 'acc', d['msm']['phase_ms'])" >> $OUT/bench_ab.txt
  done
done
cat $OUT/bench_ab.txt
