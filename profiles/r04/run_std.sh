#!/bin/bash
# Round 4: the partition pass reads the standard-form scalars the histogram pass stored (no second
# Montgomery reduction per scalar): MSM / sharded / golden / C-oracle parity, the per-proof VALU pass,
# and the headline leg x2.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/std
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -k "msm or golden or sharded or mid_size or large_proof or c5" -q -x --timeout 300 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -n 1 $OUT/parity.log)"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $R/profiles/prove_loop.py 20 1 lanes1 > /dev/null 2>&1
python3 $R/profiles/summarize_valu.py $OUT/pmc_valu > $OUT/valu_share.txt
head -1 $OUT/valu_share.txt; grep sort_ $OUT/valu_share.txt
cd $R
for k in 1 2; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-extra-legs --no-host-leg --steps 64 --msm-reps 5 > $OUT/bench_$k.json 2>> $OUT/bench.err
  echo "bench $k: $(python3 -c "import json; d=json.load(open('$OUT/bench_$k.json')); print(d['value'], d['latency_ms_single_proof'], d['msm']['phase_ms'])")"
done
