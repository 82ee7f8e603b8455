#!/bin/bash
# Round 4, late: the tree after the VALU cuts (from_mont reduction, one-lane combine, 16-lane row /
# column sums, compact Horner tile tree, coset zero-half skip): GPU parity of the NTT / MSM / proof
# tests, the per-proof VALU pass, the in-flight sweep (4 / 5 / 6 proofs per GPU) and the default bench.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/check
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_quirks.py -q -x --timeout 200 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -20 $OUT/parity.log; exit 1; }
echo "parity: $(tail -n 1 $OUT/parity.log)"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $R/profiles/prove_loop.py 20 1 lanes1 > /dev/null 2>&1
python3 $R/profiles/summarize_valu.py $OUT/pmc_valu > $OUT/valu_share.txt
head -3 $OUT/valu_share.txt
cd $R
for k in 4 5 6 4; do
  timeout -k 10 200 python3 bench.py --inflight $k --no-cpu-baseline --no-extra-legs --no-host-leg --steps 64 --msm-reps 5 > $OUT/inflight_$k.json 2>> $OUT/inflight.err
  echo "inflight $k: $(python3 -c "import json; d=json.load(open('$OUT/inflight_$k.json')); print(d['value'], d['latency_ms_single_proof'])")"
done
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 -c "import json; d=json.load(open('$OUT/bench_default.json')); print('default', d['value'], d['latency_ms_single_proof'], d['roofline']['frac'], d['host_buffer_boundary']['javascript_module'].get('ms_per_proof'), d['host_buffer_boundary']['javascript_module'].get('concurrent_proofs_per_s'))"
