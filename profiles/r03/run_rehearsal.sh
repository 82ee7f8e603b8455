#!/bin/bash
# (1) bench.py --gpus 2 started WITHOUT a launcher, gloo rehearsal on the one-GPU box: the script
#     launches its two ranks itself (torch.distributed.run), the configs[3]/[4] legs run the
#     distributed prover with per-rank SRS slices; (2) the JS single-proof latency with diagnostics
set -e
cd "$(dirname "$0")/../.."
OUT=gpurun_out/r03d
mkdir -p $OUT
KGS_BENCH_BACKEND=gloo timeout -k 10 500 python3 bench.py --gpus 2 --steps 8 --warmup 2 --no-cpu-baseline --no-host-leg --c4-nbits 20 --sv-nbits 18 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err
echo "rc=$?"
cat $OUT/bench_n2_gloo.json
P=/tmp/kgs_bench_p20.ptau
[ -f $P ] || timeout -k 10 300 python3 -c "import bench; K=bench.load_pkg(); c=K.Context(0); c.write_synthetic_ptau('$P', 20, bench.bench_tau())"
KGS_JS_CONTEXTS=8 KGS_DEVICES=0 timeout -k 10 300 node kzg-grandsums-study_amd/js/test/time_prove.js $P 20 5 16 > $OUT/js.json
cat $OUT/js.json
