#!/bin/bash
# round 6: MSM windows up to c = 20 — parity first (default c = 20 at the 2^20+ sizes; forced c = 18 /
# 20 on the small tests), then an interleaved A/B of the headline at c = 17 vs 20 (MSM leg included)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/wide
mkdir -p $O
export PYTHONUNBUFFERED=1
PT="python -u -m pytest -x -q --timeout 600 --timeout-method thread -m gpu"
timeout -k 10 400 $PT tests/test_gpu_parity.py > $O/parity_default.log 2>&1 || { echo "parity default failed"; tail -30 $O/parity_default.log; exit 1; }
tail -1 $O/parity_default.log
timeout -k 10 400 $PT tests/test_gpu_configs.py -k "c1_ or c3_ or c5_" > $O/configs_exact.log 2>&1 || { echo "configs failed"; tail -30 $O/configs_exact.log; exit 1; }
tail -1 $O/configs_exact.log
for cc in 20 18; do
  KGS_MSM_C=$cc timeout -k 10 300 $PT tests/test_gpu_parity.py -k "msm or golden or builder or mid_size" > $O/parity_c$cc.log 2>&1 || { echo "parity c=$cc failed"; tail -30 $O/parity_c$cc.log; exit 1; }
  tail -1 $O/parity_c$cc.log
done
for rep in 1 2; do
  for cc in 17 20; do
    KGS_MSM_C=$cc timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-extra-legs --no-host-leg > $O/bench_c${cc}_$rep.json 2> $O/bench_c${cc}_$rep.log || { echo "bench c=$cc failed"; tail -20 $O/bench_c${cc}_$rep.log; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_c${cc}_$rep.json'));m=d['msm'];print('c=$cc rep $rep', d['value'], 'proofs/s; msm', m['ms'], m['phase_ms'], 'latency', d['latency_ms_single_proof'])"
  done
done
