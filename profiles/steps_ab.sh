# The headline's timed-region length: the default 32 steps (~0.35 s) against 256 steps (~2.7 s) and
# 32 steps after 64 warm-up steps, same box, interleaved (headline leg only)
# usage: bash profiles/steps_ab.sh [reps=2]
set -e
for rep in $(seq 1 ${1:-2}); do
  for v in "32 4" "256 4" "32 64"; do
    set -- $v
    echo "== rep $rep steps $1 warmup $2"
    timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --no-extra-legs --no-cpu-baseline --no-host-leg --msm-reps 1 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])"
  done
done
