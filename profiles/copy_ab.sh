# Single-proof latency through the host-buffer boundary (Python kgs_prove and the JavaScript module),
# same box, interleaved: the previous build (lib_ab/prev: par_copy in fixed 1 MiB pieces, so each
# 2 MiB piece of F_0 was copied by 2 threads) against the in-tree build (pieces spread over the copy
# threads), and two A/B knobs of the in-tree build: non-coherent input staging, 4 MiB feed pieces
# Result (profiles/r05/boundary/copy_split_ab.txt): no difference in F_0's copy time or the latency;
# the piece change and both knobs were reverted, so only `prev` vs `new` is meaningful on later trees.
# usage: bash profiles/copy_ab.sh [reps=3]
set -e
PREV=$PWD/kzg-grandsums-study_amd/lib_ab/prev
PTAU=/tmp/kgs_bench_p20.ptau
JS=kzg-grandsums-study_amd/js/test/time_prove.js
for rep in $(seq 1 ${1:-3}); do
  for v in prev new new_nc new_feed4; do
    unset KGS_LIB KGS_STAGE_NC KGS_FEED0_MB LD_LIBRARY_PATH_KGS
    LDP=""
    case $v in
      prev) export KGS_LIB=$PREV/libkgs.so; LDP=$PREV ;;
      new_nc) export KGS_STAGE_NC=1 ;;
      new_feed4) export KGS_FEED0_MB=4 ;;
    esac
    echo "== rep $rep $v"
    timeout -k 10 120 python -u profiles/hip_runtime_ab.py torch 20 9 | grep -E "median|ms \|" | tail -4
    LD_LIBRARY_PATH=$LDP${LDP:+:}$LD_LIBRARY_PATH timeout -k 10 120 node $JS $PTAU 20 7 0 | python3 -c "
import json, sys
d = json.loads(sys.stdin.read().strip().splitlines()[-1])
b = d['best_inside_libkgs']
print('js best', d['latency_ms']['min'], 'median', d['latency_ms']['median'], '| exec', b['exec_ms'], 'copy', b['libkgs_timing_ms'][6], 'prove', b['libkgs_timing_ms'][7])"
  done
done
