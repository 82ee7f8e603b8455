#!/bin/bash
# Round 4, VERDICT r3 Next #6: where the JS single call's time goes (target <= 15 ms). One proof at a
# time, 8 samples each (every sample printed: wall, time inside libkgs, libkgs rounds), variants
# interleaved x2: default pool (8 contexts), output buffers registered for DMA in place
# (KGS_JS_OUT_REGISTER=1), two spare pre-registered output buffers per size kept ready by a background
# thread (KGS_JS_OUT_POOL=2), a one-context pool; then the Python host-buffer probe beside it.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js
mkdir -p $OUT
timeout -k 10 200 python3 profiles/boundary_probe.py 20 3 > $OUT/boundary.txt 2>&1
grep -v amdgpu.ids $OUT/boundary.txt | tail -8
JS=kzg-grandsums-study_amd/js/test/time_prove.js
for rep in 1 2; do
  for v in default reg pool ctx1; do
    case $v in
      default) E="KGS_JS_CONTEXTS=8";;
      reg) E="KGS_JS_CONTEXTS=8 KGS_JS_OUT_REGISTER=1";;
      pool) E="KGS_JS_CONTEXTS=8 KGS_JS_OUT_POOL=2";;
      ctx1) E="KGS_JS_CONTEXTS=1";;
    esac
    env $E KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 200 node $JS /tmp/kgs_bench_p20.ptau 20 8 0 > $OUT/js_${v}_$rep.json
    echo "$v rep $rep: $(cat $OUT/js_${v}_$rep.json)"
  done
done
# the 16-way concurrent rate with the pool (the bench's JS leg shape)
for v in default pool; do
  case $v in
    default) E="KGS_JS_CONTEXTS=8";;
    pool) E="KGS_JS_CONTEXTS=8 KGS_JS_OUT_POOL=2";;
  esac
  env $E KGS_DEVICES=0 timeout -k 10 300 node $JS /tmp/kgs_bench_p20.ptau 20 3 16 > $OUT/js_conc_$v.json
  echo "$v conc: $(cat $OUT/js_conc_$v.json)"
done
