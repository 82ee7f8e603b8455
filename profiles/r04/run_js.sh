#!/bin/bash
# Round 4, VERDICT r3 Next #6: where the JS single call's time goes (target <= 15 ms). One proof at a
# time, 8 samples each (every sample printed: wall, the native call's wall and its queue / completion
# waits, time inside libkgs, libkgs rounds), variants interleaved x2: default pool (8 contexts), 8
# hardware queues per process instead of 4 (8 contexts, 1 context), and the default with V8's GC trace.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/js
mkdir -p $OUT
timeout -k 10 200 python3 profiles/boundary_probe.py 20 3 > $OUT/boundary.txt 2>&1
grep -v amdgpu.ids $OUT/boundary.txt | tail -12
JS=kzg-grandsums-study_amd/js/test/time_prove.js
for rep in 1 2; do
  for v in default hwq8 gctrace hwq8ctx1; do
    case $v in
      default) E="KGS_JS_CONTEXTS=8";;
      hwq8ctx1) E="KGS_JS_CONTEXTS=1 GPU_MAX_HW_QUEUES=8";;
      hwq8) E="KGS_JS_CONTEXTS=8 GPU_MAX_HW_QUEUES=8";;
      gctrace) E="KGS_JS_CONTEXTS=8";;
    esac
    NF=""
    [ $v = gctrace ] && NF="--trace-gc"
    env $E KGS_DEVICES=0 KGS_JS_TIME_ALL=1 timeout -k 10 200 node $NF $JS /tmp/kgs_bench_p20.ptau 20 8 0 > $OUT/js_${v}_$rep.out 2>&1
    echo "$v rep $rep: $(grep '^{' $OUT/js_${v}_$rep.out | tail -n 1)"
  done
done
