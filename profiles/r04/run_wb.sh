#!/bin/bash
# Round 4: full GPU suite on the tree (write-back stream, peer-access attach, quirks mode), then the
# host-boundary latency A/B: Montgomery write-back on the copy stream after the round-1 MSMs (wb_base)
# vs its own stream right after each conversion (this tree), interleaved.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/wb
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
for rep in 1 2; do
  for L in kzg-grandsums-study_amd/lib_ab/wb_base/libkgs.so kzg-grandsums-study_amd/lib/libkgs.so; do
    echo "== $L rep $rep" >> $OUT/boundary_ab.txt
    KGS_LIB=$R/$L timeout -k 10 120 python3 profiles/boundary_probe.py 20 4 >> $OUT/boundary_ab.txt 2>&1
  done
done
grep -E "==|host  " $OUT/boundary_ab.txt | head -40
timeout -k 10 300 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
python3 -c "import json;d=json.load(open('$OUT/bench_default.json'));print(d['value'], d['latency_ms_single_proof'], d['host_buffer_boundary']['ms_per_proof'], d['host_buffer_boundary']['javascript_module']['ms_per_proof'], d['host_buffer_boundary']['javascript_module']['concurrent_proofs_per_s'])"
