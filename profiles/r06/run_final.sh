#!/bin/bash
# Round-6 tree measurement: full GPU suite, smoke, default bench under rocprofv3 (kernel + marker
# trace, windows cut to the timed region and the MSM leg), FETCH/WRITE counter passes and the clock /
# VALU pass of the MSM at 2^20 points, then a plain default bench. Each GPU step under its own limit.
set -e
cd "$(dirname "$0")/../.."
R=$PWD
OUT=$R/gpurun_out/r06/${FINAL_DIR:-final}
mkdir -p $OUT
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1100 python3 -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { grep -E "FAILED|Error" $OUT/gpu_tests.log | head -30; tail -5 $OUT/gpu_tests.log; exit 1; }
  tail -1 $OUT/gpu_tests.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $OUT/bench_prof -o run -- python3 $R/bench.py > $OUT/bench_under_rocprof.json 2> $OUT/bench_under_rocprof.err
cat $OUT/bench_under_rocprof.json
python3 $R/profiles/summarize_window.py $OUT/bench_prof/run 5 kgs_bench_msm_leg > $OUT/bench_windows.txt
python3 $R/profiles/summarize_window.py $OUT/bench_prof/run 32 >> $OUT/bench_windows.txt
python3 $R/profiles/summarize_trace.py $OUT/bench_prof/run_kernel_trace.csv $OUT/bench_kernel_by_grid.csv > $OUT/bench_trace_summary.txt
head -8 $OUT/bench_windows.txt
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 $R/profiles/msm_loop.py 20 3 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 $R/profiles/msm_loop.py 20 3 > /dev/null 2>&1
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES --output-format csv -d $OUT/pmc_clock -o run -- python3 $R/profiles/msm_loop.py 20 5 > /dev/null 2>&1
python3 $R/profiles/summarize_clock.py $OUT/pmc_clock/run_counter_collection.csv > $OUT/clock_valu.txt
cat $OUT/clock_valu.txt
cd $R
timeout -k 10 600 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
cat $OUT/bench_default.json
# per-kernel VALU share of one proof (VERDICT r4 Next #3)
cd /tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $OUT/pmc_valu -o run -- python3 $R/profiles/prove_loop.py 20 1 lanes1 > /dev/null 2>&1
python3 $R/profiles/summarize_valu.py $OUT/pmc_valu > $OUT/valu_share_per_proof_2p20.txt
head -12 $OUT/valu_share_per_proof_2p20.txt
cd $R
# the N = 2 path rehearsed on the one-GPU box (gloo host collectives; VERDICT r4 Next #4/#7)
KGS_BENCH_BACKEND=gloo timeout -k 10 600 python3 bench.py --gpus 2 --steps 16 --no-cpu-baseline --c4-proofs 1 --sv-proofs 1 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err
cat $OUT/bench_n2_gloo.json
