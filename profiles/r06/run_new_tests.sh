#!/bin/bash
# round 6, first GPU call: the new / changed tests, the host-copy ubench, one default bench line
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06
mkdir -p $O
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -v --timeout 900 --timeout-method thread -m gpu \
  "tests/test_gpu_parity.py::test_failed_call_leaves_no_transfer_pending" \
  "tests/test_gpu_quirks.py::test_replay_failure_on_one_rank_aborts_the_group" \
  "tests/test_gpu_dist.py::test_host_group_two_processes" \
  "tests/test_gpu_parity.py::test_caller_pinned_inputs" \
  "tests/test_gpu_configs.py::test_c1_grandsum_2p20_exact" \
  "tests/test_gpu_configs.py::test_c3_grandproduct_2p20" \
  "tests/test_gpu_configs.py::test_c5_selected_vector_2p22_k4" \
  --durations=0 > $O/new_tests.log 2>&1 || { echo "new tests rc=$?"; tail -30 $O/new_tests.log; exit 1; }
tail -15 $O/new_tests.log
timeout -k 10 120 ./profiles/ubench/host_copy_bw > $O/host_copy_bw.txt 2>&1 || { echo "ubench failed"; exit 1; }
cat $O/host_copy_bw.txt
lscpu > $O/lscpu.txt 2>&1; cat /sys/fs/cgroup/cpu.max >> $O/lscpu.txt 2>/dev/null
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.log || { echo "bench rc=$?"; tail -20 $O/bench_default.log; exit 1; }
cat $O/bench_default.json
