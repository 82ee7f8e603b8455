#!/bin/bash
# round 6: the Montgomery write-back's D2H through hipMemcpyDtoHAsync (default) against
# hipMemcpyAsync(..., hipMemcpyDeviceToHost) (KGS_WB_API=memcpy), which the runtime ran as copyBuffer
# shader kernels into pinned memory. Parity of the host path first, then proofs in flight (device and
# host, 4 contexts) interleaved x 3, then the kernel / memory-copy trace of the default.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r06/wb_api
mkdir -p $O
R=$PWD
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_js_dropin.py -m gpu -x -q \
  --timeout 300 --timeout-method thread -k "pinned or host or golden or c1_grandsum_2p20_exact or js_proofs_match or transfer_pending" \
  > $O/parity.log 2>&1 || { echo "parity rc=$?"; tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
for rep in 1 2 3; do
  for v in dtoh memcpy; do
    if [ $v = memcpy ]; then export KGS_WB_API=memcpy; else unset KGS_WB_API; fi
    echo "== rep $rep write-back $v"
    timeout -k 10 200 python -u profiles/host_inflight.py 20 4 48 1 device,host || exit 1
  done
done 2>&1 | grep -v amdgpu.ids | tee $O/inflight_ab.txt
unset KGS_WB_API
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace_host -o run -- \
  python3 $R/profiles/host_inflight.py 20 4 48 1 host > $O/trace_host.log 2>&1 || { echo "rocprof rc=$?"; exit 1; }
grep "proofs/s" $O/trace_host.log
python3 - <<EOF
import csv
O = "$O/trace_host"
for r in csv.DictReader(open(f"{O}/run_kernel_stats.csv")):
    if "rocclr" in r["Name"]:
        print(f"  kernel {r['Name'][:40]:40s} calls {r['Calls']:>6} total {float(r['TotalDurationNs'])/1e6:9.2f} ms")
for r in csv.DictReader(open(f"{O}/run_memory_copy_stats.csv")):
    print(f"  copy {r['Name'][:40]:40s} calls {r['Calls']:>6} total {float(r['TotalDurationNs'])/1e6:9.2f} ms avg {float(r['AverageNs'])/1e3:8.1f} us")
EOF
