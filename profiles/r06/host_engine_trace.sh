#!/bin/bash
# round 6: which engine moves the host-buffer path's bytes in flight (SDMA copies vs blit kernels on the
# CUs), and what else the host path adds to the GPU beside the device-resident proofs: kernel and
# memory-copy trace of 4 contexts in flight, device-resident then host, 48 steps each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=$PWD/gpurun_out/r06/host_engine
mkdir -p $O
R=$PWD
cd /tmp && export TMPDIR=/tmp
for m in device host; do
  timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/$m -o run -- \
    python3 $R/profiles/host_inflight.py 20 4 48 1 $m > $O/$m.log 2>&1 || { echo "rocprof $m rc=$?"; tail -5 $O/$m.log; exit 1; }
  grep "proofs/s" $O/$m.log
done
python3 - <<EOF
import csv, collections
O = "$O"
for m in ("device", "host"):
    print("==", m)
    ks = list(csv.DictReader(open(f"{O}/{m}/run_kernel_stats.csv")))
    tot = sum(float(r["TotalDurationNs"]) for r in ks)
    for r in ks:
        if "copy" in r["Name"].lower() or "fill" in r["Name"].lower() or "rocclr" in r["Name"].lower():
            print(f"  kernel {r['Name'][:60]:60s} calls {r['Calls']:>6} total {float(r['TotalDurationNs'])/1e6:9.2f} ms")
    print(f"  all kernels total {tot/1e6:.1f} ms")
    try:
        for r in csv.DictReader(open(f"{O}/{m}/run_memory_copy_stats.csv")):
            print(f"  copy {r['Name'][:40]:40s} calls {r['Calls']:>6} total {float(r['TotalDurationNs'])/1e6:9.2f} ms avg {float(r['AverageNs'])/1e3:8.1f} us")
    except FileNotFoundError:
        print("  no memory copy stats")
EOF
