#!/bin/bash
# round 6: per-pass kernel times of the NTT pair (rocprofv3 kernel trace) for the in-tree 2^11 tiles
# and the 2^12-tile variant, at 2^20 / 2^21 / 2^22
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06/ntt_e12_trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
E12=$PWD/kzg-grandsums-study_amd/lib_ab/e12/libkgs.so
for v in e11 e12; do
  if [ $v = e11 ]; then unset KGS_LIB; else export KGS_LIB=$E12; fi
  for lg in 20 21 22; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$v-$lg -o run -- python3 -u profiles/ntt_ab.py $lg 20 \
      > $O/$v-$lg.log 2>&1 || { echo "rocprof $v $lg rc=$?"; tail -5 $O/$v-$lg.log; exit 1; }
    grep "pair" $O/$v-$lg.log
  done
done
python3 - <<'EOF'
import csv, glob, os, collections
O = "gpurun_out/r06/ntt_e12_trace"
for d in sorted(glob.glob(f"{O}/e1*-*")):
    if not os.path.isdir(d):
        continue
    f = glob.glob(f"{d}/**/*kernel_stats.csv", recursive=True)
    if not f:
        continue
    print("==", os.path.basename(d))
    for r in csv.DictReader(open(f[0])):
        if "ntt" in r["Name"]:
            print(f"  {int(r['Calls']):6d} calls  avg {float(r['AverageNs'])/1e3:8.2f} us  {r['Name'][:110]}")
EOF
