#!/usr/bin/env python3
"""rocprofv3 --kernel-trace CSV -> per-(kernel, grid) duration summary, so a kernel that runs at
several sizes (k_accumulate at 2^20 and 2^21 points in one proof) can be compared with bench.py's
live HIP-event timing of one size.
usage: summarize_trace.py run_kernel_trace.csv out.csv [KERNEL LAST_N]
With KERNEL and LAST_N, also print the average of the last LAST_N dispatches of KERNEL (bench.py's
MSM leg, the dispatches its roofline times, runs last on the GPU)."""
import collections
import csv
import sys


def main():
    src, out = sys.argv[1], sys.argv[2]
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(src)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        grid = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        d[(name, grid)].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    rows = sorted(d.items(), key=lambda kv: -sum(kv[1]))
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel", "GridThreads", "Calls", "AverageNs", "MinNs", "MaxNs", "TotalNs"])
        for (name, grid), v in rows:
            w.writerow([name, grid, len(v), round(sum(v) / len(v)), min(v), max(v), sum(v)])
    for (name, grid), v in rows[:12]:
        print(f"{name[:40]:40s} grid {grid:9d} calls {len(v):4d} avg {sum(v) / len(v) / 1e3:9.1f} us")
    if len(sys.argv) > 4:
        kern, last = sys.argv[3], int(sys.argv[4])
        seq = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
               for r in csv.DictReader(open(src)) if kern in r["Kernel_Name"]]
        seq.sort()
        tail = [d for _, d in seq[-last:]]
        print(f"last {len(tail)} dispatches of {kern}: avg {sum(tail) / len(tail) / 1e6:.4f} ms "
              f"(min {min(tail) / 1e6:.4f}, max {max(tail) / 1e6:.4f})")


if __name__ == "__main__":
    main()
