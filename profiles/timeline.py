#!/usr/bin/env python3
"""Timeline of the last proof in a rocprofv3 kernel trace (prove_loop.py under --kernel-trace): every
kernel of the proof with its start offset from the proof's first kernel, duration and queue, so the
single-proof critical path (serial kernels, gaps) can be read off.
usage: timeline.py run_kernel_trace.csv [FIRST_KERNEL_SUBSTRING=k_to_mont]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    first = sys.argv[2] if len(sys.argv) > 2 else "k_to_mont"
    starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
    # the proof's first kernel: the first of the last run of consecutive `first` kernels
    i0 = starts[-1]
    while i0 - 1 in starts:
        i0 -= 1
    t0 = int(rows[i0]["Start_Timestamp"])
    end = max(int(r["End_Timestamp"]) for r in rows[i0:])
    busy = {}
    for r in rows[i0:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        q = r.get("Queue_Id", r.get("Stream_Id", "?"))
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kgs::", "")
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  q{q:>3}  {name}")
        busy.setdefault(name, 0)
        busy[name] += e - s
    print(f"# proof span {(end - t0) / 1e3:.1f} us; kernel time by name (sum over queues):")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:25]:
        print(f"#   {v / 1e3:9.1f} us  {k}")


if __name__ == "__main__":
    main()
