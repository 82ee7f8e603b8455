#!/usr/bin/env python3
"""Cut a rocprofv3 kernel trace to the bench's timed region and summarise it.

usage: summarize_window.py PREFIX STEPS [MARKER]
  PREFIX : rocprofv3 output prefix (PREFIX_kernel_trace.csv and PREFIX_marker_api_trace.csv)
  STEPS  : proofs in the timed region (bench.py --steps)
  MARKER : roctx range name (default kgs_bench_timed_region, pushed by bench.py)

Prints the window length, the per-proof kernel time of every kernel that STARTED inside the window
(several proofs are in flight, so kernel durations overlap and include waiting for CU slots), the
fraction of the window during which at least one kernel runs, and the fraction during which some
k_accumulate (the roofline kernel) runs."""
import collections
import csv
import sys


def union_len(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    prefix, steps = sys.argv[1], int(sys.argv[2])
    marker = sys.argv[3] if len(sys.argv) > 3 else "kgs_bench_timed_region"
    win = None
    for r in csv.DictReader(open(prefix + "_marker_api_trace.csv")):
        if any(marker in str(v) for v in r.values()):
            win = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
    if win is None:
        sys.exit(f"marker {marker} not found")
    w0, w1 = win
    per = collections.defaultdict(int)
    calls = collections.Counter()
    iv, iv_acc = [], []
    for r in csv.DictReader(open(prefix + "_kernel_trace.csv")):
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if not (w0 <= s < w1):
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kgs::", "")
        per[name] += e - s
        calls[name] += 1
        iv.append((s, min(e, w1)))
        if name.startswith("k_accumulate"):
            iv_acc.append((s, min(e, w1)))
    span = w1 - w0
    print(f"timed region: {span / 1e6:.3f} ms for {steps} proofs = {span / 1e6 / steps:.3f} ms per proof")
    print(f"some kernel running: {union_len(iv) / span:.3f} of the window; some k_accumulate running: "
          f"{union_len(iv_acc) / span:.3f}")
    tot = sum(per.values())
    print(f"{'kernel':40s} {'calls/proof':>11s} {'us/proof':>10s} {'share':>6s}   (durations overlap in flight)")
    for name, t in sorted(per.items(), key=lambda kv: -kv[1]):
        print(f"{name[:40]:40s} {calls[name] / steps:11.1f} {t / 1e3 / steps:10.1f} {t / tot:6.1%}")


if __name__ == "__main__":
    main()
