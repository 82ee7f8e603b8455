#!/usr/bin/env python3
"""rocprofv3 (ROCm 7 SQLite output, --kernel-trace) -> per-kernel stats CSV in the --stats layout.
usage: summarize_db.py <results.db> <out.csv> [proofs]   (proofs: also print per-proof ms)"""
import csv
import sqlite3
import sys


def main():
    db, out = sys.argv[1], sys.argv[2]
    proofs = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), sum(duration), avg(duration), min(duration), max(duration) "
                          "from kernels group by name order by sum(duration) desc"))
    tot = sum(r[2] for r in rows)
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
        for name, n, s, a, mn, mx in rows:
            w.writerow([name, n, s, a, 100.0 * s / tot, mn, mx])
    for name, n, s, a, mn, mx in rows[:25]:
        extra = f"  {s / proofs / 1e6:8.3f} ms/proof" if proofs else ""
        print(f"{name.split('(')[0][:48]:48s} {n:5d} {a / 1e3:9.1f} us {100 * s / tot:6.2f}%{extra}")
    print(f"total kernel time {tot / 1e6:.2f} ms")


if __name__ == "__main__":
    main()
