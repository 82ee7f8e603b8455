#!/usr/bin/env python3
"""Per-kernel VALU instruction share of one proof, from a rocprofv3 --pmc SQ_INSTS_VALU pass over
profiles/prove_loop.py (three proofs; one-time SRS / ptau kernels excluded). Reads the CSV output
(--output-format csv) or the default ROCm 7 SQLite database.
usage: summarize_valu.py <pmc dir> [PROOFS=3]
SQ_INSTS_VALU counts wave-level VALU instructions (a v_mad_u64_u32 costs ~2x a 32-bit add in issue
cycles, so this is an instruction share, not a cycle share)."""
import collections
import csv
import glob
import os
import sys

# one-time per context / domain (SRS tables, domain tables, the cached 1/(n(x-1)) of get_nxm1)
ONE_TIME = ("k_tab_dbl", "k_batch_affine", "k_tab_to29", "k_fixed_base", "k_powers", "k_nxm1", "k_fr_batch_inv",
            "k_tw29")


def main():
    d = sys.argv[1]
    proofs = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    rows = []
    csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if csvs:
        rows = [(r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r.get("Dispatch_Id"))
                for r in csv.DictReader(open(csvs[0]))]
    else:
        import sqlite3
        db = sqlite3.connect(glob.glob(os.path.join(d, "**", "*.db"), recursive=True)[0])
        # per-SE values: sum them per dispatch
        rows = list(db.execute("select kernel_name, counter_name, sum(value), dispatch_id from counters_collection "
                               "group by dispatch_id, counter_name"))
    tot = collections.defaultdict(float)
    calls = collections.Counter()
    for kname, cname, value, _ in rows:
        if cname != "SQ_INSTS_VALU":
            continue
        name = kname.split("(")[0].replace("void ", "").replace("kgs::", "")
        if name.startswith(ONE_TIME) or name.startswith("__amd"):
            continue
        tot[name] += float(value)
        calls[name] += 1
    s = sum(tot.values())
    print(f"VALU instructions per proof (wave-level): {s / proofs / 1e6:.1f} M")
    for name, v in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"{name[:40]:40s} calls/proof {calls[name] / proofs:5.1f}  {v / proofs / 1e6:8.2f} M  {v / s:6.1%}")


if __name__ == "__main__":
    main()
