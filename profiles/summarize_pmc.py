#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (run separately, per the MI355X guide)
into profiles/pmc_<round>.json and profiles/pmc_accumulate.json (read by bench.py's roofline).

Counters are in KB per dispatch. Both the raw FETCH_SIZE and the gfx950-corrected (x2) figure are
recorded; since round 6 bench.py reports the corrected one as `roofline.traffic` (the MI355X
guide's HBM recipe) with the raw one beside it.
usage: summarize_pmc.py <pmc_FETCH_SIZE dir> <pmc_WRITE_SIZE dir> <round tag>
(both passes over `python3 profiles/msm_loop.py 20 3`)
"""
import collections
import csv
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def load(d):
    out = collections.defaultdict(list)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        out[(name, int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return out


def main():
    fdir, wdir, tag = sys.argv[1:4]
    f, w = load(fdir), load(wdir)
    kernels = []
    for key in sorted(f):
        fa = sum(f[key]) / len(f[key]) * 1024
        wa = sum(w.get(key, [0])) / max(1, len(w.get(key, [1]))) * 1024
        kernels.append({"kernel": key[0], "grid_threads": key[1], "dispatches": len(f[key]),
                        "fetch_bytes_raw": round(fa), "fetch_bytes_x2": round(2 * fa), "write_bytes": round(wa)})
    with open(os.path.join(HERE, f"pmc_{tag}.json"), "w") as fh:
        json.dump({"round": tag, "kernels": kernels}, fh, indent=1)
    # run on profiles/msm_loop.py (every MSM is a 2^20-point one): the k_accumulate dispatches
    acc = [k for k in kernels if k["kernel"].split("<")[0].endswith("k_accumulate")]
    if acc:
        a = acc[0]
        with open(os.path.join(HERE, "pmc_accumulate.json"), "w") as fh:
            json.dump({"round": tag, "kernel": "k_accumulate", "msm_points": 1 << 20,
                       "hbm_bytes_per_launch": a["fetch_bytes_raw"] + a["write_bytes"],
                       "fetch_bytes_raw": a["fetch_bytes_raw"], "fetch_bytes_x2_corrected": a["fetch_bytes_x2"],
                       "write_bytes": a["write_bytes"], "source": f"profiles/pmc_{tag}.json"}, fh, indent=1)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
