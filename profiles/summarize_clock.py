#!/usr/bin/env python3
"""Held clock and VALU issue rate per kernel from one rocprofv3 counter pass.

Input: the counter_collection CSV of
  rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES \
            --output-format csv -d DIR -o run -- python3 profiles/msm_loop.py 20 5   (or prove_loop.py 20 1 lanes1)
Per dispatch (counter collection serialises dispatches, so each one has the chip to itself):
  cycles      = GRBM_GUI_ACTIVE / 8           (rocprofv3 sums the counter over the 8 XCDs; MI355X_MICROARCH.md
                                               "DVFS give-back")
  clock       = cycles / (End - Start)        (the clock the chip held during the dispatch)
  cpi         = cycles / (SQ_INSTS_VALU / 1024)  SIMD cycles per wave64 VALU instruction actually achieved
                                               (256 CUs x 4 SIMDs; lower is denser issue)
  issue_frac  = 4.93 / cpi                    against the measured v_mad_u64_u32 issue cost (ubench_r02.txt:
                                               4.93 SIMD cycles per wave64 instruction; most 32/64-bit VALU ops
                                               cost 4.2-4.4, v_add_u32 2.46, so a mixed stream can exceed 1)
usage: summarize_clock.py DIR/run_counter_collection.csv [min_us=100]"""
import collections
import csv
import sys

SIMDS = 256 * 4
MAD_CPI = 4.93


def main():
    path = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 100.0
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(path)):
        d = disp[r["Dispatch_Id"]]
        d["name"] = r["Kernel_Name"].split("(")[0].replace("kgs::", "")
        d["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        d[r["Counter_Name"]] = float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for d in disp.values():
        if "GRBM_GUI_ACTIVE" not in d or "SQ_INSTS_VALU" not in d or d["ns"] < 1000 * min_us:
            continue
        cyc = d["GRBM_GUI_ACTIVE"] / 8.0
        clk = cyc / d["ns"]  # GHz
        valu = d["SQ_INSTS_VALU"]
        cpi = cyc / (valu / SIMDS) if valu else float("inf")
        per[d["name"]].append((d["ns"] / 1e3, clk, valu / 1e6, cpi, d.get("SQ_WAVES", 0)))
    print(f"dispatches >= {min_us:.0f} us; clock = GRBM_GUI_ACTIVE/8/duration; cpi = SIMD cycles per wave64 VALU "
          f"instruction; issue_frac = {MAD_CPI}/cpi")
    print(f"{'kernel':40s} {'n':>3s} {'us':>9s} {'GHz':>6s} {'VALU M':>9s} {'cpi':>6s} {'issue_frac':>10s}")
    for name, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        n = len(v)
        us = sum(x[0] for x in v) / n
        clk = sum(x[1] for x in v) / n
        valu = sum(x[2] for x in v) / n
        cpi = sum(x[3] for x in v) / n
        print(f"{name[:40]:40s} {n:3d} {us:9.1f} {clk:6.3f} {valu:9.2f} {cpi:6.2f} {MAD_CPI / cpi:10.3f}")


if __name__ == "__main__":
    main()
