#!/usr/bin/env python3
"""Where a kernel's wave time goes, from one rocprofv3 counter pass (profiles/stall_pmc.sh):
  rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
            SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES --output-format csv -d DIR -o run -- <program>
Per wave (MI355X_MICROARCH.md "rocprofv3 PMC slots"): WAIT_ANY (parked on s_waitcnt / barrier),
WAIT_INST_ANY (ready but not issued: dependency or the SIMD's issue port busy with the other wave) and
ACTIVE_INST_ANY (issuing) add up to WAVE_CYCLES; all three count quad-cycles. Printed as shares of
WAVE_CYCLES, plus VALU instructions per wave and the SIMD cycles each one took on average across the
waves sharing a SIMD.
usage: summarize_stall.py DIR/run_counter_collection.csv [min_us=100]"""
import collections
import csv
import sys


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
        if "SQ_WAVE_CYCLES" not in d or d["ns"] < 1000 * min_us or not d["SQ_WAVE_CYCLES"]:
            continue
        w = d["SQ_WAVE_CYCLES"]
        per[d["name"]].append((d["ns"] / 1e3, d["SQ_WAIT_ANY"] / w, d["SQ_WAIT_INST_ANY"] / w,
                               d["SQ_ACTIVE_INST_ANY"] / w, d["SQ_ACTIVE_INST_VALU"] / w,
                               d["SQ_INSTS_VALU"] / max(1.0, d["SQ_WAVES"]), 4 * w / max(1.0, d["SQ_INSTS_VALU"])))
    print(f"dispatches >= {min_us:.0f} us; shares of SQ_WAVE_CYCLES; wave-cyc/VALU = 4 * WAVE_CYCLES / INSTS_VALU "
          f"(wave lifetime per VALU instruction, all waves summed)")
    print(f"{'kernel':40s} {'n':>3s} {'us':>9s} {'wait_any':>9s} {'wait_inst':>9s} {'active':>7s} {'act_valu':>9s} "
          f"{'VALU/wave':>10s} {'wave-cyc/VALU':>13s}")
    for name, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        n = len(v)
        m = [sum(x[i] for x in v) / n for i in range(7)]
        print(f"{name[:40]:40s} {n:3d} {m[0]:9.1f} {m[1]:9.1%} {m[2]:9.1%} {m[3]:7.1%} {m[4]:9.1%} {m[5]:10.0f} "
              f"{m[6]:13.2f}")


if __name__ == "__main__":
    main()
