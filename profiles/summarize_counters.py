#!/usr/bin/env python3
"""Per-kernel averages of every counter in one or more rocprofv3 counter-collection CSVs (one pass
each; the passes of one program are joined by kernel name), with the derived stall ratios:
  cycles       = GRBM_GUI_ACTIVE / 8 (rocprofv3 sums the 8 XCDs), clock = cycles / duration
  cpi          = cycles / (SQ_INSTS_VALU / 1024)   real SIMD cycles per wave64 VALU instruction
  wait_any     = SQ_WAIT_ANY / SQ_WAVE_CYCLES      share of wave time parked (s_waitcnt / barrier)
  wait_inst    = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES share of wave time stalled at issue
  wait_lds     = SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES LDS issue stalls
  active       = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  bank_conf    = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
usage: summarize_counters.py KERNEL_SUBSTRING CSV [CSV ...]"""
import collections
import csv
import sys


def main():
    sub = sys.argv[1]
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[2:]:
        disp = collections.defaultdict(dict)
        for r in csv.DictReader(open(path)):
            name = r["Kernel_Name"].split("(")[0].replace("kgs::", "").replace("void ", "")
            if sub not in name:
                continue
            d = disp[r["Dispatch_Id"]]
            d["name"] = name
            d["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            d[r["Counter_Name"]] = float(r["Counter_Value"])
        for d in disp.values():
            for k, v in d.items():
                if k != "name":
                    per[d["name"]][k].append(v)
    for name, cs in sorted(per.items()):
        avg = {k: sum(v) / len(v) for k, v in cs.items()}
        print(f"== {name}  (dispatches per pass: {len(cs['us']) // max(1, len(sys.argv) - 2)})")
        for k in sorted(avg):
            print(f"   {k:28s} {avg[k]:16.1f}")
        a = avg.get
        if a("GRBM_GUI_ACTIVE") and a("SQ_INSTS_VALU"):
            cyc = a("GRBM_GUI_ACTIVE") / 8
            print(f"   clock_GHz                    {cyc / (a('us') * 1e3):16.3f}")
            print(f"   cpi_real                     {cyc / (a('SQ_INSTS_VALU') / 1024):16.2f}")
        for num, den, label in (("SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "wait_any"),
                                ("SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "wait_inst"),
                                ("SQ_WAIT_INST_LDS", "SQ_WAVE_CYCLES", "wait_lds"),
                                ("SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", "active"),
                                ("SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "bank_conf")):
            if a(num) is not None and a(den):
                print(f"   {label:28s} {a(num) / a(den):16.3f}")


if __name__ == "__main__":
    main()
