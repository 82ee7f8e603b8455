#!/usr/bin/env python3
"""rocprofv3 kernel trace of profiles/dist_scaling.py -> per-rank kernel time of the distributed
prover. Each rank is one persistent host thread whose OS thread id the script prints
("RANKTID W=.. r=.. tid=.."); the trace's Thread_Id attributes every dispatch to its rank. Each rank
runs 1 warm-up + 3 timed proofs. With all W ranks on ONE GPU their kernels overlap, so per-kernel
durations stretch; what measures the work is the GPU busy time of the W-rank proof (the union of all
its kernel intervals): flat in W means nothing is replicated and each rank's share is 1/W of it
(what a rank does on its own GPU of a node, plus its exchanges). Also printed: the MSM share of the
summed kernel time.
usage: summarize_dist.py run_kernel_trace.csv script_stdout.txt [proofs=4]"""
import collections
import csv
import re
import sys

MSM = ("k_accumulate", "k_sort", "k_lo_", "k_combine", "k_rowcol", "k_bitsum")


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    proofs = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    ranks = collections.defaultdict(dict)  # W -> {tid: r}
    for m in re.finditer(r"RANKTID W=(\d+) r=(\d+) tid=(\d+)", open(sys.argv[2]).read()):
        ranks[int(m.group(1))][m.group(3)] = int(m.group(2))
    tid_key = "Thread_Id" if "Thread_Id" in rows[0] else [k for k in rows[0] if "hread" in k][0]
    for W in sorted(ranks):
        iv = []
        msm = oth = 0
        for r in rows:
            if r[tid_key] in ranks[W]:
                a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
                iv.append((a, b))
                if any(k in r["Kernel_Name"] for k in MSM):
                    msm += b - a
                else:
                    oth += b - a
        iv.sort()
        busy, cur_a, cur_b = 0, None, None
        for a, b in iv:
            if cur_b is None or a > cur_b:
                if cur_b is not None:
                    busy += cur_b - cur_a
                cur_a, cur_b = a, b
            else:
                cur_b = max(cur_b, b)
        if cur_b is not None:
            busy += cur_b - cur_a
        bp = busy / proofs / 1e6
        print(f"W={W:2d}: GPU busy ms per proof (all {W} ranks on one GPU) {bp:7.2f} -> per-rank share {bp / W:7.2f} ms"
              f" | MSM kernels {100.0 * msm / max(1, msm + oth):5.1f} % of kernel time")

if __name__ == "__main__":
    main()
