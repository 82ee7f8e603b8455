#!/usr/bin/env python3
"""Summarise the memory copies of a rocprofv3 --kernel-trace --memory-copy-trace database (ROCm 7
SQLite output): per direction and size, the count, mean duration and rate, and how much of the copies'
time overlaps some kernel (copies beside compute vs copies the GPU waits on).
usage: summarize_copies.py <dir with the .db>"""
import collections
import glob
import os
import sqlite3
import sys


def main():
    db = sqlite3.connect(glob.glob(os.path.join(sys.argv[1], "**", "*.db"), recursive=True)[0])
    agents = {r[0]: r[1] for r in db.execute("select id, type from rocpd_info_agent")}
    copies = list(db.execute("select start, end, size, src_agent_id, dst_agent_id from rocpd_memory_copy"))
    kern = sorted(db.execute("select start, end from kernels"))
    # merged kernel-busy intervals
    busy = []
    for s, e in kern:
        if busy and s <= busy[-1][1]:
            busy[-1][1] = max(busy[-1][1], e)
        else:
            busy.append([s, e])

    def overlap(s, e):
        tot = 0
        for bs, be in busy:
            if be <= s:
                continue
            if bs >= e:
                break
            tot += min(e, be) - max(s, bs)
        return tot

    groups = collections.defaultdict(list)
    for s, e, size, src, dst in copies:
        d = f"{agents.get(src, '?')}->{agents.get(dst, '?')}"
        groups[(d, size)].append((s, e))
    print(f"{'direction':12s} {'bytes':>10s} {'count':>6s} {'mean us':>9s} {'GB/s':>7s} {'beside kernels':>15s}")
    for (d, size), iv in sorted(groups.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
        dur = [e - s for s, e in iv]
        mean = sum(dur) / len(dur)
        ov = sum(overlap(s, e) for s, e in iv) / max(1, sum(dur))
        print(f"{d:12s} {size:10d} {len(iv):6d} {mean / 1e3:9.1f} {size / mean if mean else 0:7.1f} {ov:15.0%}")


if __name__ == "__main__":
    main()
