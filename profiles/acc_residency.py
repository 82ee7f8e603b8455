#!/usr/bin/env python3
"""When the k_accumulate blocks of one MSM (2^NBITS points, alone on the GPU) start and end, and how
many share a CU (diagnostic build only: -DKGS_DIAG_CLOCK stamps s_memrealtime at thread 0's start and
end of every block and records __smid()). Answers whether the blocks of one launch are resident for
the whole launch or part of it, and whether the CUs that got more blocks finish later.
usage: KGS_LIB=kzg-grandsums-study_amd/lib_diag/libkgs.so python3 profiles/acc_residency.py [NBITS=20]
(KGS_ACC_PRIO=0 / 2: the launch without / with the progress priority of msm.hip)"""
import collections
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    K = bench.load_pkg()
    L = K.lib()
    if not hasattr(L, "kgs_diag_clock_raw"):
        sys.exit("not a -DKGS_DIAG_CLOCK build (set KGS_LIB)")
    L.kgs_diag_clock_raw.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    n = 1 << nb
    ctx = K.Context(0)
    ptau = f"/tmp/kgs_bench_p{nb}.ptau"
    if not os.path.exists(ptau):
        ctx.write_synthetic_ptau(ptau, nb, bench.bench_tau())
    ctx.load_ptau(ptau, nb)
    sc = torch.from_numpy(bench.synth_evals(n, 777)[0].reshape(-1).copy()).cuda()
    phase = (ctypes.c_double * 4)()
    entries = ctypes.c_uint64()
    for _ in range(3):
        K._check(L.kgs_bench_msm_phases(ctx.handle, ctypes.c_void_p(sc.data_ptr()), n, 1, phase,
                                        ctypes.byref(entries)))
    buf = (ctypes.c_ulonglong * (5 * 8192))()
    cnt = L.kgs_diag_clock_raw(buf, 8192)
    if cnt <= 0:
        sys.exit("no stamps")
    recs = [tuple(buf[5 * i + k] for k in range(5)) for i in range(cnt)]
    t0 = min(r[2] for r in recs)
    t1 = max(r[3] for r in recs)
    span = (t1 - t0) * 10e-3  # us (100 MHz)
    starts = [(r[2] - t0) * 10e-3 for r in recs]
    durs = [(r[3] - r[2]) * 10e-3 for r in recs]
    ghz = [(r[1] - r[0]) / ((r[3] - r[2]) * 10.0) for r in recs if r[3] > r[2]]
    per_cu = collections.Counter(r[4] for r in recs)
    by_k = collections.defaultdict(list)
    for r, d in zip(recs, durs):
        by_k[per_cu[r[4]]].append(d)
    print(f"KGS_ACC_PRIO={os.environ.get('KGS_ACC_PRIO', '1')}: accumulate phase "
          f"{phase[1]:.3f} ms (event), {cnt} blocks, stamped span {span:.1f} us, clock {statistics.median(ghz):.3f} GHz")
    print(f"  block start offsets: median {statistics.median(starts):.1f} us, max {max(starts):.1f} us")
    print(f"  block durations: min {min(durs):.1f} median {statistics.median(durs):.1f} max {max(durs):.1f} us; "
          f"residency (sum of durations / (blocks x span)) {sum(durs) / (cnt * span):.1%}")
    print(f"  distinct CU ids {len(per_cu)}; blocks per CU id: "
          + ", ".join(f"{k}: {len(v) // k} ids" for k, v in sorted(by_k.items())))
    for k, v in sorted(by_k.items()):
        print(f"  CUs holding {k} blocks: block duration median {statistics.median(v):.1f} us "
              f"(min {min(v):.1f}, max {max(v):.1f})")
    pairs = collections.defaultdict(list)
    for r in recs:
        pairs[r[4]].append(r)
    short, long_, first_short = [], [], 0
    for cu, rs in pairs.items():
        if len(rs) != 2:
            continue
        a, b = sorted(rs, key=lambda r: r[3] - r[2])
        short.append((a[3] - a[2]) * 10e-3)
        long_.append((b[3] - b[2]) * 10e-3)
        first_short += a[2] <= b[2]
    if short:
        print(f"  per CU pair: shorter block median {statistics.median(short):.1f} us, longer {statistics.median(long_):.1f} us; "
              f"the earlier-started block is the shorter one on {first_short} of {len(short)} CUs")
    xcc = collections.defaultdict(list)
    for r in recs:
        xcc[r[4] >> 16].append((r[3] - r[2]) * 10e-3)
    print("  per XCD median block duration: " + ", ".join(f"{k}: {statistics.median(v):.0f}" for k, v in sorted(xcc.items())))
    ctx.close()


if __name__ == "__main__":
    main()
