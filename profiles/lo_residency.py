#!/usr/bin/env python3
"""How long k_lo_scatter's workgroups sit resident, alone and with four proofs in flight (diagnostic
build only; VERDICT r3 Next #4: the kernel's in-flight duration is ~28x its duration alone).

The -DKGS_DIAG_CLOCK library appends one record per k_lo_scatter block to a ring (msm.hip): the
MSM's offsets pointer (which context launched it), the 100 MHz real-time counter at block start and
end, the CU id. Per launch this gives the span (first block start -> last block end, what a kernel
trace reports as the duration), how long each block is resident, how far apart the blocks start, and
the fraction of the span during which at least one block of the launch is resident. A launch whose
blocks run briefly but start far apart is waiting for CUs, not working.
usage: KGS_LIB=kzg-grandsums-study_amd/lib_diag/libkgs.so python3 profiles/lo_residency.py"""
import collections
import ctypes
import os
import statistics
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

CAP = 1 << 16


def launches(recs):
    """split the records into launches: per context, blocks sorted by start, a new launch after a
    gap of more than 200 us between consecutive block starts"""
    by = collections.defaultdict(list)
    for ptr, t0, t1, ident in recs:
        by[ptr].append((t0, t1, ident & 0xffffffff))
    out = []
    for ptr, v in by.items():
        v.sort()
        cur = [v[0]]
        for r in v[1:]:
            if r[0] - cur[-1][0] > 20000:
                out.append(cur)
                cur = []
            cur.append(r)
        out.append(cur)
    return out


def describe(ls, label):
    rows = []
    for bl in ls:
        if len(bl) < 16:
            continue
        t0 = min(b[0] for b in bl)
        t1 = max(b[1] for b in bl)
        span = (t1 - t0) / 100.0  # us
        res = [(b[1] - b[0]) / 100.0 for b in bl]
        starts = sorted((b[0] - t0) / 100.0 for b in bl)
        # union of the resident intervals
        iv = sorted((b[0], b[1]) for b in bl)
        busy, cs, ce = 0, iv[0][0], iv[0][1]
        for a, b in iv[1:]:
            if a > ce:
                busy += ce - cs
                cs, ce = a, b
            else:
                ce = max(ce, b)
        busy += ce - cs
        rows.append((span, statistics.median(res), sum(res) / len(res), starts[len(starts) // 2], starts[-1],
                     busy / 100.0 / span if span else 1.0, len(bl), len({b[2] for b in bl})))
    if not rows:
        print(f"{label}: no launches recorded", flush=True)
        return
    med = lambda i: statistics.median(r[i] for r in rows)  # noqa: E731
    print(f"{label}: {len(rows)} launches; per launch (medians): span {med(0):.1f} us, block resident "
          f"{med(1):.1f} us (mean {med(2):.1f}), block starts median +{med(3):.1f} us / last +{med(4):.1f} us "
          f"after the first, >= 1 block resident {100 * med(5):.0f} % of the span, {med(6):.0f} blocks on "
          f"{med(7):.0f} CUs", flush=True)


def main():
    K = bench.load_pkg()
    L = K.lib()
    if not hasattr(L, "kgs_diag_lorec"):
        sys.exit("not a -DKGS_DIAG_CLOCK build (set KGS_LIB)")
    L.kgs_diag_lorec.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.POINTER(ctypes.c_uint), ctypes.c_int]
    buf = (ctypes.c_ulonglong * (4 * CAP))()

    def fetch(reset=True):
        n = ctypes.c_uint()
        K._check(L.kgs_diag_lorec(buf, CAP, ctypes.byref(n), 1 if reset else 0))
        return [tuple(buf[4 * i:4 * i + 4]) for i in range(n.value)]

    nbits = 20
    n = 1 << nbits
    ctxs = [K.Context(0) for _ in range(4)]
    ptau = f"/tmp/kgs_bench_p{nbits}.ptau"
    if not os.path.exists(ptau):
        ctxs[0].write_synthetic_ptau(ptau, nbits, bench.bench_tau())
    for c in ctxs:
        c.load_ptau(ptau, nbits)
    keep, bufs = [], []
    for ci in range(len(ctxs)):
        f, t = bench.synth_evals(n, 100 * ci)
        tf = torch.from_numpy(f.reshape(-1).copy()).cuda()
        tt = torch.from_numpy(t.reshape(-1).copy()).cuda()
        keep += [tf, tt]
        bufs.append(([tf.data_ptr()], [tt.data_ptr()]))
    torch.cuda.synchronize()

    # the MSM alone (bench.py's msm leg)
    sc = torch.from_numpy(bench.synth_evals(n, 777)[0].reshape(-1).copy()).cuda()
    phase = (ctypes.c_double * 4)()
    entries = ctypes.c_uint64()
    K._check(L.kgs_bench_msm_phases(ctxs[0].handle, ctypes.c_void_p(sc.data_ptr()), n, 2, phase, ctypes.byref(entries)))
    fetch()
    K._check(L.kgs_bench_msm_phases(ctxs[0].handle, ctypes.c_void_p(sc.data_ptr()), n, 5, phase, ctypes.byref(entries)))
    describe(launches(fetch()), "MSM alone (2^20 points)")

    # one proof at a time on one context (two MSM lanes)
    ctxs[0].set_msm_lanes(2)
    ctxs[0].prove_device(K.GRANDSUM, nbits, *bufs[0])
    fetch()
    for _ in range(3):
        ctxs[0].prove_device(K.GRANDSUM, nbits, *bufs[0])
    describe(launches(fetch()), "one proof at a time")

    # four proofs in flight (bench.py's headline configuration), one MSM lane each
    for c in ctxs:
        c.set_msm_lanes(1)

    def run(i, per):
        for _ in range(per):
            ctxs[i].prove_device(K.GRANDSUM, nbits, *bufs[i])

    for per, label in ((2, None), (2, "four proofs in flight")):
        th = [threading.Thread(target=run, args=(i, per)) for i in range(len(ctxs))]
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
        recs = fetch()
        if label:
            describe(launches(recs), label)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
