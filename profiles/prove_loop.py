#!/usr/bin/env python3
"""Profiling driver: a few back-to-back proofs of one configuration on cuda:0 (device-resident
inputs, synthetic ptau written by the product), printing per-proof wall time and round timings.
usage: prove_loop.py NBITS NPOLS [sel] [lanes1]     e.g. prove_loop.py 24 1 lanes1; prove_loop.py 22 4 sel
Run it under `rocprofv3 --kernel-trace --stats ...` for per-kernel numbers."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = bench.load_pkg()
    nb, k = int(sys.argv[1]), int(sys.argv[2])
    sel = "sel" in sys.argv[3:]
    n = 1 << nb
    ctx = K.Context(0)
    ptau = f"/tmp/kgs_bench_p{nb}.ptau"
    if not os.path.exists(ptau):
        ctx.write_synthetic_ptau(ptau, nb, bench.bench_tau())
    ctx.load_ptau(ptau, nb)
    ctx.set_msm_lanes(1 if "lanes1" in sys.argv[3:] else 2)
    keep, d_f, d_t = [], [], []
    for i in range(k):
        f, t = bench.synth_evals(n, 5000 + i)
        tf = torch.from_numpy(f.reshape(-1).copy()).cuda()
        tt = torch.from_numpy(t.reshape(-1).copy()).cuda()
        keep += [tf, tt]
        d_f.append(tf.data_ptr())
        d_t.append(tt.data_ptr())
    sfp = stp = None
    if sel:
        one = np.frombuffer(K.FR_ONE_MONT, dtype=np.uint8)
        sf = np.tile(one, n)
        st = sf.copy()
        sf[32 * (n - 1):] = 0
        st[:32] = 0
        tsf, tst = torch.from_numpy(sf).cuda(), torch.from_numpy(st).cuda()
        sfp, stp = tsf.data_ptr(), tst.data_ptr()
    for it in range(3):
        t0 = time.perf_counter()
        ctx.prove_device(K.GRANDSUM, nb, d_f, d_t, sfp, stp)
        rounds = [round(x, 2) for x in ctx.last_timing()]
        print(f"nb={nb} k={k} sel={sel} proof {it}: {1000 * (time.perf_counter() - t0):.1f} ms rounds {rounds}",
              flush=True)


if __name__ == "__main__":
    main()
