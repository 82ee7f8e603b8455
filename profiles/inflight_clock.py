#!/usr/bin/env python3
"""Clock held under k_accumulate, alone and with four proofs in flight (diagnostic build only).

The -DKGS_DIAG_CLOCK library stamps s_memtime / s_memrealtime around each accumulate block's add
loop (msm.hip); kgs_diag_clock returns the median of d(shader clock)/d(real time) x 100 MHz over the
blocks of the last launch. Counters cannot give this in flight (a --pmc pass serialises dispatches).
With the VALU instructions of one proof (profiles/r02/pmc/clock_valu_prove_loop_2p20.csv: 5,953 M)
the in-flight rate then gives the achieved SIMD cycles per VALU instruction of the whole pipeline.
usage: KGS_LIB=kzg-grandsums-study_amd/lib_diag/libkgs.so python3 profiles/inflight_clock.py"""
import ctypes
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

VALU_PER_PROOF = 5463.5e6  # wave64 VALU instructions of one 2^20 grand-sum proof (round-4 counter pass, profiles/r04/check/valu_share.txt)


def main():
    K = bench.load_pkg()
    L = K.lib()
    if not hasattr(L, "kgs_diag_clock"):
        sys.exit("not a -DKGS_DIAG_CLOCK build (set KGS_LIB)")
    L.kgs_diag_clock.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int)]

    def clock():
        g, nb = ctypes.c_double(), ctypes.c_int()
        K._check(L.kgs_diag_clock(ctypes.byref(g), ctypes.byref(nb)))
        return round(g.value, 3), nb.value

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

    # the MSM alone (as bench.py's msm leg)
    sc = torch.from_numpy(bench.synth_evals(n, 777)[0].reshape(-1).copy()).cuda()
    phase = (ctypes.c_double * 4)()
    entries = ctypes.c_uint64()
    K._check(L.kgs_bench_msm_phases(ctxs[0].handle, ctypes.c_void_p(sc.data_ptr()), n, 5, phase, ctypes.byref(entries)))
    print(f"MSM alone (2^20 points): accumulate {phase[1] / 5:.4f} ms, clock {clock()} (GHz, blocks)", flush=True)

    # one proof at a time on one context
    ctxs[0].set_msm_lanes(2)
    for _ in range(3):
        ctxs[0].prove_device(K.GRANDSUM, nbits, *bufs[0])
    t0 = time.perf_counter()
    for _ in range(8):
        ctxs[0].prove_device(K.GRANDSUM, nbits, *bufs[0])
    el = (time.perf_counter() - t0) / 8
    print(f"one proof at a time: {1e3 * el:.2f} ms per proof, clock of the last accumulate {clock()}", flush=True)

    # four proofs in flight (bench.py's headline configuration)
    for c in ctxs:
        c.set_msm_lanes(1)
    per = 32

    def run(i):
        for _ in range(per):
            ctxs[i].prove_device(K.GRANDSUM, nbits, *bufs[i])

    for rep in range(3):
        th = [threading.Thread(target=run, args=(i,)) for i in range(len(ctxs))]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        rate = per * len(ctxs) / el
        ghz, nb = clock()
        cpi = ghz * 1e9 * 1024 / (VALU_PER_PROOF * rate)
        print(f"in flight x4, rep {rep}: {rate:.2f} proofs/s, clock under the last accumulate {ghz} GHz ({nb} blocks);"
              f" pipeline {cpi:.2f} SIMD cycles per VALU instruction at that clock", flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
