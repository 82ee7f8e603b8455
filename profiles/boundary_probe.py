"""Host-buffer boundary vs device-resident latency of one grand-sum proof (one context, two MSM lanes),
round by round (kgs_last_timing): where the drop-in path's extra milliseconds go.
host_prereg: inputs pinned once by the caller (kgs_host_register), DMA'd in place.
usage: python profiles/boundary_probe.py [nbits=20] [reps=5]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import importlib  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402

K = importlib.import_module("kzg-grandsums-study_amd")


def main():
    nbits = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    ctx = K.Context(0)
    path = f"/tmp/kgs_bench_p{nbits}.ptau"
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, bench.bench_tau())
    ctx.load_ptau(path, nbits)
    ctx.set_msm_lanes(2)
    f, t = bench.synth_evals(1 << nbits, 0)
    hf, ht = [f.tobytes()], [t.tobytes()]
    df = torch.from_numpy(f.reshape(-1).copy()).cuda()
    dt = torch.from_numpy(t.reshape(-1).copy()).cuda()
    for _ in range(2):
        ctx.prove(K.GRANDSUM, nbits, hf, ht)
        ctx.prove_device(K.GRANDSUM, nbits, [df.data_ptr()], [dt.data_ptr()])
    # the same vectors in buffers the caller pinned once (kgs_host_register): DMA'd in place
    rf, rt = [bytearray(f.tobytes())], [bytearray(t.tobytes())]
    handles = [K.host_register(b) for b in rf + rt]
    wb = ([bytearray(len(hf[0]))], [bytearray(len(ht[0]))])  # recycled caller-owned write-back buffers
    fmt = lambda xs: " ".join(f"{x:6.2f}" for x in xs)  # noqa: E731
    for label, fn in (("device", lambda: ctx.prove_device(K.GRANDSUM, nbits, [df.data_ptr()], [dt.data_ptr()])),
                      ("host", lambda: ctx.prove(K.GRANDSUM, nbits, hf, ht)),
                      ("host_recycled", lambda: ctx.prove(K.GRANDSUM, nbits, hf, ht, mont_out=wb)),
                      ("host_no_mont", lambda: ctx.prove(K.GRANDSUM, nbits, hf, ht, mont_out=False)),
                      ("host_prereg", lambda: ctx.prove(K.GRANDSUM, nbits, rf, rt, mont_out=False))):
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            el = 1e3 * (time.perf_counter() - t0)
            tm = ctx.last_timing()
            print(f"{label:13s} {el:7.2f} ms | rounds {fmt(tm[:5])} | copy/prove/wb {fmt(tm[6:9]) if len(tm) > 6 else ''}",
                  flush=True)
    for h in handles:
        K.host_unregister(h)


if __name__ == "__main__":
    main()
