#!/usr/bin/env python3
"""Per-rank work of the distributed prover (kgs_ctx_set_group) on ONE GPU: W in-process ranks
(W contexts, one host thread each) prove the same statement; under `rocprofv3 --kernel-trace` the
dispatches are attributed to ranks by launching host thread, so each rank's kernel time can be
compared with the single-GPU prover's (W = 1 through the same code path).
usage: python3 profiles/dist_scaling.py NBITS [W ...]   (prints a marker line per configuration)"""
import os
import sys
import threading
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import bench  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 22
    worlds = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8]
    K = bench.load_pkg()
    import torch
    ptau = f"/tmp/kgs_bench_p{nb}.ptau"
    if not os.path.exists(ptau):
        c = K.Context(0)
        c.write_synthetic_ptau(ptau, nb, bench.bench_tau())
        c.close()
    f, t = bench.synth_evals(1 << nb, 42)
    df = torch.from_numpy(f.reshape(-1).copy()).to("cuda:0")
    dt = torch.from_numpy(t.reshape(-1).copy()).to("cuda:0")
    for W in worlds:
        g = K.Group.local(W)
        ctxs = [K.Context(0) for _ in range(W)]
        for r, c in enumerate(ctxs):
            c.load_ptau(ptau, nb)
            c.set_group(g, r)
            c.set_msm_lanes(1)
        res = [None] * W
        bar = threading.Barrier(W + 1)

        def rank(r):
            print(f"RANKTID W={W} r={r} tid={threading.get_native_id()}", flush=True)
            for reps in (1, 3):  # warm-up proof, then the timed ones
                bar.wait()
                for _ in range(reps):
                    res[r] = ctxs[r].prove_device(K.GRANDSUM, nb, [df.data_ptr()], [dt.data_ptr()])
                bar.wait()
        th = [threading.Thread(target=rank, args=(r,)) for r in range(W)]
        for x in th:
            x.start()
        for reps, tag in ((1, "warm"), (3, "timed")):
            bar.wait()
            t0 = time.perf_counter()
            bar.wait()
            el = time.perf_counter() - t0
            print(f"DIST W={W} nbits={nb} {tag} reps={reps} wall_ms_per_proof={1000 * el / reps:.2f} "
                  f"agree={all(x == res[0] for x in res)}", flush=True)
        for x in th:
            x.join()
        for c in ctxs:
            c.set_group(None)
            c.close()
        g.close()


if __name__ == "__main__":
    main()
