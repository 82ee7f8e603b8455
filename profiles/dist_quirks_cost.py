"""Cost of the reference-quirks detection in the DISTRIBUTED prover (the default-on mode
adds degree all-gathers and host syncs to every group proof). One in-process rank group of W
contexts on one GPU (one host thread per rank), grand-sum n = 2^nbits, k = 1, host inputs;
proofs timed back to back with the mode off and on, interleaved.
usage: python profiles/dist_quirks_cost.py [nbits=20] [world=4] [proofs=4] [reps=3]"""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    a = sys.argv[1:]
    nbits = int(a[0]) if len(a) > 0 else 20
    world = int(a[1]) if len(a) > 1 else 4
    proofs = int(a[2]) if len(a) > 2 else 4
    reps = int(a[3]) if len(a) > 3 else 3
    K = bench.load_pkg()
    path = f"/tmp/kgs_bench_p{nbits}.ptau"
    ctxs = [K.Context(0) for _ in range(world)]
    if not os.path.exists(path):
        ctxs[0].write_synthetic_ptau(path, nbits, bench.bench_tau())
    g = K.Group.local(world)
    for r, c in enumerate(ctxs):
        c.load_ptau(path, nbits)
        c.set_group(g, r)
    f, t = bench.synth_evals(1 << nbits, 5)
    Fs, Ts = [f.tobytes()], [t.tobytes()]

    def one_round():
        errs = []

        def run(r):
            try:
                ctxs[r].prove(K.GRANDSUM, nbits, Fs, Ts, mont_out=False)
            except Exception as e:  # pragma: no cover
                errs.append(e)
        th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        if errs:
            raise errs[0]

    for on in (0, 1):
        for c in ctxs:
            c.set_reference_quirks(on)
        one_round()  # warm
    for rep in range(reps):
        for on in (0, 1):
            for c in ctxs:
                c.set_reference_quirks(on)
            t0 = time.perf_counter()
            for _ in range(proofs):
                one_round()
            ms = 1000.0 * (time.perf_counter() - t0) / proofs
            print(f"rep {rep} quirks {'on ' if on else 'off'} W={world} 2^{nbits}: {ms:8.3f} ms/proof", flush=True)
    for c in ctxs:
        c.set_group(None)
        c.close()
    g.close()


if __name__ == "__main__":
    main()
