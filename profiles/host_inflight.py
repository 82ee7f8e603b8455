"""Proofs in flight through the host-buffer boundary (kgs_prove on pageable F/T, Montgomery write-back
into caller-owned host buffers) against the same proofs device-resident (kgs_prove_device), same box,
interleaved: where the drop-in path's in-flight throughput goes.
usage: python profiles/host_inflight.py [nbits=20] [contexts=4] [steps=32] [reps=3] [modes=device,host]
  contexts: comma-separated context counts to sweep (one MSM lane each, as bench.py's in-flight contexts)
Prints one line per (rep, mode, contexts): proofs/s."""
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    a = sys.argv[1:]
    nbits = int(a[0]) if len(a) > 0 else 20
    counts = [int(x) for x in (a[1] if len(a) > 1 else "4").split(",")]
    steps = int(a[2]) if len(a) > 2 else 32
    reps = int(a[3]) if len(a) > 3 else 3
    modes = (a[4] if len(a) > 4 else "device,host").split(",")
    K = bench.load_pkg()
    n = 1 << nbits
    path = f"/tmp/kgs_bench_p{nbits}.ptau"
    ctxs = [K.Context(0) for _ in range(max(counts))]
    if not os.path.exists(path):
        ctxs[0].write_synthetic_ptau(path, nbits, bench.bench_tau())
    data = []
    for ci, c in enumerate(ctxs):
        c.load_ptau(path, nbits)
        c.set_msm_lanes(1)
        f, t = bench.synth_evals(n, 100 * ci)
        df = torch.from_numpy(f.reshape(-1).copy()).cuda()
        dt = torch.from_numpy(t.reshape(-1).copy()).cuda()
        data.append(((df, dt), ([f.tobytes()], [t.tobytes()]), ([bytearray(32 * n)], [bytearray(32 * n)])))
    torch.cuda.synchronize()

    def run(mode, ci, count):
        c = ctxs[ci]
        (df, dt), (hf, ht), wb = data[ci]
        for _ in range(count):
            if mode == "device":
                c.prove_device(K.GRANDSUM, nbits, [df.data_ptr()], [dt.data_ptr()])
            elif mode == "host":
                c.prove(K.GRANDSUM, nbits, hf, ht, mont_out=wb)
            else:  # host inputs, no write-back
                c.prove(K.GRANDSUM, nbits, hf, ht, mont_out=False)

    def go(mode, m, total):
        share = [total // m + (1 if i < total % m else 0) for i in range(m)]
        th = [threading.Thread(target=run, args=(mode, i, share[i])) for i in range(m)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    for mode in modes:
        for m in counts:
            go(mode, m, 2 * m)  # warm
    def cpu_stat():  # the box's cgroup CPU accounting (quota throttling), when readable
        try:
            with open("/sys/fs/cgroup/cpu.stat") as fh:
                return {k: int(v) for k, v in (ln.split() for ln in fh if ln.strip())}
        except Exception:
            return None

    for r in range(reps):
        for m in counts:
            for mode in modes:
                s0 = cpu_stat()
                el = go(mode, m, steps)
                s1 = cpu_stat()
                extra = ""
                if s0 and s1:
                    d = {k: s1[k] - s0.get(k, 0) for k in ("usage_usec", "nr_throttled", "throttled_usec") if k in s1}
                    extra = (f" | cpu {d.get('usage_usec', 0) / 1e3 / el / 1e3:5.2f} cores, throttled "
                             f"{d.get('nr_throttled', 0)} periods {d.get('throttled_usec', 0) / 1e3:.1f} ms")
                print(f"rep {r} {mode:8s} contexts {m}: {steps / el:7.2f} proofs/s{extra}", flush=True)


if __name__ == "__main__":
    main()
