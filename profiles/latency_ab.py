#!/usr/bin/env python3
"""Single-proof latency of the grand-sum prover at n = 2^NBITS on cuda:0 (one context, two MSM lanes:
the latency mode), device-resident inputs: 3 warm-up proofs, then the median / min / max of PROOFS
and the per-round median. Same-box A/Bs run it once per setting in one process list, e.g.
  for v in 0 1 0 1; do KGS_X=$v python profiles/latency_ab.py 20 15; done
usage: latency_ab.py NBITS PROOFS"""
import hashlib
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    K = bench.load_pkg()
    nb, proofs = int(sys.argv[1]), int(sys.argv[2])
    n = 1 << nb
    ctx = K.Context(0)
    ptau = f"/tmp/kgs_bench_p{nb}.ptau"
    if not os.path.exists(ptau):
        ctx.write_synthetic_ptau(ptau, nb, bench.bench_tau())
    ctx.load_ptau(ptau, nb)
    ctx.set_msm_lanes(2)
    f, t = bench.synth_evals(n, 5000)
    tf = torch.from_numpy(f.reshape(-1).copy()).cuda()
    tt = torch.from_numpy(t.reshape(-1).copy()).cuda()
    ms, rounds, proof0 = [], [], None
    for it in range(3 + proofs):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = ctx.prove_device(K.GRANDSUM, nb, [tf.data_ptr()], [tt.data_ptr()], None, None)
        dt = 1000 * (time.perf_counter() - t0)
        proof0 = proof0 or p
        assert p == proof0, "proof changed between calls"
        if it >= 3:
            ms.append(dt)
            rounds.append(ctx.last_timing()[:5])
    env = {k: v for k, v in os.environ.items() if k.startswith("KGS_")}
    med = [round(statistics.median(r[i] for r in rounds), 3) for i in range(5)]
    sha = hashlib.sha256(b"".join(proof0[0] + proof0[1])).hexdigest()[:12]
    print(f"{env} n=2^{nb}: median {statistics.median(ms):.3f} ms min {min(ms):.3f} max {max(ms):.3f} "
          f"rounds {med} proof sha {sha}", flush=True)


if __name__ == "__main__":
    main()
