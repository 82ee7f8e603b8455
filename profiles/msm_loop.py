#!/usr/bin/env python3
"""Profiling driver for the MSM alone: REPS commitments of 2^NBITS random scalars on cuda:0 against the
resident SRS of a synthetic ptau (the same kgs_bench_msm_phases call bench.py's `msm` leg makes), so
every k_accumulate dispatch in the trace / PMC pass is a 2^NBITS-point launch.
usage: msm_loop.py [NBITS=20] [REPS=5] [skew]
Run it under `rocprofv3 --kernel-trace --stats ...` or one `rocprofv3 --pmc <counters> ...` pass."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    K = bench.load_pkg()
    n = 1 << nb
    ctx = K.Context(0)
    ptau = f"/tmp/kgs_bench_p{nb}.ptau"
    if not os.path.exists(ptau):
        ctx.write_synthetic_ptau(ptau, nb, bench.bench_tau())
    ctx.load_ptau(ptau, nb)
    if len(sys.argv) > 3 and sys.argv[3] == "skew":  # a selector's commitment: every scalar equal
        import numpy as np
        sc = torch.from_numpy(np.tile(np.frombuffer(K.FR_ONE_MONT, dtype=np.uint8), n)).cuda()
    else:
        sc = torch.from_numpy(bench.synth_evals(n, 777)[0].reshape(-1).copy()).cuda()
    phase = (ctypes.c_double * 4)()
    entries = ctypes.c_uint64()
    K._check(K.lib().kgs_bench_msm_phases(ctx.handle, ctypes.c_void_p(sc.data_ptr()), n, reps, phase,
                                          ctypes.byref(entries)))
    ph = [round(phase[i] / reps, 4) for i in range(4)]
    print(f"{os.environ.get('KGS_LIB', 'in-tree')}: msm 2^{nb}{' skew' if len(sys.argv) > 3 else ''}: {reps} reps, entries {entries.value}, phase ms (sort, accumulate, combine, reduce) {ph}",
          flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
