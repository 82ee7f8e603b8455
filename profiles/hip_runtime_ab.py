"""Single-proof latency through the host-buffer boundary (kgs_prove) under the HIP runtime a process
happens to load: with torch imported first, libkgs.so binds to torch's bundled libamdhip64 (ROCm 7.0
here); without torch (the JavaScript module's situation: node -> addon -> libkgs.so) it binds to
/opt/rocm's (7.2). Same box, same library, same inputs.
usage: python profiles/hip_runtime_ab.py torch|notorch [nbits=20] [reps=7]"""
import os
import sys
import time

if sys.argv[1] == "torch":
    import torch  # noqa: F401  (loads torch's libamdhip64 before libkgs.so)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def loaded_hip():
    with open("/proc/self/maps") as f:
        return sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln})


def main():
    nbits = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 7
    K = bench.load_pkg()
    ctx = K.Context(0)
    path = f"/tmp/kgs_bench_p{nbits}.ptau"
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, bench.bench_tau())
    ctx.load_ptau(path, nbits)
    ctx.set_msm_lanes(2)
    f, t = bench.synth_evals(1 << nbits, 0)
    hf, ht = [f.tobytes()], [t.tobytes()]
    wb = ([bytearray(32 << nbits)], [bytearray(32 << nbits)])
    for _ in range(2):
        ctx.prove(K.GRANDSUM, nbits, hf, ht, mont_out=wb)
    print(f"{sys.argv[1]}: {' '.join(loaded_hip())}", flush=True)
    tot = []
    for _ in range(reps):
        t0 = time.perf_counter()
        ctx.prove(K.GRANDSUM, nbits, hf, ht, mont_out=wb)
        el = 1e3 * (time.perf_counter() - t0)
        tot.append(el)
        tm = ctx.last_timing()
        print(f"{sys.argv[1]:8s} {el:7.2f} ms | rounds {' '.join(f'{x:5.2f}' for x in tm[:5])} | copy {tm[6]:5.2f}",
              flush=True)
    tot.sort()
    print(f"{sys.argv[1]} median {tot[len(tot) // 2]:.2f} ms min {tot[0]:.2f}", flush=True)


if __name__ == "__main__":
    main()
