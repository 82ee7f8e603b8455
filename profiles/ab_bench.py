"""Same-box A/B of library variants: bench.py (headline leg only) with KGS_LIB pointing at each
variant in turn, interleaved over `reps` rounds; one summary line per run.

    python profiles/ab_bench.py REPS ab/base/libkgs.so ab/x/libkgs.so ...

Each bench run is a child process under its own time limit; a failing run ends the script."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    reps, libs = int(sys.argv[1]), sys.argv[2:]
    args = ["--no-cpu-baseline", "--no-extra-legs", "--no-host-leg", "--steps", "64", "--msm-reps", "10"]
    for rep in range(1, reps + 1):
        for lib in libs:
            env = dict(os.environ, KGS_LIB=os.path.abspath(lib))
            p = subprocess.run(["timeout", "-k", "10", "180", sys.executable, os.path.join(ROOT, "bench.py")] + args,
                               env=env, capture_output=True, text=True, cwd=ROOT)
            if p.returncode != 0:
                print(f"{lib} rep {rep}: bench failed rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                sys.exit(1)
            d = json.loads(p.stdout.strip().splitlines()[-1])
            ph = d["msm"]["phase_ms"]
            print(f"{lib} rep {rep}: {d['value']:.2f} proofs/s  lat {d['latency_ms_single_proof']:.3f} ms  "
                  f"msm {d['msm']['ms']:.4f}  acc {ph['accumulate']:.4f}  combine {ph['combine']:.4f}  "
                  f"reduce {ph['reduce']:.4f}", flush=True)


if __name__ == "__main__":
    main()
