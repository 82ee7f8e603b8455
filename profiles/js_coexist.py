"""Does the JavaScript module's single-proof latency depend on another process holding contexts on
the same GPU? bench.py runs its JS leg (a node child process) while the bench process keeps its 4
in-flight contexts (streams, hardware queues, SRS copies) alive but idle.
usage: python profiles/js_coexist.py [reps=2]
Prints per mode: JS best / median of 7 single proofs, libkgs rounds of the best, 16-way proofs/s.
  alone   - no other context open in the parent
  held    - the parent holds 4 contexts that have proved (idle while node runs)
  closed  - the same contexts destroyed before node runs"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def run_node(ptau):
    js = os.path.join(ROOT, "kzg-grandsums-study_amd", "js", "test", "time_prove.js")
    env = dict(os.environ, KGS_JS_CONTEXTS="8", KGS_DEVICES="0")
    env.pop("KGS_JS_EAGER_GC", None)
    out = subprocess.run(["node", "--expose-gc", js, ptau, "20", "7", "16"], capture_output=True, text=True,
                         timeout=300, env=env)
    d = json.loads(out.stdout.strip().splitlines()[-1])
    lat = d["latency_ms"]
    rounds = d["best_inside_libkgs"]["libkgs_timing_ms"][:5]
    return (f"best {lat['min']:6.2f} median {lat['median']:6.2f} | rounds {' '.join(f'{x:5.2f}' for x in rounds)} | "
            f"16-way {d.get('concurrent_proofs_per_s', 0):6.2f}")


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    K = bench.load_pkg()
    ptau = "/tmp/kgs_bench_p20.ptau"
    c0 = K.Context(0)
    if not os.path.exists(ptau):
        c0.write_synthetic_ptau(ptau, 20, bench.bench_tau())
    c0.close()
    f, t = bench.synth_evals(1 << 20, 0)
    hf, ht = [f.tobytes()], [t.tobytes()]
    for rep in range(reps):
        print(f"rep {rep} alone  : {run_node(ptau)}", flush=True)
        ctxs = [K.Context(0) for _ in range(4)]
        for c in ctxs:
            c.load_ptau(ptau, 20)
            c.set_msm_lanes(1)
            c.prove(K.GRANDSUM, 20, hf, ht)
        print(f"rep {rep} held   : {run_node(ptau)}", flush=True)
        for c in ctxs:
            c.close()
        del ctxs
        print(f"rep {rep} closed : {run_node(ptau)}", flush=True)


if __name__ == "__main__":
    main()
