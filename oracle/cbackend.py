"""ctypes wrapper of the C restatement (oracle/c/oracle.c -> oracle/build/liboracle.so).

TEST INFRASTRUCTURE / CPU BASELINE ONLY: used by tests/ as a second, independent checker for
sizes the pure-Python oracle is too slow for, and by bench.py's `cpu_baseline` leg ("port": the
reference op list re-stated in C with OpenMP, timed on the GPU box's host cores).
"""
import ctypes
import os
import time

from . import bn254 as bn
from .ptau import read_header, read_sections

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            import subprocess
            subprocess.check_call(["make", "-C", os.path.join(HERE, "c")])
        L = ctypes.CDLL(LIB)
        P = ctypes.POINTER(ctypes.c_char_p)
        L.orc_prove.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, ctypes.c_char_p, ctypes.c_char_p,
                                ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
        L.orc_msm.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_char_p]
        L.orc_msm.restype = None
        L.orc_keccak256.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
        L.orc_keccak256.restype = None
        L.orc_ntt.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
        L.orc_ntt.restype = None
        L.orc_eval_evals_std.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p]
        _lib = L
    return _lib


def eval_evals_std(evals_std, nbits, x):
    """p(x) (int) from p's standard-form evaluations on <w_n> (barycentric, OpenMP)."""
    out = ctypes.create_string_buffer(32)
    rc = lib().orc_eval_evals_std(evals_std, nbits, int(x).to_bytes(32, "little"), out)
    if rc != 0:
        raise ValueError("x lies in the evaluation domain")
    return int.from_bytes(out.raw, "little")


def ntt(data_mont, inverse=False, threads=0):
    """Natural-order NTT / inverse NTT of Montgomery-form bytes (oracle.c ntt)."""
    buf = ctypes.create_string_buffer(bytes(data_mont), len(data_mont))
    lib().orc_ntt(buf, len(data_mont) // 32, 1 if inverse else 0, threads)
    return buf.raw[:len(data_mont)]


def load_srs_bytes(ptau_path):
    data, sections = read_sections(ptau_path)
    _, power, _ = read_header(data, sections)
    p2, s2 = sections[2][0]
    return power, data[p2:p2 + s2]


MESSAGES = {-3: None, -4: "Polynomial is not divisible", -5: "Polynomial does not divide"}


def prove_raw(kind, nbits, Fs, Ts, sF, sT, srs_bytes, threads=0):
    """kind 0/1/2 (grand-sum, grand-product, lookup); Fs/Ts lists of std bytes; sF/sT Montgomery
    bytes or None -> (coms, evs)."""
    k = len(Fs)
    sel = sF is not None
    nc = 2 * k + (2 if sel else 0) + 4
    ne = (2 if kind != 1 else 1) * k + (2 if sel else 0) + 1
    com = ctypes.create_string_buffer(64 * nc)
    ev = ctypes.create_string_buffer(32 * ne)
    FA = (ctypes.c_char_p * k)(*Fs)
    TA = (ctypes.c_char_p * k)(*Ts)
    rc = lib().orc_prove(kind, nbits, k, FA, TA, sF, sT, srs_bytes, len(srs_bytes) // 64, threads, com, ev)
    if rc == -3:
        raise ValueError("The grand-sum polynomial S is not well calculated" if kind != 1
                         else "The grand-product polynomial Z is not well calculated")
    if rc:
        raise ValueError(MESSAGES.get(rc, f"oracle error {rc}"))
    return [com.raw[64 * i:64 * i + 64] for i in range(nc)], [ev.raw[32 * i:32 * i + 32] for i in range(ne)]


def msm(srs_bytes, scalars_mont, threads=0):
    out = ctypes.create_string_buffer(64)
    lib().orc_msm(srs_bytes, scalars_mont, len(scalars_mont) // 32, threads, out)
    return out.raw


def cpu_baseline(nbits, kind="grandsum", threads=0, ptau=None, max_seconds=90.0, reps=3, inputs=None, expect=None):
    """Time the C port on the bench workload as BASELINE.md:84-87 prescribes: 1 warm-up proof, then
    the median of `reps` (>= 3) timed proofs, with their spread. If the warm-up alone shows that
    warm-up + reps would exceed `max_seconds`, fewer timed proofs are run (at least one) and the
    sample says so. `inputs` = (F list, T list) of standard-form bytes: exactly the multiset of the GPU's timed proofs
    (bench.py passes context 0's); default: the bench generator's first multiset. `expect` = the GPU
    proof (commitments, evaluations) of those inputs: the last CPU proof is compared with it byte for
    byte (`proof_identical`). Returns the bench.py `cpu_baseline` object."""
    import numpy as np
    n = 1 << nbits
    if inputs is None:
        rng = np.random.Generator(np.random.PCG64(0x4B5A4753))
        w = rng.integers(0, np.iinfo(np.uint64).max, size=(n, 4), dtype=np.uint64, endpoint=True)
        w[:, 3] &= np.uint64((1 << 61) - 1)
        f = np.ascontiguousarray(w).view(np.uint8).reshape(n, 32)
        t = np.roll(f, 1, axis=0)
        inputs = ([f.tobytes()], [t.tobytes()])
    _, srs = load_srs_bytes(ptau)
    kk = 0 if kind == "grandsum" else 1
    if threads <= 0:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    fb, tb = [bytes(x) for x in inputs[0]], [bytes(x) for x in inputs[1]]
    last = {}

    def one():
        t0 = time.perf_counter()
        last["proof"] = prove_raw(kk, nbits, fb, tb, None, None, srs, threads)
        return time.perf_counter() - t0
    warm = one()
    k = max(1, min(reps, int((max_seconds - warm) // max(warm, 1e-9))))
    times = sorted(one() for _ in range(k))
    identical = None
    if expect is not None:
        identical = list(last["proof"][0]) == list(expect[0]) and list(last["proof"][1]) == list(expect[1])
    med = times[len(times) // 2] if len(times) % 2 else 0.5 * (times[len(times) // 2 - 1] + times[len(times) // 2])
    return {"value": round(1.0 / med, 5), "unit": "proofs/s", "cores": threads, "kind": "port",
            "median_s_per_proof": round(med, 3), "min_s": round(times[0], 3), "max_s": round(times[-1], 3),
            "spread_pct": round(100.0 * (times[-1] - times[0]) / med, 1), "warmup_s": round(warm, 3),
            "proof_identical": identical,
            "sample": f"1 warm-up + median of {k} full {kind} proof(s) at n=2^{nbits}, k={len(fb)} (oracle/c C restatement "
                      f"of the reference op list incl. 4n multiply, OpenMP {threads} threads) on the multiset of the GPU's "
                      f"timed proofs: {med:.2f} s/proof "
                      f"(min {times[0]:.2f}, max {times[-1]:.2f})" + ("" if k >= 3 else f"; capped at {max_seconds:.0f} s")}
