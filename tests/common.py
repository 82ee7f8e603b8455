"""Shared helpers for the test-suite: package loader, deterministic inputs, ptau fixtures.

Inputs reproduce the reference tests' patterns (test/mset_eq_kzg_grandsum.test.js:24-104):
F random, T = F rotated by one (T[0] = F[n-1], T[i] = F[i-1]); selectors all ones except
selF[n-1] = 0 and selT[0] = 0. Unlike the reference (unseeded Fr.random()), they are seeded.
"""
import hashlib
import importlib.util
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import bn254 as bn  # noqa: E402
from oracle import ptau as opt  # noqa: E402

R = bn.R
_PKG = None


def load_pkg():
    global _PKG
    if _PKG is None:
        spec = importlib.util.spec_from_file_location(
            "kgs_amd", os.path.join(ROOT, "kzg-grandsums-study_amd", "__init__.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _PKG = mod
    return _PKG


def std_bytes(vals):
    return b"".join(bn.fr_std_to_bytes(v) for v in vals)


def mont_bytes(vals):
    return b"".join(bn.fr_to_bytes(v) for v in vals)


def make_inputs(seed, nbits, npols, selected):
    """-> (list of F std-bytes, list of T std-bytes, selF mont-bytes|None, selT mont-bytes|None)"""
    rnd = random.Random(seed)
    n = 1 << nbits
    Fs, Ts = [], []
    for _ in range(npols):
        f = [rnd.randrange(R) for _ in range(n)]
        t = [f[-1]] + f[:-1]
        Fs.append(std_bytes(f))
        Ts.append(std_bytes(t))
    sF = sT = None
    if selected:
        a = [1] * n
        a[-1] = 0
        b = [1] * n
        b[0] = 0
        sF, sT = mont_bytes(a), mont_bytes(b)
    return Fs, Ts, sF, sT


def make_lookup_inputs(seed, nbits, npols, unselected=0):
    """Lookup inputs (test/lookup_kzg_grandsum.test.js:24-44 pattern, generalised): a random table T
    (k columns), every F row a random table row, `unselected` F rows switched off in selF, and the
    multiplicities m[j] = #selected F rows equal to table row j.
    -> (F std-bytes list, T std-bytes list, selF mont-bytes, m mont-bytes)"""
    rnd = random.Random(seed)
    n = 1 << nbits
    T = [[rnd.randrange(R) for _ in range(n)] for _ in range(npols)]
    rows = [rnd.randrange(n) for _ in range(n)]
    sel = [1] * n
    for i in rnd.sample(range(n), unselected):
        sel[i] = 0
    m = [0] * n
    for i in range(n):
        m[rows[i]] += sel[i]
    Fs = [std_bytes([T[c][rows[i]] for i in range(n)]) for c in range(npols)]
    return Fs, [std_bytes(t) for t in T], mont_bytes(sel), mont_bytes(m)


def lookup_dup_table(seed, nbits):
    """A table with every value twice (T[2j] = T[2j+1]); F rows drawn from it; each looked-up
    value's multiplicity split at random between its two table rows."""
    rnd = random.Random(seed)
    n = 1 << nbits
    vals = [rnd.randrange(R) for _ in range(n // 2)]
    t = [vals[j // 2] for j in range(n)]
    f = [vals[rnd.randrange(n // 2)] for _ in range(n)]
    m = [0] * n
    for v in f:
        j = vals.index(v)
        m[2 * j + rnd.randrange(2)] += 1
    return [std_bytes(f)], [std_bytes(t)], mont_bytes([1] * n), mont_bytes(m)


def lookup_all_zero(seed, nbits):
    """selF and the multiplicities all zero, F unrelated to T: trivially satisfied (the reference's
    prover warns "The selection buffers are all zeros", prover.js:66-68, and proves)."""
    rnd = random.Random(seed)
    n = 1 << nbits
    f = [rnd.randrange(R) for _ in range(n)]
    t = [rnd.randrange(R) for _ in range(n)]
    return [std_bytes(f)], [std_bytes(t)], mont_bytes([0] * n), mont_bytes([0] * n)


def reference_standard_lookup(seed=3, nbits=2):
    """The reference's commented-out "standard lookup" case (test/lookup_kzg_grandsum.test.js:24-44):
    T random, F = T with F[1] = F[n-1] = F[0], selF all ones, multiplicities one except m[0] = 3,
    m[1] = m[n-1] = 0."""
    rnd = random.Random(seed)
    n = 1 << nbits
    t = [rnd.randrange(R) for _ in range(n)]
    f = list(t)
    f[1] = f[0]
    f[n - 1] = f[0]
    m = [1] * n
    m[0], m[1], m[n - 1] = 3, 0, 0
    return [std_bytes(f)], [std_bytes(t)], mont_bytes([1] * n), mont_bytes(m)


def inputs_digest(Fs, Ts, sF, sT):
    h = hashlib.sha256()
    for x in Fs + Ts + [sF or b"", sT or b""]:
        h.update(x)
    return h.hexdigest()


TAU = None


def tau():
    global TAU
    if TAU is None:
        TAU = opt.bench_tau()
    return TAU


def oracle_ptau(power):
    """Synthetic ptau written by the ORACLE's writer (cached under /tmp)."""
    path = f"/tmp/kgs_test_oracle_p{power}.ptau"
    if not os.path.exists(path):
        tmp = path + f".{os.getpid()}"
        opt.write_synthetic_ptau(tmp, power, tau())
        os.replace(tmp, path)
    return path
