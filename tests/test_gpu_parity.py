"""GPU parity tests: the HIP path (through the C-ABI, lib/libkgs.so) against the CPU oracle.

Bit-exact on every output (integer arithmetic). Small sizes compare byte-for-byte with the oracle
and the committed golden vectors; large sizes (2^16 .. 2^20) use size-independent properties:
the proof verifies (trapdoor form of the reference's pairing check, O(1) group work) and the
transcript-independent commitments equal the closed form f(tau)·G1 computed barycentrically from
the evaluations.
"""
import json
import os
import random

import pytest

import common
from oracle import bn254 as bn
from oracle import poly as OP
from oracle import protocol as P

pytestmark = pytest.mark.gpu
R = bn.R
GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


@pytest.fixture(scope="module")
def K():
    return common.load_pkg()


@pytest.fixture(scope="module")
def ctx9(K):
    c = K.Context(0)
    c.load_ptau(common.oracle_ptau(9))
    return c


def rv(rnd, n):
    return [rnd.randrange(R) for _ in range(n)]


def unmb(b):
    return [bn.fr_from_bytes(b[32 * i:32 * i + 32]) for i in range(len(b) // 32)]


def test_synthetic_ptau_writer_matches_oracle(K):
    c = K.Context(0)
    for power in (3, 9):
        path = f"/tmp/kgs_test_gpu_p{power}.ptau"
        c.write_synthetic_ptau(path, power, common.tau())
        assert open(path, "rb").read() == open(common.oracle_ptau(power), "rb").read()
    c.close()


def test_to_mont(ctx9):
    rnd = random.Random(1)
    v = rv(rnd, 777)
    assert ctx9.fr_to_mont(common.std_bytes(v)) == common.mont_bytes(v)
    # non-canonical standard forms (r <= x < 2^256): the Evaluations buffers are read mod r (oracle
    # protocol.Evaluations.std_values); k_to_mont's 29-bit product takes any x < 2^256
    raw = [R, R + 1, 2 * R - 1, 5 * R - 1, (1 << 256) - 1] + [rnd.randrange(R, 1 << 256) for _ in range(300)]
    b = b"".join(x.to_bytes(32, "little") for x in raw)
    assert ctx9.fr_to_mont(b) == common.mont_bytes([x % R for x in raw])


def test_from_mont_and_batch_inverse(ctx9):
    # [ffjs] Fr.batchFromMontgomery / Fr.batchInverse (grandsum.js:41): ragged sizes across the
    # 32-element per-thread chunks, zeros (kept zero), one and r - 1
    rnd = random.Random(3)
    for n in (1, 2, 31, 32, 33, 777, 4099):
        v = rv(rnd, n)
        v[0] = 0
        if n > 2:
            v[1], v[-1] = 1, R - 1
        if n > 40:
            v[32] = v[33] = 0
        assert ctx9.fr_from_mont(common.mont_bytes(v)) == common.std_bytes(v)
        assert unmb(ctx9.fr_batch_inverse(common.mont_bytes(v))) == [pow(x, R - 2, R) for x in v]
    assert ctx9.fr_from_mont(b"") == b"" and ctx9.fr_batch_inverse(b"") == b""


# 0..10: radix-8/4/2 passes only; 11..17: LDS-staged passes of 6/5/4 stages (k_ntt_lds_pass<3,3>,
# <3,2>, <2,2>) followed by radix-8/4/2 passes, in every combination (11 = 6+5, 13 = 6+6+1,
# 14 = 6+6+2, 15 = 6+6+3, 16 = 6+6+4, 17 = 6+6+5)
@pytest.mark.parametrize("logm", list(range(0, 18)))
def test_ntt(ctx9, logm):
    rnd = random.Random(logm)
    v = rv(rnd, 1 << logm)
    assert unmb(ctx9.ntt(common.mont_bytes(v), False)) == OP.ntt(v, False)
    assert unmb(ctx9.ntt(common.mont_bytes(v), True)) == OP.ntt(v, True)


# 18..22: three-pass plans with up to 9 stages in one pass (lds_plan: 9+9, 6+6+7, 6+6+8, 6+6+9, 7+6+9),
# byte-for-byte against the C restatement's transform (oracle.c ntt)
@pytest.mark.parametrize("logm", [18, 19, 20, 21, 22])
def test_ntt_large_vs_c_oracle(ctx9, logm):
    import numpy as np
    from oracle import cbackend as C
    rng = np.random.Generator(np.random.PCG64(logm))
    w = rng.integers(0, 2**64 - 1, size=(1 << logm, 4), dtype=np.uint64, endpoint=True)
    w[:, 3] &= np.uint64((1 << 60) - 1)  # < r: canonical Montgomery-form elements
    x = w.tobytes()
    for inverse in (False, True):
        assert ctx9.ntt(x, inverse) == C.ntt(x, inverse), inverse


_T32 = """
import hashlib, json, sys
sys.path.insert(0, {tests!r})
import numpy as np
import common
K = common.load_pkg()
c = K.Context(0)
out = {{}}
for logm in (11, 14, 17, 20, 21):
    rng = np.random.Generator(np.random.PCG64(100 + logm))
    w = rng.integers(0, 2**64 - 1, size=(1 << logm, 4), dtype=np.uint64, endpoint=True)
    w[:, 3] &= np.uint64((1 << 60) - 1)
    x = w.tobytes()
    out[str(logm)] = [hashlib.sha256(c.ntt(x, inv)).hexdigest() for inv in (False, True)]
path = "/tmp/kgs_test_t32_p13.ptau"
c.write_synthetic_ptau(path, 13, common.tau())
c.load_ptau(path, 12)
rng = np.random.Generator(np.random.PCG64(7))
f = rng.integers(0, 2**64 - 1, size=(1 << 12, 4), dtype=np.uint64, endpoint=True)
f[:, 3] &= np.uint64((1 << 60) - 1)
t = np.roll(f, 1, axis=0)
coms, evs, mf, mt = c.prove(K.GRANDSUM, 12, [f.tobytes()], [t.tobytes()])
out["proof"] = hashlib.sha256(b"".join(coms) + b"".join(evs)).hexdigest()
print(json.dumps(out))
"""


def test_ntt_8x32_products_identical():
    """The NTT LDS passes multiply by 29-bit twiddle / scaling records (fr29.hpp) by default and by the
    8 x 32-bit words with KGS_NTT_T29=0: both builds give the same transforms (2^11..2^21, forward and
    inverse with 1/m) and the same proof (coset transforms of the quotient), each in a fresh process
    (the knob is read once per process)."""
    import json
    import subprocess
    import sys
    code = _T32.format(tests=os.path.dirname(os.path.abspath(__file__)))
    res = []
    for t29 in ("1", "0"):
        env = dict(os.environ, KGS_NTT_T29=t29)
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        res.append(json.loads(out.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1]


_PRIO = """
import hashlib, json, sys
sys.path.insert(0, {tests!r})
import numpy as np
import common
K = common.load_pkg()
out = {{}}
path = "/tmp/kgs_test_prio_p17.ptau"
c = K.Context(0)
c.write_synthetic_ptau(path, 17, common.tau())
c.load_ptau(path, 17)
rng = np.random.Generator(np.random.PCG64(11))
for nb in (12, 16, 17):
    w = rng.integers(0, 2**64 - 1, size=(1 << nb, 4), dtype=np.uint64, endpoint=True)
    w[:, 3] &= np.uint64((1 << 60) - 1)
    for lanes in (2, 1):
        c.set_msm_lanes(lanes)
        out[f"msm{{nb}}/{{lanes}}"] = c.msm(w.tobytes()).hex()
c.set_msm_lanes(2)
f = rng.integers(0, 2**64 - 1, size=(1 << 14, 4), dtype=np.uint64, endpoint=True)
f[:, 3] &= np.uint64((1 << 60) - 1)
t = np.roll(f, 1, axis=0)
coms, evs, mf, mt = c.prove(K.GRANDSUM, 14, [f.tobytes()], [t.tobytes()])
out["proof"] = hashlib.sha256(b"".join(coms) + b"".join(evs)).hexdigest()
print(json.dumps(out))
"""


def test_accumulate_priority_identical():
    """The accumulate's progress-stepped wave priority (KGS_ACC_PRIO: 1 = two-lane contexts, the
    default; 0 = off; 2 = every launch) only reorders issue: MSMs of 2^12..2^17 points on two-lane and
    one-lane contexts and a 2^14 proof are identical under all three, each in a fresh process (the
    knob is read once per process)."""
    import json
    import subprocess
    import sys
    code = _PRIO.format(tests=os.path.dirname(os.path.abspath(__file__)))
    res = []
    for prio in ("1", "0", "2"):
        env = dict(os.environ, KGS_ACC_PRIO=prio)
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        res.append(json.loads(out.stdout.strip().splitlines()[-1]))
    assert res[0] == res[1] == res[2]
    assert res[0]["msm16/2"] == res[0]["msm16/1"]


def test_msm(ctx9):
    srs = P.SRS(common.oracle_ptau(9), common.tau())
    rnd = random.Random(2)
    for n in (1, 2, 3, 31, 256, 1000, 1023):
        v = rv(rnd, n)
        assert ctx9.msm(common.mont_bytes(v)) == bn.g1_to_lem(srs.msm(v)), n
    # degenerate scalars: zeros, ones, r-1, repeated digits
    for v in ([0] * 5, [1] * 64, [R - 1] * 9, [1 << 200] * 17, [0, 0, 7]):
        assert ctx9.msm(common.mont_bytes(v)) == bn.g1_to_lem(srs.msm(v))
    assert ctx9.msm(common.mont_bytes([0] * 8)) == bytes(64)  # infinity


def test_msm_skewed_buckets(K):
    """Repeated scalars pile every point into one bucket per window (a selector polynomial's
    coefficients are all equal): exercises the chunked combine levels (k_combine_level)."""
    nbits = 16
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    srs = P.SRS(path, common.tau())
    rnd = random.Random(99)
    a, b = rnd.randrange(R), rnd.randrange(R)
    n = 1 << nbits
    cases = {
        "all-equal": [a] * n,
        "minus-1/n (selector pattern)": [(-pow(n, -1, R)) % R] * n,
        "two-valued": [a if i % 3 else b for i in range(n)],
        "mostly-zero": [a if i % 1000 == 0 else 0 for i in range(n)],
        "equal-then-random": [a] * (n // 2) + [rnd.randrange(R) for _ in range(n // 2)],
        "all-equal-odd-length": [b] * (n - 3),
    }
    for name, v in cases.items():
        assert ctx.msm(common.mont_bytes(v)) == bn.g1_to_lem(srs.msm(v)), name
    ctx.close()


def test_msm_skewed_multitile_linearity(K):
    """2^21 equal scalars: each window's 2^21 entries land in ONE bucket, so each partition is cut into
    SL_G chunks of 32 K entries, more than one LDS tile (k_lo_scatter's multi-tile path). Checked by
    linearity against two MSMs of random (non-skewed, single-tile) scalars: msm(a) = msm(r) + msm(a - r)."""
    nbits = 21
    n = 1 << nbits
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    rnd = random.Random(2121)
    a = rnd.randrange(R)
    rs = [rnd.randrange(R) for _ in range(n)]
    # Montgomery forms are linear: (a - r) of the byte values is the Montgomery form of the difference
    eq = a.to_bytes(32, "little") * n
    rb = b"".join(x.to_bytes(32, "little") for x in rs)
    db = b"".join(((a - x) % R).to_bytes(32, "little") for x in rs)
    p_eq = bn.g1_from_lem(ctx.msm(eq))
    p_sum = bn.g1_add(bn.g1_from_lem(ctx.msm(rb)), bn.g1_from_lem(ctx.msm(db)))
    assert p_eq == p_sum
    ctx.close()


@pytest.mark.parametrize("c", [18, 19, 20])
def test_msm_wide_windows(K, monkeypatch, c):
    """Windows wider than the default 17 (KGS_MSM_C; 512 / 1024 / 2048 sort partitions, a 2^17-2^19
    bucket tail): MSMs of random, degenerate and skewed scalars against oracle/c, and a proof
    byte-identical to the C restatement. A ptau file of its own keeps these tables from being shared
    with the default-window contexts."""
    from oracle import cbackend as C
    monkeypatch.setenv("KGS_MSM_C", str(c))
    nbits = 12
    path = f"/tmp/kgs_test_gpu_wide{c}.{os.getpid()}.ptau"
    try:
        ctx = K.Context(0)
        ctx.write_synthetic_ptau(path, nbits, common.tau())
        ctx.load_ptau(path, nbits)
        assert ctx.srs_info()[2] == c
        _, sb = C.load_srs_bytes(path)
        rnd = random.Random(c)
        n = 1 << nbits
        for v in (rv(rnd, 1), rv(rnd, 777), rv(rnd, n), [7] * n, [R - 1] * 33, [0] * 9 + [5]):
            mb = common.mont_bytes(v)
            assert ctx.msm(mb) == C.msm(sb, mb), len(v)
        Fs, Ts, sF, sT = common.make_inputs(3000 + c, 11, 2, True)
        got = ctx.prove(K.GRANDSUM, 11, Fs, Ts, sF, sT, mont_out=False)[:2]
        assert got == tuple(C.prove_raw(K.GRANDSUM, 11, Fs, Ts, sF, sT, sb, 0))
        ctx.close()
    finally:
        if os.path.exists(path):
            os.remove(path)


@pytest.mark.parametrize("kind", [0, 1])
@pytest.mark.parametrize("sel", [False, True])
@pytest.mark.parametrize("nbits", [1, 4, 11, 13])
def test_grand_builder(K, kind, sel, nbits):
    ctx = K.Context(0)
    ctx.load_ptau(common.oracle_ptau(3))
    rnd = random.Random(nbits * 10 + kind)
    n = 1 << nbits
    f = rv(rnd, n)
    t = [f[-1]] + f[:-1]
    g = rnd.randrange(R)
    sF = sT = None
    if sel:
        sF = [1] * n
        sF[-1] = 0
        sT = [1] * n
        sT[0] = 0
    got = ctx.grand_build(kind, common.mont_bytes(f), common.mont_bytes(t), bn.fr_to_bytes(g),
                          common.mont_bytes(sF) if sel else None, common.mont_bytes(sT) if sel else None)
    fn = P._grandsum_S if kind == 0 else P._grandproduct_Z
    assert unmb(got) == OP.ntt(fn(f, t, sF or [1] * n, sT or [1] * n, g).coef, False)
    # not a multiset -> the reference's error
    t2 = list(t)
    t2[3 % n] = (t2[3 % n] + 1) % R
    with pytest.raises(K.KgsError, match="not well calculated"):
        ctx.grand_build(kind, common.mont_bytes(f), common.mont_bytes(t2), bn.fr_to_bytes(g),
                        common.mont_bytes(sF) if sel else None, common.mont_bytes(sT) if sel else None)
    ctx.close()


@pytest.mark.parametrize("L", [2, 3, 8, 2047, 2048, 2049, 6000, 70000])
def test_eval_and_division(ctx9, L):
    rnd = random.Random(L)
    c = rv(rnd, L)
    x = rnd.randrange(R)
    assert bn.fr_from_bytes(ctx9.poly_eval(common.mont_bytes(c), bn.fr_to_bytes(x))) == OP.Polynomial(c).evaluate(x)
    c[0] = (c[0] - OP.Polynomial(c).evaluate(x)) % R
    q = unmb(ctx9.poly_div_x_sub(common.mont_bytes(c), bn.fr_to_bytes(x)))
    assert q == OP.Polynomial(list(c)).div_by_x_sub_value(x).coef
    c[0] = (c[0] + 1) % R
    K = common.load_pkg()
    with pytest.raises(K.KgsError, match="Polynomial does not divide"):
        ctx9.poly_div_x_sub(common.mont_bytes(c), bn.fr_to_bytes(x))


@pytest.mark.parametrize("case", GOLD["cases"],
                         ids=lambda c: f'{c["kind"]}-k{c["npols"]}-s{int(c["selected"])}-n{c["nbits"]}')
def test_golden_proofs(K, case):
    Fs, Ts, sF, sT = common.make_inputs(case["seed"], case["nbits"], case["npols"], case["selected"])
    assert common.inputs_digest(Fs, Ts, sF, sT) == case["inputs_sha256"]
    eF = [K.Evaluations(x) for x in Fs]
    eT = [K.Evaluations(x) for x in Ts]
    fn = K.grandsum_prover if case["kind"] == "grandsum" else K.grandproduct_prover
    proof = fn(common.oracle_ptau(11), eF if case["npols"] > 1 else eF[0], eT if case["npols"] > 1 else eT[0],
               K.Evaluations(sF) if sF else None, K.Evaluations(sT) if sT else None)
    got = {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}
    assert got == case["proof"]
    # the reference writes the Montgomery form back into the caller's objects (prover.js:147-148)
    for i in range(case["npols"]):
        vals = [int.from_bytes(Fs[i][32 * j:32 * j + 32], "little") for j in range(1 << case["nbits"])]
        assert eF[i].eval == common.mont_bytes(vals)


def test_pairing_verifies_gpu_proof(K):
    Fs, Ts, sF, sT = common.make_inputs(77, 4, 2, True)
    for kind, fn in (("grandsum", K.grandsum_prover), ("grandproduct", K.grandproduct_prover)):
        proof = fn(common.oracle_ptau(9), [K.Evaluations(x) for x in Fs], [K.Evaluations(x) for x in Ts],
                   K.Evaluations(sF), K.Evaluations(sT))
        assert P.verify(kind, common.oracle_ptau(9), proof, 4)


def test_error_paths(K):
    path = common.oracle_ptau(9)
    Fs, Ts, _, _ = common.make_inputs(5, 3, 1, False)
    Fs2, _, _, _ = common.make_inputs(6, 3, 1, False)
    with pytest.raises(ValueError, match="The grand-sum polynomial S is not well calculated"):
        K.grandsum_prover(path, K.Evaluations(Fs[0]), K.Evaluations(Fs2[0]))
    with pytest.raises(ValueError, match="The grand-product polynomial Z is not well calculated"):
        K.grandproduct_prover(path, K.Evaluations(Fs[0]), K.Evaluations(Fs2[0]))
    sel = common.mont_bytes([2] + [1] * 7)
    for fn in (K.grandsum_prover, K.grandproduct_prover):
        with pytest.raises(ValueError, match="Polynomial is not divisible"):
            fn(path, K.Evaluations(Fs[0]), K.Evaluations(Fs[0]), K.Evaluations(sel), K.Evaluations(sel))
    with pytest.raises(ValueError, match="Polynomial length must be a power of two."):
        K.grandsum_prover(path, K.Evaluations(Fs[0][:96]), K.Evaluations(Ts[0][:96]))
    big, bigT, _, _ = common.make_inputs(1, 10, 1, False)
    with pytest.raises(ValueError, match="not sufficiently large"):
        K.grandsum_prover(path, K.Evaluations(big[0]), K.Evaluations(bigT[0]))


def test_trivial_identity_multiset(K, monkeypatch):
    """F == T: S == 0 (grand-sum) / Z == 1; commitments of zero polynomials are infinity. The quotient
    is zero, on which the reference's divZh throws V8's RangeError (oracle quirk Q3,
    tests/test_gpu_quirks.py): so does the default (reference-identical) mode; the exact-math mode
    (KGS_REFERENCE_QUIRKS=0) proves it with the exact values (oracle quirks=False)."""
    from oracle import poly as OP
    Fs, _, _, _ = common.make_inputs(8, 3, 1, False)
    srs = P.SRS(common.oracle_ptau(9), common.tau())
    for kind, fn in (("grandsum", K.grandsum_prover), ("grandproduct", K.grandproduct_prover)):
        monkeypatch.delenv("KGS_REFERENCE_QUIRKS", raising=False)
        with pytest.raises(K.RangeError, match="offset is out of bounds"):
            fn(common.oracle_ptau(9), K.Evaluations(Fs[0]), K.Evaluations(Fs[0]))
        with pytest.raises(OP.JSRangeError, match="offset is out of bounds"):
            P.prove(kind, srs, P.EvalBuffer(Fs[0]), P.EvalBuffer(Fs[0]))
        monkeypatch.setenv("KGS_REFERENCE_QUIRKS", "0")
        got = fn(common.oracle_ptau(9), K.Evaluations(Fs[0]), K.Evaluations(Fs[0]))
        exp = P.prove(kind, srs, P.EvalBuffer(Fs[0]), P.EvalBuffer(Fs[0]), quirks=False)
        assert got == exp


def test_all_zero_selectors(K, monkeypatch):
    """selF = selT = 0 with F, T unrelated: trivially satisfied — the reference warns "The selection
    buffers are all zeros" (src/grandsum/mset_eq_kzg_prover.js:66-68); S = 0 and Z = 1, so several
    commitments are of constant polynomials and the quotient is zero, on which the reference's divZh
    then throws V8's RangeError (oracle quirk Q3) — and so does the default mode. Exact-math mode
    (KGS_REFERENCE_QUIRKS=0): byte-exact vs the oracle's exact values (quirks=False), verified."""
    from oracle import poly as OP
    ptau = common.oracle_ptau(9)
    srs = P.SRS(ptau, common.tau())
    Fs, _, _, _ = common.make_inputs(31, 4, 2, False)
    Ts, _, _, _ = common.make_inputs(32, 4, 2, False)
    zero = common.mont_bytes([0] * 16)
    for kind, fn, vf in (("grandsum", K.grandsum_prover, K.grandsum_verifier),
                         ("grandproduct", K.grandproduct_prover, K.grandproduct_verifier)):
        monkeypatch.delenv("KGS_REFERENCE_QUIRKS", raising=False)
        with pytest.raises(K.RangeError, match="offset is out of bounds"):
            fn(ptau, [K.Evaluations(x) for x in Fs], [K.Evaluations(x) for x in Ts], K.Evaluations(zero),
               K.Evaluations(zero))
        monkeypatch.setenv("KGS_REFERENCE_QUIRKS", "0")
        got = fn(ptau, [K.Evaluations(x) for x in Fs], [K.Evaluations(x) for x in Ts],
                 K.Evaluations(zero), K.Evaluations(zero))
        exp = P.prove(kind, srs, [P.EvalBuffer(x) for x in Fs], [P.EvalBuffer(x) for x in Ts],
                      P.EvalBuffer(zero), P.EvalBuffer(zero), quirks=False)
        assert got == exp
        assert vf(ptau, got, 4) is True
        with pytest.raises(OP.JSRangeError, match="offset is out of bounds"):
            P.prove(kind, srs, [P.EvalBuffer(x) for x in Fs], [P.EvalBuffer(x) for x in Ts],
                    P.EvalBuffer(zero), P.EvalBuffer(zero))


def _bary_eval(vals, nbits, x):
    """p(x) from evaluations on <w_n> (barycentric), O(n) with one batch inversion."""
    n = 1 << nbits
    w = bn.FR_W[nbits]
    dens, wi = [], 1
    ws = []
    for i in range(n):
        ws.append(wi)
        dens.append((x - wi) % R)
        wi = wi * w % R
    inv = OP.batch_inverse(dens)
    s = 0
    for i in range(n):
        s = (s + vals[i] * ws[i] % R * inv[i]) % R
    return (pow(x, n, R) - 1) * pow(n, R - 2, R) % R * s % R


@pytest.mark.parametrize("kind,nbits,npols,sel", [("grandsum", 16, 1, False), ("grandproduct", 16, 2, True),
                                                  ("grandsum", 20, 1, False)])
def test_large_proof_properties(K, kind, nbits, npols, sel):
    ctx = K.Context(0)
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    rnd = random.Random(nbits)
    n = 1 << nbits
    Fs, Ts, fvals = [], [], []
    for _ in range(npols):
        f = [rnd.getrandbits(253) for _ in range(n)]
        fvals.append(f)
        Fs.append(common.std_bytes(f))
        Ts.append(common.std_bytes([f[-1]] + f[:-1]))
    sF = sT = None
    if sel:
        a = [1] * n
        a[-1] = 0
        b = [1] * n
        b[0] = 0
        sF, sT = common.mont_bytes(a), common.mont_bytes(b)
    kk = K.GRANDSUM if kind == "grandsum" else K.GRANDPRODUCT
    coms, evs, _, _ = ctx.prove(kk, nbits, Fs, Ts, sF, sT, mont_out=False)
    cn, en = K.proof_names(kk, npols, sel)
    proof = {"commitments": dict(zip(cn, coms)), "evaluations": dict(zip(en, evs))}
    from oracle.ptau import PTau
    assert P.verify(kind, PTau(path), proof, nbits, tau=common.tau())
    # and with the native pairing verifier (kgs_verify_ptau), as the reference's verifier module does
    vf = K.grandsum_verifier if kind == "grandsum" else K.grandproduct_verifier
    assert vf(path, proof, nbits) is True
    # transcript-independent commitment: C(F0) == F0(tau) G1
    ftau = _bary_eval(fvals[0], nbits, common.tau())
    assert proof["commitments"]["F0" if npols > 1 else "F"] == bn.g1_to_lem(bn.g1_mul(bn.G1_GEN, ftau))
    # determinism
    coms2, evs2, _, _ = ctx.prove(kk, nbits, Fs, Ts, sF, sT, mont_out=False)
    assert coms2 == coms and evs2 == evs
    ctx.close()


@pytest.mark.parametrize("kind,nbits,npols,sel", [("grandsum", 14, 1, False), ("grandproduct", 14, 1, False),
                                                  ("grandsum", 13, 2, True), ("grandproduct", 13, 3, True)])
def test_mid_size_vs_c_oracle(K, kind, nbits, npols, sel):
    """Byte-for-byte against the C restatement at sizes the Python oracle is too slow for, in both
    context modes: two MSM lanes (one proof at a time; NTT passes built for 2 waves/SIMD) and one lane
    (proofs in flight; NTT passes built for 3 waves/SIMD, ntt.hip)."""
    from oracle import cbackend as C
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    Fs, Ts, sF, sT = common.make_inputs(nbits * 3 + npols, nbits, npols, sel)
    kk = K.GRANDSUM if kind == "grandsum" else K.GRANDPRODUCT
    _, srs = C.load_srs_bytes(path)
    ecoms, eevs = C.prove_raw(kk, nbits, Fs, Ts, sF, sT, srs, 0)
    for lanes in (2, 1):
        ctx.set_msm_lanes(lanes)
        coms, evs, _, _ = ctx.prove(kk, nbits, Fs, Ts, sF, sT, mont_out=False)
        assert coms == ecoms and evs == eevs, lanes
    ctx.close()


@pytest.mark.parametrize("which", ["all", "some"])
def test_caller_pinned_inputs(K, which):
    """Inputs the caller pinned with kgs_host_register are DMA'd in place ("all"); a mix of pinned
    and pageable inputs ("some") takes the staging path. Same bytes as the C restatement either way,
    and the Montgomery write-back is unchanged."""
    from oracle import cbackend as C
    nbits, npols = 13, 2  # 256 KiB vectors: each its own pages (registration is page-granular)
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    Fs, Ts, sF, sT = common.make_inputs(77, nbits, npols, True)
    bufs = [bytearray(x) for x in Fs + Ts + [sF, sT]]
    pinned = bufs if which == "all" else bufs[::2]
    handles = [K.host_register(b) for b in pinned]
    try:
        bF, bT = bufs[:npols], bufs[npols:2 * npols]
        coms, evs, mf, mt = ctx.prove(K.GRANDSUM, nbits, bF, bT, bufs[-2], bufs[-1])
        coms2, evs2, mf2, mt2 = ctx.prove(K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    finally:
        for h in handles:
            K.host_unregister(h)
    _, srs = C.load_srs_bytes(path)
    ecoms, eevs = C.prove_raw(K.GRANDSUM, nbits, Fs, Ts, sF, sT, srs, 0)
    assert coms == ecoms and evs == eevs
    assert coms2 == ecoms and evs2 == eevs
    assert mf == mf2 and mt == mt2
    assert [bytes(b) for b in bufs] == Fs + Ts + [sF, sT]  # inputs untouched
    ctx.close()


def test_failed_call_leaves_no_transfer_pending(K):
    """VERDICT r5 Next #1: a kgs_prove that fails after it has enqueued the DMAs of caller-pinned
    inputs (here: a domain larger than the loaded SRS, refused at the prover's start) returns with
    every stream of the context drained, so the caller may unregister and free its buffers at once;
    the context then proves normally (same bytes as the C restatement), and so does a new one."""
    from oracle import cbackend as C
    nbits = 13
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits - 1)  # SRS for domains up to 2^12 only
    Fs, Ts, sF, sT = common.make_inputs(78, nbits, 2, True)
    for rep in range(3):
        bufs = [bytearray(x) for x in Fs + Ts + [sF, sT]]
        outs = [bytearray(32 << nbits) for _ in range(4)]
        handles = [K.host_register(b) for b in bufs + outs]
        try:
            with pytest.raises(K.KgsError):
                ctx.prove(K.GRANDSUM, nbits, bufs[:2], bufs[2:4], bufs[4], bufs[5], mont_out=(outs[:2], outs[2:]))
            assert ctx.idle(), "a failed kgs_prove returned with transfers still pending"
        finally:
            for h in handles:
                K.host_unregister(h)
        del bufs, outs
    ctx.load_ptau(path, nbits)
    coms, evs, _, _ = ctx.prove(K.GRANDSUM, nbits, Fs, Ts, sF, sT)
    _, srs = C.load_srs_bytes(path)
    ecoms, eevs = C.prove_raw(K.GRANDSUM, nbits, Fs, Ts, sF, sT, srs, 0)
    assert coms == ecoms and evs == eevs
    assert ctx.idle()
    ctx.close()
    ctx2 = K.Context(0)
    ctx2.load_ptau(path, nbits)
    assert ctx2.prove(K.GRANDSUM, nbits, Fs, Ts, sF, sT, mont_out=False)[:2] == (ecoms, eevs)
    ctx2.close()


def _sharded_run(K, world, ptau, nbits, kind, Fs, Ts, sF, sT):
    """`world` contexts (one per simulated rank, all on cuda:0), one host thread each, MSMs
    point-range sharded through an in-process all-gather. Returns every rank's proof."""
    import threading
    grp = K.ThreadGroup(world)
    ctxs = [K.Context(0) for _ in range(world)]
    for r, c in enumerate(ctxs):
        c.load_ptau(ptau, nbits)
        c.set_shard(r, world, grp.allgather(r))
    out, err = [None] * world, [None] * world

    def run(r):
        try:
            out[r] = ctxs[r].prove(kind, nbits, Fs, Ts, sF, sT, mont_out=False)[:2]
        except Exception as e:  # pragma: no cover
            err[r] = e
            grp._bar.abort()
    th = [threading.Thread(target=run, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=300)
    for c in ctxs:
        c.close()
    assert not any(err), err
    return out


@pytest.mark.parametrize("kind,nbits,npols,sel,world", [("grandsum", 9, 1, False, 2), ("grandproduct", 9, 2, True, 3),
                                                        ("grandsum", 4, 1, True, 8)])
def test_sharded_prover_matches_golden_path(K, kind, nbits, npols, sel, world):
    """MSM point-range sharding (kgs_ctx_set_shard): every rank's proof equals the unsharded one."""
    ptau = common.oracle_ptau(max(nbits, 9))
    Fs, Ts, sF, sT = common.make_inputs(900 + nbits + world, nbits, npols, sel)
    kk = K.GRANDSUM if kind == "grandsum" else K.GRANDPRODUCT
    ctx = K.Context(0)
    ctx.load_ptau(ptau, nbits)
    want = ctx.prove(kk, nbits, Fs, Ts, sF, sT, mont_out=False)[:2]
    ctx.close()
    got = _sharded_run(K, world, ptau, nbits, kk, Fs, Ts, sF, sT)
    for r in range(world):
        assert got[r] == want, r


def test_sharded_prover_large(K):
    """2^16 grand-sum k=2, 2 ranks: sharded proof == unsharded proof, and it verifies."""
    nbits = 16
    path = f"/tmp/kgs_test_gpu_p{nbits}.ptau"
    ctx = K.Context(0)
    if not os.path.exists(path):
        ctx.write_synthetic_ptau(path, nbits, common.tau())
    ctx.load_ptau(path, nbits)
    Fs, Ts, sF, sT = common.make_inputs(4242, nbits, 2, False)
    want = ctx.prove(K.GRANDSUM, nbits, Fs, Ts, sF, sT, mont_out=False)[:2]
    ctx.close()
    got = _sharded_run(K, 2, path, nbits, K.GRANDSUM, Fs, Ts, sF, sT)
    assert got[0] == want and got[1] == want


def test_shard_callback_failure_is_reported(K):
    ctx = K.Context(0)
    ctx.load_ptau(common.oracle_ptau(9), 4)

    def bad(data):
        raise RuntimeError("transport down")
    ctx.set_shard(0, 2, bad)
    Fs, Ts, sF, sT = common.make_inputs(5, 4, 1, False)
    with pytest.raises(K.KgsError) as ei:
        ctx.prove(K.GRANDSUM, 4, Fs, Ts, sF, sT, mont_out=False)
    assert ei.value.code == -8
    ctx.set_shard(0, 1)
    ctx.prove(K.GRANDSUM, 4, Fs, Ts, sF, sT, mont_out=False)
    ctx.close()


def _gloo_prover_rank(rank, world, port, ptau, q):
    try:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
        K = common.load_pkg()
        ctx = K.Context(0)
        ctx.load_ptau(ptau, 10)
        ctx.set_shard(rank, world, K.torch_allgather())
        Fs, Ts, sF, sT = common.make_inputs(31337, 10, 2, True)
        coms, evs = ctx.prove(K.GRANDSUM, 10, Fs, Ts, sF, sT, mont_out=False)[:2]
        ctx.close()
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, coms, evs))
    except Exception as e:  # pragma: no cover
        q.put((rank, None, repr(e)))


def test_sharded_prover_two_processes(K):
    """one process per rank (as under torchrun), torch.distributed transport (gloo host tensors)"""
    import multiprocessing as mp
    import socket
    ptau = common.oracle_ptau(11)
    ctx = K.Context(0)
    ctx.load_ptau(ptau, 10)
    Fs, Ts, sF, sT = common.make_inputs(31337, 10, 2, True)
    want = ctx.prove(K.GRANDSUM, 10, Fs, Ts, sF, sT, mont_out=False)[:2]
    ctx.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    procs = [mpc.Process(target=_gloo_prover_rank, args=(r, 2, port, ptau, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    for rank, coms, evs in res:
        assert coms is not None, evs
        assert (coms, evs) == want, rank
