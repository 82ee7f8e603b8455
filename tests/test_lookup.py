"""Lookup argument (include/kgs.h KGS_LOOKUP): the selected grand-sum with the
table's multiplicities in selT and no binary constraint on them.

The reference has no lookup prover: test/lookup_kzg_grandsum.test.js:24-111 is commented out, and
its "standard lookup" case calls the grand-sum prover with (F, T, ones, multiplicities), which the
grand-sum's selT-binary constraint (prover.js:241-244) rejects. Parity is therefore against the
oracle's restatement (oracle/protocol.py prove("lookup"), oracle/c orc_prove kind 2) and the
committed vectors in tests/golden/lookup.json (gen_golden.py --lookup): "parity unpinned" against
the reference itself. Soundness-side checks: honest lookups verify (trapdoor and pairing), proofs
fail the grand-sum verifier, and every way of breaking the lookup relation is refused with the
grand-sum's messages.
"""
import json
import os

import numpy as np
import pytest

import common
from oracle import bn254 as bn
from oracle import protocol as P

R = bn.R
HERE = os.path.dirname(os.path.abspath(__file__))
LOOK = json.load(open(os.path.join(HERE, "golden", "lookup.json")))


def case_id(c):
    return f'{c["gen"]}-k{c["npols"]}-u{c["unselected"]}-n{c["nbits"]}'


def case_inputs(c):
    if c["gen"] == "reference_standard":
        return common.reference_standard_lookup(c["seed"], c["nbits"])
    if c["gen"] == "dup_table":
        return common.lookup_dup_table(c["seed"], c["nbits"])
    if c["gen"] == "all_zero":
        return common.lookup_all_zero(c["seed"], c["nbits"])
    return common.make_lookup_inputs(c["seed"], c["nbits"], c["npols"], c["unselected"])


def hexproof(proof):
    return {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}


def unhex(case):
    return {sec: {k: bytes.fromhex(v) for k, v in case["proof"][sec].items()} for sec in ("commitments", "evaluations")}


def oracle_prove(kind, srs, Fs, Ts, sF, sT):
    eF = [P.EvalBuffer(x) for x in Fs]
    eT = [P.EvalBuffer(x) for x in Ts]
    return P.prove(kind, srs, eF if len(Fs) > 1 else eF[0], eT if len(Ts) > 1 else eT[0],
                   P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None)


@pytest.fixture(scope="module")
def srs11():
    return P.SRS(common.oracle_ptau(11), common.tau())


# ------------------------------------------------------------------ CPU: oracle and host verifier
@pytest.mark.parametrize("case", [c for c in LOOK["cases"] if c["nbits"] <= 5], ids=case_id)
def test_oracle_reproduces_lookup_vectors(srs11, case):
    Fs, Ts, sF, sM = case_inputs(case)
    assert common.inputs_digest(Fs, Ts, sF, sM) == case["inputs_sha256"]
    assert hexproof(oracle_prove("lookup", srs11, Fs, Ts, sF, sM)) == case["proof"]


@pytest.mark.parametrize("case", LOOK["cases"], ids=case_id)
def test_c_oracle_matches_lookup_vectors(case):
    from oracle import cbackend as C
    Fs, Ts, sF, sM = case_inputs(case)
    _, srs = C.load_srs_bytes(common.oracle_ptau(11))
    coms, evs = C.prove_raw(2, case["nbits"], Fs, Ts, sF, sM, srs, 0)
    K = common.load_pkg()
    cn, en = K.proof_names(K.LOOKUP, case["npols"], True)
    assert {"commitments": {k: v.hex() for k, v in zip(cn, coms)},
            "evaluations": {k: v.hex() for k, v in zip(en, evs)}} == case["proof"]


@pytest.mark.parametrize("case", LOOK["cases"], ids=case_id)
def test_native_lookup_verifier(case):
    """kgs_verify_ptau(KGS_LOOKUP): host transcript replay + optimal-ate pairing. Lookup proofs with
    a multiplicity outside {0, 1} must fail the grand-sum verifier (its r0 keeps selT - selT^2)."""
    K = common.load_pkg()
    ptau = common.oracle_ptau(11)
    proof = unhex(case)
    assert K.lookup_verifier(ptau, proof, case["nbits"]) is True
    _, _, _, sM = case_inputs(case)
    m = [bn.fr_from_bytes(sM[32 * i:32 * i + 32]) for i in range(len(sM) // 32)]
    if any(x not in (0, 1) for x in m):
        assert K.grandsum_verifier(ptau, proof, case["nbits"]) is False
        assert P.verify("grandsum", ptau, proof, case["nbits"], tau=common.tau()) is False


def test_lookup_tampering_rejected():
    K = common.load_pkg()
    case = next(c for c in LOOK["cases"] if c["npols"] == 3 and c["nbits"] == 5)
    ptau = common.oracle_ptau(11)
    good = unhex(case)
    for sec in ("commitments", "evaluations"):
        for name in good[sec]:
            bad = {s: dict(v) for s, v in good.items()}
            if sec == "commitments":
                bad[sec][name] = bn.g1_to_lem(bn.g1_mul(bn.G1_GEN, 3))
            else:
                bad[sec][name] = bn.fr_to_bytes((bn.fr_from_bytes(good[sec][name]) + 1) % R)
            assert K.lookup_verifier(ptau, bad, 5) is False, name
    # a lookup proof always carries the selectors
    stripped = {s: {k: v for k, v in good[s].items() if not k.startswith("sel")} for s in good}
    assert K.lookup_verifier(ptau, stripped, 5) is False
    assert P.verify("lookup", ptau, stripped, 5, tau=common.tau()) is False


def test_reference_standard_lookup_pairing(srs11):
    """The reference's own (commented-out) case, checked with the restated optimal-ate pairing."""
    Fs, Ts, sF, sM = common.reference_standard_lookup()
    proof = oracle_prove("lookup", srs11, Fs, Ts, sF, sM)
    assert P.verify("lookup", srs11.ptau, proof, 2)
    # the reference's grand-sum prover refuses it: multiplicity 3 breaks selT's binary constraint
    with pytest.raises(ValueError, match="Polynomial is not divisible"):
        oracle_prove("grandsum", srs11, Fs, Ts, sF, sM)


def lookup_failures(nbits=4, seed=41):
    """(inputs, expected message) for every way to break the lookup relation"""
    Fs, Ts, sF, sM = common.make_lookup_inputs(seed, nbits, 1, 1)
    n = 1 << nbits
    f = [int.from_bytes(Fs[0][32 * i:32 * i + 32], "little") for i in range(n)]
    m = [bn.fr_from_bytes(sM[32 * i:32 * i + 32]) for i in range(n)]
    sel = [bn.fr_from_bytes(sF[32 * i:32 * i + 32]) for i in range(n)]
    i_on = sel.index(1)
    out = []
    # a selected f value that is not in the table
    f2 = list(f)
    f2[i_on] = (f2[i_on] + 1) % R
    out.append(((([common.std_bytes(f2)], Ts, sF, sM)), "The grand-sum polynomial S is not well calculated"))
    # a wrong multiplicity
    m2 = list(m)
    j = m2.index(max(m2))
    m2[j] -= 1
    out.append((((Fs, Ts, sF, common.mont_bytes(m2))), "The grand-sum polynomial S is not well calculated"))
    # a non-binary selF (the multiplicities adjusted so that the sums still agree)
    sel3 = list(sel)
    sel3[i_on] = 2
    tv = [int.from_bytes(Ts[0][32 * i:32 * i + 32], "little") for i in range(n)]
    m3 = list(m)
    m3[tv.index(f[i_on])] += 1
    out.append((((Fs, Ts, common.mont_bytes(sel3), common.mont_bytes(m3))), "Polynomial is not divisible"))
    return out


def test_lookup_failures_oracle(srs11):
    for (Fs, Ts, sF, sM), msg in lookup_failures():
        with pytest.raises(ValueError, match=msg):
            oracle_prove("lookup", srs11, Fs, Ts, sF, sM)
    from oracle import cbackend as C
    _, srs = C.load_srs_bytes(common.oracle_ptau(11))
    for (Fs, Ts, sF, sM), msg in lookup_failures():
        with pytest.raises(ValueError, match=msg):
            C.prove_raw(2, 4, Fs, Ts, sF, sM, srs, 0)
    Fs, Ts, _, _ = common.make_lookup_inputs(5, 3, 1)
    with pytest.raises(ValueError, match="A lookup needs the multiplicities of the table."):
        P.prove("lookup", srs11, P.EvalBuffer(Fs[0]), P.EvalBuffer(Ts[0]))


def test_all_ones_lookup_keeps_selectors(srs11):
    """F == T with multiplicities all one: the grand-sum drops all-one selectors (prover.js:63-68),
    the lookup keeps them (its proof layout always has selF / selT)."""
    Fs, _, _, _ = common.make_inputs(12, 3, 1, False)
    ones = common.mont_bytes([1] * 8)
    proof = oracle_prove("lookup", srs11, Fs, Fs, ones, ones)
    assert "selF" in proof["commitments"] and "selTxi" in proof["evaluations"]
    assert P.verify("lookup", srs11.ptau, proof, 3, tau=common.tau())


# ------------------------------------------------------------------ GPU: the HIP path
@pytest.mark.gpu
@pytest.mark.parametrize("case", LOOK["cases"], ids=case_id)
def test_gpu_lookup_golden(case):
    K = common.load_pkg()
    Fs, Ts, sF, sM = case_inputs(case)
    eF = [K.Evaluations(x) for x in Fs]
    eT = [K.Evaluations(x) for x in Ts]
    proof = K.lookup_prover(common.oracle_ptau(11), eF if case["npols"] > 1 else eF[0],
                            eT if case["npols"] > 1 else eT[0], K.Evaluations(sF), K.Evaluations(sM))
    assert hexproof(proof) == case["proof"]


@pytest.mark.gpu
def test_gpu_lookup_failures():
    K = common.load_pkg()
    ptau = common.oracle_ptau(11)
    E = K.Evaluations
    for (Fs, Ts, sF, sM), msg in lookup_failures():
        with pytest.raises(ValueError, match=msg):
            K.lookup_prover(ptau, E(Fs[0]), E(Ts[0]), E(sF), E(sM))
    Fs, Ts, sF, sM = common.reference_standard_lookup()
    with pytest.raises(ValueError, match="Polynomial is not divisible"):
        K.grandsum_prover(ptau, E(Fs[0]), E(Ts[0]), E(sF), E(sM))
    with pytest.raises(ValueError, match="A lookup needs the multiplicities of the table."):
        K.lookup_prover(ptau, E(Fs[0]), E(Ts[0]))
    # the C-ABI refuses a lookup without selectors and an unknown kind
    ctx = K.Context(0)
    ctx.load_ptau(ptau, 2)
    with pytest.raises(K.KgsError, match="a lookup needs both selectors"):
        ctx.prove(K.LOOKUP, 2, Fs, Ts, None, None, mont_out=False)
    with pytest.raises(K.KgsError, match="unknown argument kind"):
        ctx.prove(7, 2, Fs, Ts, None, None, mont_out=False)
    ctx.close()


def np_lookup_inputs(seed, nbits, npols, unselected):
    """make_lookup_inputs' shapes with numpy (2^20 rows in about a second)."""
    n = 1 << nbits
    rng = np.random.Generator(np.random.PCG64(seed))
    Ts = []
    for _ in range(npols):
        w = rng.integers(0, np.iinfo(np.uint64).max, size=(n, 4), dtype=np.uint64, endpoint=True)
        w[:, 3] &= np.uint64((1 << 61) - 1)
        Ts.append(np.ascontiguousarray(w).view(np.uint8).reshape(n, 32))
    rows = rng.integers(0, n, size=n)
    sel = np.ones(n, dtype=np.int64)
    sel[rng.choice(n, size=unselected, replace=False)] = 0
    m = np.bincount(rows, weights=sel, minlength=n).astype(np.int64)
    mont = np.frombuffer(common.mont_bytes(range(int(m.max()) + 1)), dtype=np.uint8).reshape(-1, 32)
    Fs = [t[rows].tobytes() for t in Ts]
    return (Fs, [t.tobytes() for t in Ts], mont[sel].tobytes(), mont[m].tobytes(), rows, sel, m)


@pytest.mark.gpu
@pytest.mark.parametrize("nbits,npols,unselected", [(13, 2, 100), (14, 1, 0)])
def test_gpu_lookup_mid_size_vs_c_oracle(nbits, npols, unselected):
    from oracle import cbackend as C
    from test_gpu_configs import gpu_ptau
    K = common.load_pkg()
    path = gpu_ptau(K, nbits)
    Fs, Ts, sF, sM, _, _, _ = np_lookup_inputs(nbits * 7 + npols, nbits, npols, unselected)
    ctx = K.Context(0)
    ctx.load_ptau(path, nbits)
    got = ctx.prove(K.LOOKUP, nbits, Fs, Ts, sF, sM, mont_out=False)[:2]
    ctx.close()
    _, srs = C.load_srs_bytes(path)
    assert got == tuple(C.prove_raw(2, nbits, Fs, Ts, sF, sM, srs, 0))


@pytest.mark.gpu
def test_gpu_lookup_large_properties():
    """2^20 rows: the proof verifies (trapdoor + native pairing), fails as a grand-sum proof,
    C(selT) is the multiplicities' closed form m(tau) G1, and the prover is deterministic."""
    from test_gpu_configs import gpu_ptau
    from test_gpu_parity import _bary_eval
    K = common.load_pkg()
    nbits = 20
    path = gpu_ptau(K, nbits)
    Fs, Ts, sF, sM, rows, sel, m = np_lookup_inputs(20, nbits, 1, 1000)
    ctx = K.Context(0)
    ctx.load_ptau(path, nbits)
    coms, evs = ctx.prove(K.LOOKUP, nbits, Fs, Ts, sF, sM, mont_out=False)[:2]
    cn, en = K.proof_names(K.LOOKUP, 1, True)
    proof = {"commitments": dict(zip(cn, coms)), "evaluations": dict(zip(en, evs))}
    from oracle.ptau import PTau
    assert P.verify("lookup", PTau(path), proof, nbits, tau=common.tau())
    assert K.lookup_verifier(path, proof, nbits) is True
    assert K.grandsum_verifier(path, proof, nbits) is False
    mtau = _bary_eval([int(x) for x in m], nbits, common.tau())
    assert proof["commitments"]["selT"] == bn.g1_to_lem(bn.g1_mul(bn.G1_GEN, mtau))
    assert ctx.prove(K.LOOKUP, nbits, Fs, Ts, sF, sM, mont_out=False)[:2] == (coms, evs)
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("world,nbits,npols", [(2, 9, 1), (4, 12, 2)])
def test_gpu_lookup_distributed(world, nbits, npols):
    """The distributed prover (local group) proves lookups byte-identically to one GPU."""
    from test_gpu_configs import gpu_ptau
    from test_gpu_dist import run_group, single
    K = common.load_pkg()
    ptau = gpu_ptau(K, max(nbits, 9))
    Fs, Ts, sF, sM, _, _, _ = np_lookup_inputs(300 + world, nbits, npols, 7)
    want = single(K, ptau, K.LOOKUP, nbits, Fs, Ts, sF, sM)
    g = K.Group.local(world)
    got, err = run_group(K, g, world, ptau, K.LOOKUP, nbits, Fs, Ts, sF, sM)
    g.close()
    assert not any(err), err
    for r in range(world):
        assert got[r] == want, r


# ------------------------------------------------------------------ JavaScript drop-in modules
JS = os.path.join(common.ROOT, "kzg-grandsums-study_amd", "js")
_HAVE_NODE = __import__("shutil").which("node") is not None and os.path.exists(
    os.path.join(JS, "build", "kgs_addon.node"))


@pytest.mark.skipif(not _HAVE_NODE, reason="node or the N-API addon is missing")
def test_js_lookup_verifier(tmp_path):
    """lookup_kzg_grandsum_verifier (host only): the golden lookup proofs verify, a tampered one
    does not, and the grand-sum verifier module refuses a lookup proof."""
    import subprocess
    cases = []
    for c in LOOK["cases"][::2]:
        cases.append({"kind": "lookup", "nbits": c["nbits"], **c["proof"]})
        bad = json.loads(json.dumps(c["proof"]))
        bad["evaluations"]["sxiw"] = bn.fr_to_bytes((bn.fr_from_bytes(bytes.fromhex(bad["evaluations"]["sxiw"])) + 1)
                                                    % R).hex()
        cases.append({"kind": "lookup", "nbits": c["nbits"], **bad})
    ref = LOOK["cases"][0]  # the reference's standard lookup: multiplicity 3
    cases.append({"kind": "grandsum", "nbits": ref["nbits"], **ref["proof"]})
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"ptau": common.oracle_ptau(11), "cases": cases}))
    out = subprocess.run(["node", os.path.join(JS, "test", "verify_from_json.js"), str(spec)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert json.loads(out.stdout)["verdicts"] == [True, False] * ((len(cases) - 1) // 2) + [False]


@pytest.mark.gpu
@pytest.mark.skipif(not _HAVE_NODE, reason="node or the N-API addon is missing")
def test_js_lookup_prover(tmp_path):
    """lookup_kzg_grandsum_prover through N-API: byte-identical to the golden lookup proofs, the
    proof object keeps the grand-sum's key order, and a broken lookup gives the grand-sum message."""
    import subprocess
    picks = [c for c in LOOK["cases"] if c["nbits"] <= 5][::2]
    cases = []
    for c in picks:
        Fs, Ts, sF, sM = case_inputs(c)
        cases.append({"kind": "lookup", "F": [x.hex() for x in Fs], "T": [x.hex() for x in Ts],
                      "selF": sF.hex(), "selT": sM.hex()})
    (Fs, Ts, sF, sM), msg = lookup_failures()[0]
    cases.append({"kind": "lookup", "F": [x.hex() for x in Fs], "T": [x.hex() for x in Ts],
                  "selF": sF.hex(), "selT": sM.hex()})
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"ptau": common.oracle_ptau(11), "cases": cases}))
    out = json.loads(subprocess.check_output(["node", os.path.join(JS, "test", "prove_from_json.js"), str(spec)],
                                             timeout=600))
    for got, c in zip(out["proofs"], picks):
        assert {"commitments": got["commitments"], "evaluations": got["evaluations"]} == c["proof"]
        assert list(got["commitments"])[-6:] == ["selF", "selT", "S", "Q", "Wxi", "Wxiw"]
    assert out["proofs"][-1]["error"] == msg
