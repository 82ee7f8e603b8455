"""The CPU oracle's prove -> verify round trips (all 4 variants x 2 arguments), input-check error
messages (mset_eq_kzg_prover.js:22-81) and the semantic failure paths, plus closed-form vs
Pippenger commitment consistency. Pure Python, no GPU."""
import random

import pytest

import common
from oracle import bn254 as bn
from oracle import protocol as P

R = bn.R


@pytest.fixture(scope="module")
def srs6():
    return P.SRS(common.oracle_ptau(6), common.tau())


def _prove(kind, srs, nbits, npols, selected, seed=7):
    Fs, Ts, sF, sT = common.make_inputs(seed, nbits, npols, selected)
    eF = [P.EvalBuffer(x) for x in Fs]
    eT = [P.EvalBuffer(x) for x in Ts]
    return P.prove(kind, srs, eF if npols > 1 else eF[0], eT if npols > 1 else eT[0],
                   P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None), eF, eT, Fs


@pytest.mark.parametrize("kind", ["grandsum", "grandproduct"])
@pytest.mark.parametrize("npols,selected", [(1, False), (3, False), (1, True), (2, True)])
def test_prove_verify_trapdoor(srs6, kind, npols, selected):
    for nbits in (1, 3, 5):
        proof, _, _, _ = _prove(kind, srs6, nbits, npols, selected, seed=nbits)
        assert P.verify(kind, srs6.ptau, proof, nbits, tau=common.tau())


@pytest.mark.parametrize("kind", ["grandsum", "grandproduct"])
def test_prove_verify_pairing(srs6, kind):
    proof, _, _, _ = _prove(kind, srs6, 2, 2, True)
    assert P.verify(kind, srs6.ptau, proof, 2)
    # tamper: swap two commitments -> fails
    com = dict(proof["commitments"])
    com["Wxi"], com["Wxiw"] = com["Wxiw"], com["Wxi"]
    assert not P.verify(kind, srs6.ptau, {"commitments": com, "evaluations": proof["evaluations"]}, 2)


def test_tampered_evaluation_fails(srs6):
    proof, _, _, _ = _prove("grandsum", srs6, 3, 1, False)
    ev = dict(proof["evaluations"])
    ev["sxiw"] = bn.fr_to_bytes((bn.fr_from_bytes(ev["sxiw"]) + 1) % R)
    assert not P.verify("grandsum", srs6.ptau, {"commitments": proof["commitments"], "evaluations": ev}, 3,
                        tau=common.tau())


def test_montgomery_side_effect(srs6):
    _, eF, eT, Fs = _prove("grandsum", srs6, 3, 1, False)
    vals = [int.from_bytes(Fs[0][32 * i:32 * i + 32], "little") for i in range(8)]
    assert eF[0].eval == common.mont_bytes(vals)


def test_closed_form_equals_pippenger():
    srs_cf = P.SRS(common.oracle_ptau(6), common.tau())
    srs_pp = P.SRS(common.oracle_ptau(6), None)
    rnd = random.Random(5)
    for n in (1, 7, 64, 127):
        sc = [rnd.randrange(R) for _ in range(n)]
        assert srs_cf.msm(sc) == srs_pp.msm(sc)


def test_input_errors(srs6):
    Fs, Ts, _, _ = common.make_inputs(1, 3, 2, False)
    E = P.EvalBuffer
    with pytest.raises(ValueError, match="The lengths of the two vector multisets must be the same."):
        P.prove("grandsum", srs6, [E(Fs[0]), E(Fs[1])], [E(Ts[0])])
    with pytest.raises(ValueError, match="The number of multisets must be greater than 0."):
        P.prove("grandsum", srs6, [], [])
    with pytest.raises(ValueError, match="The 0-th multiset buffers must have the same length."):
        P.prove("grandsum", srs6, E(Fs[0]), E(Ts[0][:64]))
    with pytest.raises(ValueError, match="Polynomial length must be a power of two."):
        P.prove("grandsum", srs6, E(Fs[0][:96]), E(Ts[0][:96]))
    big, bigT, _, _ = common.make_inputs(1, 7, 1, False)
    with pytest.raises(ValueError, match="not sufficiently large"):
        P.prove("grandsum", srs6, E(big[0]), E(bigT[0]))


@pytest.mark.parametrize("kind,msg", [("grandsum", "The grand-sum polynomial S is not well calculated"),
                                      ("grandproduct", "The grand-product polynomial Z is not well calculated")])
def test_not_a_multiset(srs6, kind, msg):
    Fs, _, _, _ = common.make_inputs(2, 3, 1, False)
    Ts2, _, _, _ = common.make_inputs(3, 3, 1, False)
    with pytest.raises(ValueError, match=msg):
        P.prove(kind, srs6, P.EvalBuffer(Fs[0]), P.EvalBuffer(Ts2[0]))


@pytest.mark.parametrize("kind", ["grandsum", "grandproduct"])
def test_non_binary_selector_not_divisible(srs6, kind):
    n = 8
    f = [random.Random(9).randrange(R) for _ in range(n)]
    # F == T elementwise: the multiset check passes for any selector; selector value 2 breaks the
    # binary constraint -> divZh throws (polynomial.js:878)
    sel = [2] + [1] * (n - 1)
    with pytest.raises(ValueError, match="Polynomial is not divisible"):
        P.prove(kind, srs6, P.EvalBuffer(common.std_bytes(f)), P.EvalBuffer(common.std_bytes(f)),
                P.EvalBuffer(common.mont_bytes(sel)), P.EvalBuffer(common.mont_bytes(sel)))


def test_reference_quirks_on_degenerate_multisets(srs6):
    """oracle/poly.py Q1-Q3: F = w^i (degree 1) makes the reference's multiply
    mis-sized, F == T gives a zero quotient; the exact semantics prove both and the proofs verify."""
    from oracle import poly as OP
    nb, n = 3, 8
    w = bn.FR_W[nb]
    f = [pow(w, i, R) for i in range(n)]
    rot = [f[-1]] + f[:-1]
    cases = [("grandsum", f, rot, "Polynomial is not divisible"), ("grandproduct", f, rot, "Polynomial does not divide"),
             ("grandsum", f, f, None), ("grandproduct", f, f, None)]
    for kind, fv, tv, msg in cases:
        def args():  # fresh buffers: the prover writes the Montgomery form back into them
            return (kind, srs6, P.EvalBuffer(common.std_bytes(fv)), P.EvalBuffer(common.std_bytes(tv)))
        if msg is None:
            with pytest.raises(OP.JSRangeError, match="offset is out of bounds"):
                P.prove(*args())
        else:
            with pytest.raises(ValueError, match=msg):
                P.prove(*args())
        proof = P.prove(*args(), quirks=False)
        assert P.verify(kind, srs6.ptau, proof, nb, tau=common.tau())
