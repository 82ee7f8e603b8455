"""Native verifiers (kgs_verify / kgs_verify_ptau: host C++ transcript replay + BN254 optimal-ate
pairing) against the reference-derived golden proofs, plus the rejection cases
the reference's verifiers have: a point off G1, an evaluation >= r, any altered commitment or
evaluation, and a proof checked against a different SRS. Host only (no GPU)."""
import json
import os
import shutil
import subprocess

import pytest

import common
from oracle import bn254 as O
from oracle import protocol as P

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
JS = os.path.join(common.ROOT, "kzg-grandsums-study_amd", "js")


def proof_of(case):
    return {sec: {k: bytes.fromhex(v) for k, v in case["proof"][sec].items()} for sec in ("commitments", "evaluations")}


def verifier(K, kind):
    return K.grandsum_verifier if kind == "grandsum" else K.grandproduct_verifier


@pytest.mark.parametrize("case", GOLD["cases"],
                         ids=lambda c: f'{c["kind"]}-k{c["npols"]}-s{int(c["selected"])}-n{c["nbits"]}')
def test_golden_proofs_verify(case):
    K = common.load_pkg()
    assert verifier(K, case["kind"])(common.oracle_ptau(11), proof_of(case), case["nbits"]) is True


def _pick(kind, npols, selected, nbits):
    for c in GOLD["cases"]:
        if (c["kind"], c["npols"], c["selected"], c["nbits"]) == (kind, npols, selected, nbits):
            return c
    raise KeyError


@pytest.mark.parametrize("kind", ["grandsum", "grandproduct"])
def test_tampering_is_rejected(kind):
    K = common.load_pkg()
    case = _pick(kind, 3, True, 5)
    ptau = common.oracle_ptau(11)
    vf = verifier(K, kind)
    good = proof_of(case)
    assert vf(ptau, good, 5)
    g1 = O.g1_to_lem(O.G1_GEN)
    for name in good["commitments"]:
        bad = {s: dict(v) for s, v in good.items()}
        bad["commitments"][name] = g1 if good["commitments"][name] != g1 else O.g1_to_lem(O.g1_mul(O.G1_GEN, 2))
        assert vf(ptau, bad, 5) is False, name
    for name in good["evaluations"]:
        bad = {s: dict(v) for s, v in good.items()}
        x = O.fr_from_bytes(good["evaluations"][name])
        bad["evaluations"][name] = O.fr_to_bytes((x + 1) % O.R)
        assert vf(ptau, bad, 5) is False, name
    # wrong domain size
    assert vf(ptau, good, 6) is False


def test_invalid_encodings_are_rejected():
    K = common.load_pkg()
    case = _pick("grandsum", 1, False, 3)
    ptau = common.oracle_ptau(11)
    good = proof_of(case)
    bad = {s: dict(v) for s, v in good.items()}
    bad["commitments"]["S"] = O.fq_to_bytes(1) + O.fq_to_bytes(3)  # (1, 3) is not on y^2 = x^3 + 3
    assert K.grandsum_verifier(ptau, bad, 3) is False
    bad = {s: dict(v) for s, v in good.items()}
    bad["evaluations"]["fxi"] = O.R.to_bytes(32, "little")  # not < r (valueBelongsToField)
    assert K.grandsum_verifier(ptau, bad, 3) is False
    bad = {s: dict(v) for s, v in good.items()}
    del bad["evaluations"]["sxiw"]
    assert K.grandsum_verifier(ptau, bad, 3) is False


def test_other_srs_rejects(tmp_path):
    """the same proof against [tau']_2 of another ceremony fails the pairing equation"""
    from oracle import ptau as PT
    K = common.load_pkg()
    case = _pick("grandproduct", 1, True, 8)
    other = str(tmp_path / "other.ptau")
    PT.write_synthetic_ptau(other, 9, (common.tau() + 1) % O.R)
    assert K.grandproduct_verifier(common.oracle_ptau(11), proof_of(case), 8)
    assert K.grandproduct_verifier(other, proof_of(case), 8) is False


def test_native_agrees_with_oracle_pairing():
    """one case through the oracle's own restated pairing (slow, pure Python) for an independent check"""
    K = common.load_pkg()
    case = _pick("grandsum", 3, True, 2)
    ptau = common.oracle_ptau(11)
    assert P.verify("grandsum", ptau, proof_of(case), 2) is True
    assert K.grandsum_verifier(ptau, proof_of(case), 2) is True
    bad = proof_of(case)
    bad["evaluations"]["sxiw"] = O.fr_to_bytes(7)
    assert P.verify("grandsum", ptau, bad, 2) is False
    assert K.grandsum_verifier(ptau, bad, 2) is False


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(os.path.join(JS, "build", "kgs_addon.node")),
                    reason="node or the N-API addon is missing")
def test_js_dropin_verifiers(tmp_path):
    cases = []
    for c in GOLD["cases"][::3]:
        cases.append({"kind": c["kind"], "nbits": c["nbits"], **c["proof"]})
        bad = json.loads(json.dumps(c["proof"]))
        k = next(iter(bad["evaluations"]))
        x = O.fr_from_bytes(bytes.fromhex(bad["evaluations"][k]))
        bad["evaluations"][k] = O.fr_to_bytes((x + 5) % O.R).hex()
        cases.append({"kind": c["kind"], "nbits": c["nbits"], **bad})
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"ptau": common.oracle_ptau(11), "cases": cases}))
    out = subprocess.run(["node", os.path.join(JS, "test", "verify_from_json.js"), str(spec)], capture_output=True,
                         text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    verdicts = json.loads(out.stdout)["verdicts"]
    assert verdicts == [True, False] * (len(cases) // 2)
