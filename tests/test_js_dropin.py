"""The JavaScript drop-in modules (kzg-grandsums-study_amd/js: reference module API over the N-API
addon and libkgs.so). CPU: the addon loads in Node and its host-only entry (keccak) matches.
GPU: proofs made through the JS modules are byte-identical to the oracle's, the Montgomery
write-back happens, the reference's own test cases run, and error messages match."""
import json
import os
import shutil
import subprocess

import pytest

import common
from oracle import protocol as P
from oracle.keccak import keccak256

JS = os.path.join(common.ROOT, "kzg-grandsums-study_amd", "js")
ADDON = os.path.join(JS, "build", "kgs_addon.node")
NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def test_addon_loads_and_keccak():
    if not os.path.exists(ADDON):
        pytest.skip("addon not built")
    out = subprocess.check_output([NODE, "-e", f"const a=require({ADDON!r});"
                                   "process.stdout.write(Buffer.from(a.keccak256(Buffer.from('abc'))).toString('hex'))"])
    assert out.decode() == keccak256(b"abc").hex()


def test_curve_shim():
    out = subprocess.check_output([NODE, "-e", "require(%r).getCurveFromName('bn128').then(c=>{"
                                   "process.stdout.write(c.Fr.toString(c.Fr.w[28])+' '+Buffer.from(c.Fr.one).toString('hex'))})"
                                   % os.path.join(JS, "src", "curve.js")])
    w28, one = out.decode().split()
    assert int(w28) == 19103219067921713944291392827692070036145651957329286315305642004821462161904
    assert bytes.fromhex(one) == common.mont_bytes([1])


@pytest.mark.gpu
def test_js_proofs_match_oracle(tmp_path):
    ptau = common.oracle_ptau(9)
    srs = P.SRS(ptau, common.tau())
    cases, expect = [], []
    seed = 500
    for kind in ("grandsum", "grandproduct"):
        for npols, sel in ((1, False), (3, False), (1, True), (2, True)):
            nbits = 3 + npols
            Fs, Ts, sF, sT = common.make_inputs(seed, nbits, npols, sel)
            seed += 1
            cases.append({"kind": kind, "F": [x.hex() for x in Fs], "T": [x.hex() for x in Ts],
                          "selF": sF.hex() if sF else None, "selT": sT.hex() if sT else None})
            eF = [P.EvalBuffer(x) for x in Fs]
            eT = [P.EvalBuffer(x) for x in Ts]
            pr = P.prove(kind, srs, eF if npols > 1 else eF[0], eT if npols > 1 else eT[0],
                         P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None)
            expect.append(({sec: {k: v.hex() for k, v in pr[sec].items()} for sec in ("commitments", "evaluations")},
                           [e.eval.hex() for e in eF]))
    # error case: not a multiset
    Fs, _, _, _ = common.make_inputs(1, 3, 1, False)
    F2, _, _, _ = common.make_inputs(2, 3, 1, False)
    cases.append({"kind": "grandsum", "F": [Fs[0].hex()], "T": [F2[0].hex()], "selF": None, "selT": None})
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"ptau": ptau, "cases": cases}))
    out = json.loads(subprocess.check_output([NODE, os.path.join(JS, "test", "prove_from_json.js"), str(spec)],
                                             timeout=600))
    for got, (exp, mont) in zip(out["proofs"], expect):
        assert {"commitments": got["commitments"], "evaluations": got["evaluations"]} == exp
        assert got["montF"] == mont
        # key insertion order = the reference's
        assert list(got["commitments"]) == list(exp["commitments"])
    assert out["proofs"][-1]["error"] == "The grand-sum polynomial S is not well calculated"


@pytest.mark.gpu
def test_js_concurrent_provers_match_oracle(tmp_path):
    """12 prover() Promises in flight at once (Promise.all), grand-sum and grand-product mixed, 1-3
    vectors, with and without selectors, two domain sizes: every proof byte-identical to the oracle
    (the reference's provers are independent async calls, src/grandsum/mset_eq_kzg_prover.js:12)."""
    ptau = common.oracle_ptau(9)
    srs = P.SRS(ptau, common.tau())
    cases, expect = [], []
    for i in range(12):
        kind = "grandsum" if i % 2 == 0 else "grandproduct"
        npols, sel, nbits = 1 + i % 3, i % 4 >= 2, 5 + (i % 5 == 0) * 2
        Fs, Ts, sF, sT = common.make_inputs(7000 + i, nbits, npols, sel)
        cases.append({"kind": kind, "F": [x.hex() for x in Fs], "T": [x.hex() for x in Ts],
                      "selF": sF.hex() if sF else None, "selT": sT.hex() if sT else None})
        eF = [P.EvalBuffer(x) for x in Fs]
        eT = [P.EvalBuffer(x) for x in Ts]
        pr = P.prove(kind, srs, eF if npols > 1 else eF[0], eT if npols > 1 else eT[0],
                     P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None)
        expect.append({sec: {k: v.hex() for k, v in pr[sec].items()} for sec in ("commitments", "evaluations")})
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"ptau": ptau, "cases": cases, "concurrent": True}))
    env = dict(os.environ, KGS_JS_CONTEXTS="4")
    out = json.loads(subprocess.check_output([NODE, os.path.join(JS, "test", "prove_from_json.js"), str(spec)],
                                             timeout=600, env=env))
    for i, (got, exp) in enumerate(zip(out["proofs"], expect)):
        assert "error" not in got, (i, got)
        assert {"commitments": got["commitments"], "evaluations": got["evaluations"]} == exp, i
    # the calls really overlapped: the pool grew to its capacity
    assert out["pool"]["contexts"] == 4 and out["pool"]["waiting"] == 0


@pytest.mark.gpu
def test_reference_style_cases():
    out = subprocess.check_output([NODE, os.path.join(JS, "test", "reference_style.test.js"), common.oracle_ptau(9)],
                                  timeout=600)
    assert b"reference-style cases passed: 8" in out
