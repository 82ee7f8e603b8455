"""The oracle reproduces the committed golden vectors (tests/golden/golden.json, made by
tests/golden/gen_golden.py). The same vectors are the target of the GPU parity tests."""
import json
import os

import pytest

import common
from oracle import protocol as P

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def test_golden_ptau_pinned():
    assert int(GOLD["ptau"]["tau"]) == common.tau()


@pytest.mark.parametrize("case", [c for c in GOLD["cases"] if c["nbits"] <= 8],
                         ids=lambda c: f'{c["kind"]}-k{c["npols"]}-s{int(c["selected"])}-n{c["nbits"]}')
def test_oracle_matches_golden(case):
    srs = P.SRS(common.oracle_ptau(11), common.tau())
    Fs, Ts, sF, sT = common.make_inputs(case["seed"], case["nbits"], case["npols"], case["selected"])
    assert common.inputs_digest(Fs, Ts, sF, sT) == case["inputs_sha256"]
    eF = [P.EvalBuffer(x) for x in Fs]
    eT = [P.EvalBuffer(x) for x in Ts]
    proof = P.prove(case["kind"], srs, eF if case["npols"] > 1 else eF[0], eT if case["npols"] > 1 else eT[0],
                    P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None)
    got = {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}
    assert got == case["proof"]


@pytest.mark.parametrize("case", [c for c in GOLD["cases"] if c["nbits"] <= 8],
                         ids=lambda c: f'{c["kind"]}-k{c["npols"]}-s{int(c["selected"])}-n{c["nbits"]}')
def test_exact_semantics_match_golden(case):
    """The oracle's exact-value semantics (quirks=False: what the MI355X prover computes by default,
    DESIGN.md §4 "Reference quirks") give the reference's proof on every golden (non-degenerate) case."""
    srs = P.SRS(common.oracle_ptau(11), common.tau())
    Fs, Ts, sF, sT = common.make_inputs(case["seed"], case["nbits"], case["npols"], case["selected"])
    eF = [P.EvalBuffer(x) for x in Fs]
    eT = [P.EvalBuffer(x) for x in Ts]
    proof = P.prove(case["kind"], srs, eF if case["npols"] > 1 else eF[0], eT if case["npols"] > 1 else eT[0],
                    P.EvalBuffer(sF) if sF else None, P.EvalBuffer(sT) if sT else None, quirks=False)
    got = {sec: {k: v.hex() for k, v in proof[sec].items()} for sec in ("commitments", "evaluations")}
    assert got == case["proof"]
