"""GPU: a proof through the Python mirror with the "kgs" logger at INFO writes the reference's log
(prover.js:13-140,164-412) with the oracle's challenges, and all-zero selectors raise the
reference's warning (prover.js:66-68)."""
import logging

import pytest

import common
from oracle import protocol as P


@pytest.mark.gpu
def test_python_prover_log_lines(caplog):
    K = common.load_pkg()
    ptau = common.oracle_ptau(9)
    srs = P.SRS(ptau, common.tau())
    Fs, Ts, sF, sT = common.make_inputs(8300, 5, 2, True)
    tr = {}
    P.prove("grandsum", srs, [P.EvalBuffer(x) for x in Fs], [P.EvalBuffer(x) for x in Ts], P.EvalBuffer(sF),
            P.EvalBuffer(sT), trace=tr)
    with caplog.at_level(logging.INFO, logger="kgs"):
        K.grandsum_prover(ptau, [K.Evaluations(x) for x in Fs], [K.Evaluations(x) for x in Ts], K.Evaluations(sF),
                          K.Evaluations(sT))
    lines = [r.getMessage() for r in caplog.records if r.name == "kgs"]
    assert lines[0] == "> MULTISET EQUALITY KZG GRAND-SUM PROVER STARTED"
    assert "  Domain size: 32" in lines and "  Number of polynomials: 2" in lines and "  Selectors: Yes" in lines
    assert lines[-1] == "> MULTISET EQUALITY KZG GRAND-SUM PROVER FINISHED"
    ch = tr["challenges"]
    for name, sym in (("beta", "𝛃"), ("gamma", "𝜸"), ("alpha", "𝜶"), ("xi", "𝔷")):
        assert f"···      {sym}  = {ch[name]}" in lines, name
    caplog.clear()
    zero = bytes(32 * 32)
    # (the warning comes first; then, like the reference's divZh on the zero quotient, the default
    # reference-identical mode throws RangeError)
    with caplog.at_level(logging.WARNING, logger="kgs"), pytest.raises(K.RangeError, match="offset is out of bounds"):
        K.grandsum_prover(ptau, K.Evaluations(Fs[0]), K.Evaluations(Ts[0]), K.Evaluations(zero), K.Evaluations(zero))
    msgs = [r.getMessage() for r in caplog.records if r.name == "kgs"]
    assert msgs == ["The selection buffers are all zeros. The argument is trivially satisfied."]
