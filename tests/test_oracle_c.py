"""The C restatement (oracle/c, used for large-n parity and as bench.py's cpu_baseline) agrees with
the Python oracle: every golden vector, keccak, and MSM vs the closed form."""
import ctypes
import json
import os
import random

import pytest

import common
from oracle import bn254 as bn
from oracle import cbackend as C
from oracle import protocol as P
from oracle.keccak import keccak256

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))


def test_keccak():
    out = ctypes.create_string_buffer(32)
    for m in (b"", b"abc", b"z" * 136, b"q" * 500):
        C.lib().orc_keccak256(m, len(m), out)
        assert out.raw == keccak256(m)


@pytest.mark.parametrize("logm", [0, 1, 2, 5, 8, 10])
def test_ntt_matches_python_oracle(logm):
    """oracle.c's transform (the checker of the GPU NTT at 2^18..2^22) against poly.ntt."""
    from oracle import poly as OP
    rnd = random.Random(logm)
    v = [rnd.randrange(bn.R) for _ in range(1 << logm)]
    for inverse in (False, True):
        assert C.ntt(common.mont_bytes(v), inverse) == common.mont_bytes(OP.ntt(v, inverse))


def test_msm_closed_form():
    _, srs = C.load_srs_bytes(common.oracle_ptau(9))
    o = P.SRS(common.oracle_ptau(9), common.tau())
    rnd = random.Random(4)
    for n in (1, 5, 100, 1023):
        v = [rnd.randrange(bn.R) for _ in range(n)]
        assert C.msm(srs, common.mont_bytes(v), 2) == bn.g1_to_lem(o.msm(v))


@pytest.mark.parametrize("case", GOLD["cases"],
                         ids=lambda c: f'{c["kind"]}-k{c["npols"]}-s{int(c["selected"])}-n{c["nbits"]}')
def test_c_oracle_matches_golden(case):
    _, srs = C.load_srs_bytes(common.oracle_ptau(11))
    K = common.load_pkg()
    kind = 0 if case["kind"] == "grandsum" else 1
    Fs, Ts, sF, sT = common.make_inputs(case["seed"], case["nbits"], case["npols"], case["selected"])
    coms, evs = C.prove_raw(kind, case["nbits"], Fs, Ts, sF, sT, srs, 2)
    cn, en = K.proof_names(kind, case["npols"], case["selected"])
    got = {"commitments": {k: v.hex() for k, v in zip(cn, coms)},
           "evaluations": {k: v.hex() for k, v in zip(en, evs)}}
    assert got == case["proof"]


def test_c_oracle_errors():
    _, srs = C.load_srs_bytes(common.oracle_ptau(6))
    Fs, Ts, _, _ = common.make_inputs(5, 3, 1, False)
    Fs2, _, _, _ = common.make_inputs(6, 3, 1, False)
    with pytest.raises(ValueError, match="not well calculated"):
        C.prove_raw(0, 3, Fs, Fs2, None, None, srs, 1)
    sel = common.mont_bytes([2] + [1] * 7)
    with pytest.raises(ValueError, match="Polynomial is not divisible"):
        C.prove_raw(1, 3, Fs, Fs, sel, sel, srs, 1)
