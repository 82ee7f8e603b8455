"""The drop-in provers' input checks with the reference's exact messages
(src/grandsum/mset_eq_kzg_prover.js:22-81; the grand-product prover has the same checks): through
the Python mirror and through the JavaScript modules. The checks run before any device work, so
this file needs no GPU."""
import json
import os
import shutil
import subprocess

import pytest

import common

JS = os.path.join(common.ROOT, "kzg-grandsums-study_amd", "js")
MESSAGES = [
    "The lengths of the two vector multisets must be the same.",
    "The number of multisets must be greater than 0.",
    "The 0-th multiset buffers must have the same length.",
    "The multiset buffers must all have the same length.",
    "The selection buffers must have the same length.",
    "The selection buffers must have the same length as the multiset buffers.",
    "Polynomial length must be a power of two.",
    "The Powers of Tau file is not sufficiently large to commit the polynomials.",
]


def _py_cases(K):
    ev = lambda n: K.Evaluations(common.std_bytes(list(range(1, n + 1))))  # noqa: E731
    one = lambda n: K.Evaluations(common.mont_bytes([1] * n))  # noqa: E731
    return [
        ([ev(8), ev(8)], [ev(8)], None, None),
        ([], [], None, None),
        (ev(8), ev(4), None, None),
        ([ev(8), ev(4)], [ev(8), ev(4)], None, None),
        (ev(8), ev(8), one(8), one(4)),
        (ev(8), ev(8), one(4), one(4)),
        (ev(6), ev(6), None, None),
        (ev(256), ev(256), None, None),
    ]


@pytest.mark.parametrize("kind", ["grandsum", "grandproduct", "lookup"])
def test_python_mirror_input_errors(kind):
    K = common.load_pkg()
    fn = {"grandsum": K.grandsum_prover, "grandproduct": K.grandproduct_prover, "lookup": K.lookup_prover}[kind]
    ptau = common.oracle_ptau(6)
    for (F, T, sF, sT), msg in zip(_py_cases(K), MESSAGES):
        if kind == "lookup" and sT is None:  # a lookup needs its multiplicities before anything else
            n = (F[0].length() if F else 8) if isinstance(F, list) else F.length()
            sT = K.Evaluations(common.mont_bytes([1] * n))
        with pytest.raises(ValueError) as e:
            fn(ptau, F, T, sF, sT)
        assert str(e.value) == msg


@pytest.mark.skipif(shutil.which("node") is None or not os.path.exists(os.path.join(JS, "build", "kgs_addon.node")),
                    reason="node or the N-API addon is missing")
def test_js_module_input_errors():
    out = subprocess.run(["node", os.path.join(JS, "test", "input_errors.js"), common.oracle_ptau(6)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    got = json.loads(out.stdout)
    for kind in ("grandsum", "grandproduct", "lookup"):
        assert got[kind] == MESSAGES, kind
