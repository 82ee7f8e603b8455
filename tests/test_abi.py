"""The C-ABI library (lib/libkgs.so) loads without a GPU and exports every symbol include/kgs.h
declares; host-only entry points (keccak) are exercised. No compute on a device here."""
import ctypes
import os
import re

import pytest

import common
from oracle.keccak import keccak256

HDR = os.path.join(common.ROOT, "include", "kgs.h")
LIB = os.path.join(common.ROOT, "kzg-grandsums-study_amd", "lib", "libkgs.so")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kgs_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(LIB)


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("kgs_ctx_create", "kgs_srs_load_ptau", "kgs_prove", "kgs_prove_device", "kgs_msm", "kgs_ntt",
              "kgs_grand_build", "kgs_poly_eval", "kgs_poly_div_x_sub", "kgs_keccak256"):
        assert s in syms


def test_every_declared_symbol_is_exported(lib):
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_keccak_via_abi(lib):
    f = lib.kgs_keccak256
    f.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    for msg in (b"", b"abc", bytes(range(256)) * 3):
        out = ctypes.create_string_buffer(32)
        assert f(msg, len(msg), out) == 0
        assert out.raw == keccak256(msg)


def test_proof_shape(lib):
    nc, ne = ctypes.c_int(), ctypes.c_int()
    lib.kgs_proof_shape(0, 3, 1, ctypes.byref(nc), ctypes.byref(ne))
    assert (nc.value, ne.value) == (2 * 3 + 2 + 4, 2 * 3 + 2 + 1)
    lib.kgs_proof_shape(1, 1, 0, ctypes.byref(nc), ctypes.byref(ne))
    assert (nc.value, ne.value) == (6, 2)


def test_python_mirror_names():
    K = common.load_pkg()
    com, ev = K.proof_names(K.GRANDSUM, 1, False)
    assert com == ["F", "T", "S", "Q", "Wxi", "Wxiw"] and ev == ["fxi", "txi", "sxiw"]
    com, ev = K.proof_names(K.GRANDPRODUCT, 2, True)
    assert com == ["F0", "T0", "F1", "T1", "selF", "selT", "Z", "Q", "Wxi", "Wxiw"]
    assert ev == ["f0xi", "f1xi", "selFxi", "selTxi", "zxiw"]


@pytest.mark.parametrize("length,span", [(1, 2 << 20), (1000, 2 << 20), (32 << 20, 2 << 20), ((32 << 20) + 77, 8 << 20),
                                         (3 << 20, 256 << 10), (5 << 20, 100)])
def test_stream_copy_spans_in_order(lib, length, span):
    """kgs_prove's staging copy (prover.cpp stream_copy, host only): every byte copied, every DMA span
    reported once, in address order, each only after all of its bytes were written."""
    import numpy as np
    rng = np.random.default_rng(length)
    src = rng.integers(0, 256, size=length, dtype=np.uint8)
    dst = np.zeros(length, dtype=np.uint8)
    span_eff = max(256 << 10, span // (256 << 10) * (256 << 10))
    nmax = (length + span_eff - 1) // span_eff
    spans = (ctypes.c_uint64 * max(nmax, 1))()
    n = ctypes.c_int()
    rc = lib.kgs_test_stream_copy(ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(src.ctypes.data),
                                  ctypes.c_uint64(length), ctypes.c_uint64(span), -1, spans, nmax, ctypes.byref(n))
    assert rc == 0
    assert np.array_equal(dst, src)
    assert n.value == nmax
    assert list(spans)[:nmax] == [i * span_eff for i in range(nmax)]


def test_stream_copy_failed_span_still_completes(lib):
    """A span whose DMA enqueue fails: the error is returned only after every piece is copied (the
    pool's helpers never write into the staging after the call), and no later span is reported."""
    import numpy as np
    length = 24 << 20
    src = np.arange(length, dtype=np.uint64).astype(np.uint8)
    dst = np.zeros(length, dtype=np.uint8)
    spans = (ctypes.c_uint64 * 16)()
    n = ctypes.c_int()
    rc = lib.kgs_test_stream_copy(ctypes.c_void_p(dst.ctypes.data), ctypes.c_void_p(src.ctypes.data),
                                  ctypes.c_uint64(length), ctypes.c_uint64(2 << 20), 3, spans, 16, ctypes.byref(n))
    assert rc != 0
    lib.kgs_last_error.restype = ctypes.c_char_p
    assert b"injected span failure" in lib.kgs_last_error()
    assert n.value == 3  # spans 0, 1, 2 reported; the failing one and the rest not
    assert np.array_equal(dst, src)
