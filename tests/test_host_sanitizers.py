"""CPU sanitizer tests of the host code that parses untrusted bytes.

tests/native builds the product's host-only units — ptau_io.cpp (ptau header + section table:
readBinFile / readPTauHeader, src/ptau_utils.js:3-24) and verifier.cpp with host_field.hpp /
host_pairing.hpp (kgs_verify on proof bytes: src/grandsum/mset_eq_kzg_verifier.js:9-313) — under
AddressSanitizer + UndefinedBehaviorSanitizer (-fno-sanitize-recover: any report aborts), and drives
them with malformed ptau files (truncated at every structural boundary, bad magic / version /
section sizes / n8 / curve / header size / power, missing sections) and malformed proofs (off-curve
points, coordinates >= q, evaluations >= r, wrong statement), plus a seeded random fuzz loop.
Every case must end with a clean exit and the expected verdict.
"""
import json
import os
import shutil
import struct
import subprocess

import pytest

import common

NATIVE = os.path.join(common.ROOT, "tests", "native")
EXE = os.path.join(NATIVE, "build", "host_check_asan")
GOLD = json.load(open(os.path.join(common.ROOT, "tests", "golden", "golden.json")))


@pytest.fixture(scope="module")
def exe():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.check_call(["make", "-s", "-C", NATIVE])
    return EXE


def run(exe, *args):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=86",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=87")
    p = subprocess.run([exe, *map(str, args)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, (args, p.returncode, p.stderr[-3000:])
    assert "Sanitizer" not in p.stderr and "runtime error" not in p.stderr, p.stderr[-3000:]
    return p.stdout


def ptau_bytes():
    return open(common.oracle_ptau(3), "rb").read()


def sections(d):
    """[(id, payload_pos, size)] of a well-formed ptau"""
    n = struct.unpack_from("<I", d, 8)[0]
    out, pos = [], 12
    for _ in range(n):
        sid, size = struct.unpack_from("<IQ", d, pos)
        out.append((sid, pos + 12, size))
        pos += 12 + size
    return out


def malformed_ptaus():
    d = ptau_bytes()
    secs = sections(d)
    s1 = [s for s in secs if s[0] == 1][0]
    s2 = [s for s in secs if s[0] == 2][0]
    s3 = [s for s in secs if s[0] == 3][0]
    cases = {}
    # truncation at every structural boundary (and one byte either side)
    cuts = {0, 3, 4, 8, 11, 12, 13, 23, s1[1] - 1, s1[1], s1[1] + 4, s1[1] + 36, s1[1] + 43, s2[1] - 12,
            s2[1], s2[1] + 64, s3[1] - 12, s3[1], s3[1] + 128, s3[1] + 255}
    for c in sorted(cuts):
        cases[f"trunc{c}"] = d[:c]
    b = bytearray(d)
    b[0:4] = b"ptaX"
    cases["magic"] = bytes(b)
    b = bytearray(d)
    struct.pack_into("<I", b, 4, 2)
    cases["version"] = bytes(b)
    b = bytearray(d)
    struct.pack_into("<I", b, 8, 0xFFFFFFFF)
    cases["nsections_huge"] = bytes(b)
    b = bytearray(d)
    struct.pack_into("<I", b, 8, 0)
    cases["nsections_zero"] = bytes(b)
    for name, val in (("size_max", 2**64 - 1), ("size_wrap", 2**64 - 12), ("size_big", 1 << 40)):
        b = bytearray(d)
        struct.pack_into("<Q", b, 16, val)  # first section's size
        cases[name] = bytes(b)
    b = bytearray(d)
    struct.pack_into("<Q", b, s1[1] - 8, 45)
    cases["header_size"] = bytes(b)
    b = bytearray(d)
    struct.pack_into("<I", b, s1[1], 48)
    cases["n8_48"] = bytes(b)
    b = bytearray(d)
    b[s1[1] + 4] ^= 1
    cases["curve_q"] = bytes(b)
    for name, pw in (("power_0", 0), ("power_64", 64), ("power_huge", 0xFFFFFFFF)):
        b = bytearray(d)
        struct.pack_into("<I", b, s1[1] + 36, pw)
        cases[name] = bytes(b)
    # second header section appended
    b = bytearray(d) + struct.pack("<IQ", 1, 44) + d[s1[1]:s1[1] + 44]
    struct.pack_into("<I", b, 8, struct.unpack_from("<I", d, 8)[0] + 1)
    cases["two_headers"] = bytes(b)
    # tauG2 section shorter than 2 points
    b = bytearray(d[:s3[1] - 12]) + struct.pack("<IQ", 3, 100) + bytes(100)
    cases["g2_short"] = bytes(b)
    return cases


def test_malformed_ptau_files(exe, tmp_path):
    good = run(exe, "ptau", common.oracle_ptau(3)).split("\n")
    assert good[0] == "power 0 3" and good[1].startswith("g2 0 ")
    for name, data in malformed_ptaus().items():
        p = tmp_path / f"{name}.ptau"
        p.write_bytes(data)
        out = run(exe, "ptau", p).split("\n")
        rc_power = int(out[0].split()[1])
        rc_g2 = int(out[1].split()[1])
        # every malformed file is rejected by the header parser or, if the header is intact but a
        # later section is short, by the tauG2 reader
        assert rc_power < 0 or rc_g2 < 0, (name, out)


def _proof_bin(case):
    K = common.load_pkg()
    kind = K.GRANDSUM if case["kind"] == "grandsum" else K.GRANDPRODUCT
    cn, en = K.proof_names(kind, case["npols"], case["selected"])
    pr = case["proof"]
    com = b"".join(bytes.fromhex(pr["commitments"][n]) for n in cn)
    ev = b"".join(bytes.fromhex(pr["evaluations"][n]) for n in en)
    return kind, com, ev


@pytest.mark.parametrize("idx", [0, 7, 13, 30, 47])
def test_malformed_proofs(exe, tmp_path, idx):
    from oracle import bn254 as bn
    case = GOLD["cases"][idx]
    kind, com, ev = _proof_bin(case)
    ptau = common.oracle_ptau(11)
    args = [kind, case["nbits"], case["npols"], int(case["selected"]), ptau]

    def verdict(c, e):
        p = tmp_path / "proof.bin"
        p.write_bytes(c + e)
        return run(exe, "verify", *args, p).strip()
    assert verdict(com, ev) == "verify 1"
    q = bn.Q.to_bytes(32, "little")
    r = bn.R.to_bytes(32, "little")
    bad = []
    c = bytearray(com)
    c[5] ^= 0x40  # x no longer on the curve
    bad.append((bytes(c), ev))
    c = bytearray(com)
    c[0:32] = q  # coordinate == q (non-canonical)
    bad.append((bytes(c), ev))
    c = bytearray(com)
    c[32:64] = b"\xff" * 32  # y >= q
    bad.append((bytes(c), ev))
    e = bytearray(ev)
    e[0:32] = r  # evaluation == r
    bad.append((com, bytes(e)))
    e = bytearray(ev)
    e[-32:] = b"\xff" * 32  # evaluation >= r
    bad.append((com, bytes(e)))
    e = bytearray(ev)
    e[0] ^= 1  # a valid encoding of the wrong value: the pairing check fails
    bad.append((com, bytes(e)))
    c = bytearray(com)
    c[-64:] = bytes(64)  # Wxiw = infinity: valid point, wrong proof
    bad.append((bytes(c), ev))
    for c, e in bad:
        assert verdict(c, e) == "verify 0"
    # a proof checked against a statement of another shape
    p = tmp_path / "proof.bin"
    p.write_bytes(com + ev)
    assert run(exe, "verify", kind, case["nbits"], case["npols"] + 1, int(case["selected"]), ptau, p).strip() \
        == "shape-mismatch"
    assert run(exe, "verify", kind, 0, case["npols"], int(case["selected"]), ptau, p).strip() == "verify -1"
    assert run(exe, "verify", kind, 29, case["npols"], int(case["selected"]), ptau, p).strip() == "verify -1"


def test_fuzz(exe):
    out = run(exe, "fuzz", 20261016, 4000, common.oracle_ptau(3))
    assert "fuzz done iters 4000 accepted 0" in out
