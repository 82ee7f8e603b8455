"""CPU checks of the 29-bit twiddle product of the NTT passes (kzg-grandsums-study_amd/csrc/fr29.hpp):
its constants, and mul29's exact CIOS row schedule run on Python integers — every 64-bit column
accumulator below 2^64 at every step, the result congruent to a * w * 2^-261 mod r and below 2r (the
[0, 2p) contract of the lazy butterflies it replaces, ntt.hip), for a < 2^256 (the DIF differences go
in unreduced, < 4p) and twiddle records of canonical w * 2^261 mod r.

The GPU side (bit-identical transforms 2^0..2^22, every proof) is covered by test_gpu_parity.py."""
import os
import random
import re

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
MASK = (1 << 29) - 1
HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "kzg-grandsums-study_amd", "csrc", "fr29.hpp")


def _hdr():
    with open(HDR) as fh:
        return fh.read()


def _arr(name, text):
    m = re.search(r"%s\[\d+\]\s*=\s*\{([^}]*)\}" % re.escape(name), text)
    assert m, name
    return [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",") if x.strip()]


def _const(name, text):
    return int(re.search(r"%s = (0x[0-9a-f]+)u" % re.escape(name), text).group(1), 16)


T = _hdr()
P = _arr("P", T)
INV, INV32 = _const("INV", T), _const("INV32", T)


def test_constants():
    assert sum(p << (29 * j) for j, p in enumerate(P)) == R
    assert all(p <= MASK for p in P)
    assert (R * INV) % (1 << 29) == MASK                      # -r^-1 mod 2^29
    assert (P[0] * INV32) % (1 << 32) == (1 << 32) - 1        # -P[0]^-1 mod 2^32
    assert R % (1 << 28) == 1 and INV == INV32 == (1 << 28) - 1
    c32 = _arr("C32", T)
    assert sum(w << (32 * i) for i, w in enumerate(c32)) == (32 << 256) % R
    tm = _arr("TO_MONT", T)  # k_to_mont's record: mul29(x, TO_MONT) = x * 2^256
    assert all(x <= MASK for x in tm) and sum(x << (29 * j) for j, x in enumerate(tm)) == pow(2, 517, R)


def unpack(x):
    return [(x >> (29 * j)) & MASK for j in range(8)] + [x >> 232]


def mul29(a, w):
    """fr29.hpp mul29 step by step; returns (result value, largest accumulator seen)"""
    al, wl = unpack(a), unpack(w)
    t, worst = [0] * 9, 0
    for i in range(9):
        for j in range(9):
            t[j] += al[i] * wl[j]
        worst = max(worst, max(t))
        if i < 8:
            m = (t[0] * INV32) % (1 << 32)
            u = m * P[0] + t[0]
            assert u % (1 << 32) == 0
            for j in range(1, 9):
                t[j] += m * P[j]
            worst = max(worst, u, max(t))
            t = t[1:] + [0]
            t[0] += (u >> 32) * 8
        else:
            m = (t[0] * INV) & MASK
            u = m * P[0] + t[0]
            assert u % (1 << 29) == 0
            for j in range(1, 9):
                t[j] += m * P[j]
            worst = max(worst, u, max(t))
            t = t[1:] + [0]
            t[0] += u >> 29
        worst = max(worst, max(t))
    val = sum(x << (29 * j) for j, x in enumerate(t))
    return val, worst


def check(a, w):
    v, worst = mul29(a, w)
    assert worst < (1 << 64), "column overflow"
    assert v % R == a * w * pow(2, -261, R) % R
    assert v < 2 * R
    return worst


def test_row_schedule_extremes_and_random():
    rnd = random.Random(29)
    wmax = R - 1
    worst = 0
    cases = [((1 << 256) - 1, wmax), (4 * R - 1, wmax), (2 * R - 1, wmax), (0, wmax), ((1 << 256) - 1, 0),
             ((1 << 256) - 1, (1 << 254) % R)]
    # limb-wise maxima: every limb of a at 2^29 - 1 below 2^256, w with maximal low limbs below r
    cases.append((sum(MASK << (29 * j) for j in range(8)) + (((1 << 24) - 1) << 232), wmax))
    for _ in range(3000):
        a = rnd.randrange(1 << 256) if rnd.random() < 0.5 else rnd.randrange(4 * R)
        cases.append((a, rnd.randrange(R)))
    for a, w in cases:
        worst = max(worst, check(a, w))
    assert worst < (1 << 64)


def test_column_bound_analysis():
    """worst case over ALL inputs: per-limb maxima (a < 2^256: limbs < 2^29, the top < 2^24; w < r)"""
    amax = [MASK] * 8 + [(1 << 24) - 1]
    wmax = [MASK] * 8 + [R >> 232]
    t, worst = [0] * 9, 0
    for i in range(9):
        for j in range(9):
            t[j] += amax[i] * wmax[j]
        mbits = 32 if i < 8 else 29
        m = (1 << mbits) - 1
        u = m * P[0] + t[0]
        for j in range(1, 9):
            t[j] += m * P[j]
        worst = max(worst, u, max(t))
        t = t[1:] + [0]
        t[0] += u >> mbits
    assert worst < (1 << 64) and worst < 1.1 * (1 << 63), worst  # < 2^63.14: the header's bound
    # value bound: (a w + M r) / 2^261 with M < 2^261 (1 + 2^-25) (32-bit m in rows 0..7)
    out = ((1 << 256) * (R - 1) >> 261) + R + (R >> 25) + 1
    assert out < 2 * R
