"""Executable specification of the distributed prover's data layouts (CPU, pure Python).

The multi-GPU prover (kgs_ctx_set_group, csrc/prover_dist.cpp + csrc/dist.hip) keeps every
vector distributed over W ranks in one of three layouts, for a vector of size N (M = N / W):
  BLOCK  : rank r holds natural indices [r M, (r+1) M)                       (H-evaluations, division)
  CYCLIC : rank r holds indices r + W j (j < N / W), for ANY length          (coefficients)
  E      : rank r holds k1 M + r (M / W) + t, k1 < W, t < M / W, stored as W blocks of M / W
           (block k1 at local offset k1 (M / W))                            (NTT-domain evaluations)
and moves between them with exactly one all-to-all each:
  forward DFT  CYCLIC -> E : local M-point DFT of the rank's cyclic slice, twiddle w_N^(n1 k2),
                             all-to-all by k2 chunk, W-point DFT over n1
  inverse DFT  E -> CYCLIC : W-point inverse DFT over k1, twiddle w_N^-(n1 k2), all-to-all,
                             local M-point inverse DFT (scaled by 1/N)
  BLOCK -> E               : all-to-all of contiguous M / W chunks, no arithmetic
  CYCLIC -> BLOCK          : all-to-all of contiguous N / W^2 chunks, interleaved on receipt
plus the cross-rank steps that are not all-to-alls: the builder's prefix scan (one all-gather of
rank totals), Horner on CYCLIC (one all-gather of 32 B per rank), synthetic division on BLOCK
(one all-gather of (R_lo, z^len) carries, Polynomial.divByXSubValue, polynomial.js:814-851).
This model is checked here against the oracle's NTT / division / scan on small sizes, and the HIP
implementation follows it index for index.
"""
import random

import pytest

import common  # noqa: F401  (sys.path)
from oracle import bn254 as bn
from oracle import poly as OP

R = bn.R


def w_(k):
    return bn.FR_W[k]


def dft(a, inverse=False):
    """natural-order DFT of a power-of-two length list (no 1/N for the inverse)"""
    n = len(a)
    k = n.bit_length() - 1
    w = w_(k) if not inverse else pow(w_(k), R - 2, R)
    return [sum(a[j] * pow(w, i * j, R) for j in range(n)) % R for i in range(n)]


# ------------------------------------------------------------------ layouts
def to_block(x, W):
    M = len(x) // W
    return [x[r * M:(r + 1) * M] for r in range(W)]


def to_cyclic(x, W):
    return [x[r::W] for r in range(W)]


def to_e(x, W):
    N = len(x)
    M = N // W
    b = M // W
    return [[x[k1 * M + r * b + t] for k1 in range(W) for t in range(b)] for r in range(W)]


def from_e(parts, W):
    N = sum(len(p) for p in parts)
    M = N // W
    b = M // W
    x = [0] * N
    for r in range(W):
        for k1 in range(W):
            for t in range(b):
                x[k1 * M + r * b + t] = parts[r][k1 * b + t]
    return x


def alltoall(send, W):
    """send[r] = W equal chunks (chunk j -> rank j); returns recv[r] = concat_j chunk r of rank j"""
    c = len(send[0]) // W
    return [sum((send[j][r * c:(r + 1) * c] for j in range(W)), []) for r in range(W)]


# ------------------------------------------------------------------ distributed DFTs
def fwd_cyclic_to_e(cyc, N, W, shift=1):
    """cyc[r] = rank r's cyclic slice (zero-padded to N / W); returns E parts of DFT(shift^i x_i)"""
    M = N // W
    b = M // W
    wN = w_(N.bit_length() - 1)
    send = []
    for n1 in range(W):
        xs = [(v * pow(shift, n1 + W * j, R)) % R for j, v in enumerate(cyc[n1])]
        xs += [0] * (M - len(xs))
        Z = dft(xs)  # local M-point DFT (w_M = w_N^W)
        Z = [Z[k2] * pow(wN, n1 * k2, R) % R for k2 in range(M)]  # twiddle
        send.append(Z)  # chunk j = k2 in [j b, (j+1) b)
    recv = alltoall(send, W)
    out = []
    for r in range(W):
        part = [0] * M
        for t in range(b):
            v = [recv[r][n1 * b + t] for n1 in range(W)]
            V = dft(v)  # W-point DFT over n1 (w_W = w_N^M)
            for k1 in range(W):
                part[k1 * b + t] = V[k1]
        out.append(part)
    return out


def inv_e_to_cyclic(parts, N, W, shift=1):
    """E parts of evaluations -> cyclic slices of (1/N) iDFT, divided by shift^i"""
    M = N // W
    b = M // W
    wNi = pow(w_(N.bit_length() - 1), R - 2, R)
    ninv = pow(N, R - 2, R)
    sinv = pow(shift, R - 2, R)
    send = []
    for r in range(W):
        s = [0] * M
        for t in range(b):
            k2 = r * b + t
            v = [parts[r][k1 * b + t] for k1 in range(W)]
            y = dft(v, inverse=True)
            for n1 in range(W):
                s[n1 * b + t] = y[n1] * pow(wNi, n1 * k2, R) % R
        send.append(s)
    recv = alltoall(send, W)  # rank n1: natural k2 order
    out = []
    for n1 in range(W):
        x = dft(recv[n1], inverse=True)
        out.append([x[n2] * ninv * pow(sinv, n1 + W * n2, R) % R for n2 in range(M)])
    return out


def block_to_e(blocks, W):
    return alltoall(blocks, W)


def cyclic_to_block(cyc, W):
    L = sum(len(c) for c in cyc)
    c2 = L // (W * W)
    recv = alltoall(cyc, W)
    out = []
    for d in range(W):
        loc = [0] * (L // W)
        for src in range(W):
            for t in range(c2):
                loc[src + W * t] = recv[d][src * c2 + t]
        out.append(loc)
    return out


def block_to_cyclic(blocks, W):
    """BLOCK -> CYCLIC (the openings before their commitment MSMs): rank r sends chunk d = its block's
    elements d + W t (global r M + d + W t, i.e. cyclic position r c2 + t of rank d); the received
    chunks in source order ARE the cyclic slice (prover_dist.cpp block_to_cyc, dist.hip k_pack_b2c)"""
    M = len(blocks[0])
    c2 = M // W
    send = [[blk[d + W * t] for d in range(W) for t in range(c2)] for blk in blocks]
    return alltoall(send, W)


# ------------------------------------------------------------------ tests
@pytest.mark.parametrize("W,logN", [(2, 3), (2, 5), (4, 4), (4, 6), (8, 6)])
def test_dft_roundtrip_matches_oracle(W, logN):
    rnd = random.Random(W * 100 + logN)
    N = 1 << logN
    x = [rnd.randrange(R) for _ in range(N)]
    # coefficients of half length (zero-padded, as the coset transforms of round 3), coset shift 5
    half = x[:N // 2] + [0] * (N // 2)
    cyc = [c[:(N // 2) // W] for c in to_cyclic(half, W)]
    E = fwd_cyclic_to_e(cyc, N, W, shift=5)
    assert from_e(E, W) == OP.ntt([v * pow(5, i, R) % R for i, v in enumerate(half)], False)
    back = inv_e_to_cyclic(E, N, W, shift=5)
    assert back == to_cyclic(half, W)
    # iNTT of H-evaluations given in BLOCK layout (round 2's S): BLOCK -> E -> CYCLIC
    Eb = block_to_e(to_block(x, W), W)
    assert Eb == to_e(x, W)
    assert inv_e_to_cyclic(Eb, N, W) == to_cyclic(OP.ntt(x, True), W)


@pytest.mark.parametrize("W,logL", [(2, 3), (4, 5), (8, 7)])
def test_cyclic_to_block(W, logL):
    rnd = random.Random(logL)
    L = 1 << logL
    x = [rnd.randrange(R) for _ in range(L)]
    assert cyclic_to_block(to_cyclic(x, W), W) == to_block(x, W)


@pytest.mark.parametrize("W,logL", [(2, 3), (4, 5), (8, 7), (8, 8)])
def test_block_to_cyclic(W, logL):
    rnd = random.Random(100 + logL)
    L = 1 << logL
    x = [rnd.randrange(R) for _ in range(L)]
    assert block_to_cyclic(to_block(x, W), W) == to_cyclic(x, W)
    assert cyclic_to_block(block_to_cyclic(to_block(x, W), W), W) == to_block(x, W)


def test_builder_scan_over_ranks():
    """S[i] = sum_{j<i} s_j from per-rank local scans + one all-gather of rank totals"""
    rnd = random.Random(7)
    W, N = 4, 32
    s = [rnd.randrange(R) for _ in range(N)]
    blocks = to_block(s, W)
    totals = [sum(b) % R for b in blocks]  # all-gathered
    got = []
    for r in range(W):
        off = sum(totals[:r]) % R
        acc = off
        for v in blocks[r]:
            got.append(acc)
            acc = (acc + v) % R
    assert got == [sum(s[:i]) % R for i in range(N)]


@pytest.mark.parametrize("W", [2, 4, 8])
def test_division_carries(W):
    """Polynomial.divByXSubValue on BLOCK slices: local recurrence with zero carry-in, one
    all-gather of (R_lo, z^len), carry fold from the top rank, fix-up q_j += z^(len-1-j) c"""
    rnd = random.Random(W)
    L = 8 * W
    z = rnd.randrange(R)
    q_true = [rnd.randrange(R) for _ in range(L - 1)]
    a = [0] * L  # a = (X - z) q_true, exactly divisible
    for i, c in enumerate(q_true):
        a[i + 1] = (a[i + 1] + c) % R
        a[i] = (a[i] - z * c) % R
    Lb = L // W
    blocks = to_block(a, W)
    loc, Rlo = [], []
    for blk in blocks:
        r_ = [0] * (Lb + 1)
        for i in range(Lb - 1, -1, -1):
            r_[i] = (blk[i] + z * r_[i + 1]) % R
        loc.append([r_[i + 1] for i in range(Lb)])  # q_loc[j] = R_{j+1} (R_Lb = 0)
        Rlo.append(r_[0])
    zl = pow(z, Lb, R)
    c = [0] * W
    for r in range(W - 1, 0, -1):
        c[r - 1] = (Rlo[r] + zl * c[r]) % R
    rem = (Rlo[0] + zl * c[0]) % R
    assert rem == 0
    q = []
    for r in range(W):
        q += [(loc[r][j] + pow(z, Lb - 1 - j, R) * c[r]) % R for j in range(Lb)]
    assert q[:L - 1] == q_true and q[L - 1] == 0


def test_horner_on_cyclic():
    rnd = random.Random(11)
    W, N = 4, 16
    c = [rnd.randrange(R) for _ in range(N)]
    x = rnd.randrange(R)
    parts = to_cyclic(c, W)
    xW = pow(x, W, R)
    v = [sum(cj * pow(xW, j, R) for j, cj in enumerate(p)) % R for p in parts]
    assert sum(pow(x, r, R) * v[r] for r in range(W)) % R == sum(ci * pow(x, i, R) for i, ci in enumerate(c)) % R
