"""CPU checks of the 9 x 29-bit Fq representation used by the MSM bucket accumulation
(kzg-grandsums-study_amd/csrc/field29.hpp): its constants, and the interval analysis that proves
no limb, column or value overflow in g1_acc29::add_aff for the exact multiples of q it uses.

The GPU side is covered by the MSM / prover parity tests in test_gpu_parity.py (bit-exact
commitments); this file pins the arithmetic argument those tests rely on.
"""
import math
import os
import re


Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
MASK = (1 << 29) - 1
RBITS = 261
HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "kzg-grandsums-study_amd", "csrc", "field29.hpp")


def _hdr():
    with open(HDR) as fh:
        return fh.read()


def _words(name, text):
    m = re.search(r"%s\s*=\s*\{\{?([^}]*)\}" % re.escape(name), text)
    assert m, name
    return [int(x.strip().rstrip("u"), 16) for x in m.group(1).split(",") if x.strip()]


def _d29(ws):
    return sum(w << (29 * j) for j, w in enumerate(ws))


def _d32(ws):
    return sum(w << (32 * j) for j, w in enumerate(ws))


def test_constants():
    t = _hdr()
    assert _d29(_words("L9 Q", t)) == Q
    assert all(w <= MASK for w in _words("L9 Q", t))
    assert _d29(_words("L9 ONE", t)) == pow(2, 261, Q)
    assert _d29(_words("L9 C256", t)) == pow(2, 256, Q)
    assert _d29(_words("L9 C266", t)) == pow(2, 266, Q)
    assert _d32(_words("C261W[8]", t)) == pow(2, 261, Q)
    inv = int(re.search(r"INV = (0x[0-9a-f]+)u", t).group(1), 16)
    assert (Q * inv) % (1 << 29) == (1 << 29) - 1  # -q^-1 mod 2^29
    inv32 = int(re.search(r"INV32 = (0x[0-9a-f]+)u", t).group(1), 16)
    q0 = _words("L9 Q", t)[0]
    assert (q0 * inv32) % (1 << 32) == (1 << 32) - 1  # -q0^-1 mod 2^32 (reduce_row32)
    assert inv32 % (1 << 29) == inv


def _spread(k, s):
    K = k * Q
    d = [(K >> (29 * j)) & MASK for j in range(8)] + [K >> 232]
    out = [d[0] + (s << 29)] + [d[j] + (s << 29) - s for j in range(1, 8)] + [d[8] - s]
    assert sum(x << (29 * j) for j, x in enumerate(out)) == K
    assert all(0 <= x < (1 << 32) for x in out)
    return out


class V:
    """value < val, every limb <= limb (val may be refined per limb by the top limb bound)"""

    def __init__(self, val, limb):
        self.val, self.limb = val, limb

    def limb_max(self, j):
        return min(self.limb, (self.val - 1) >> (29 * j)) if j == 8 else self.limb


QL = [(Q >> (29 * j)) & MASK for j in range(8)] + [Q >> 232]


def _m32_rows():
    """KGS_M32_ROWS / KGS_M32_ROWS_MUL2 of the header: CIOS rows that take reduce_row32's 32-bit m"""
    t = _hdr()
    return (int(re.search(r"#define KGS_M32_ROWS (\d+)", t).group(1)),
            int(re.search(r"#define KGS_M32_ROWS_MUL2 (\d+)", t).group(1)))


def _col_bounds(rows, m32):
    """upper bounds of the CIOS column accumulators: rows(i) -> [(column, max product)] added in row
    i; rows < m32 reduce with m < 2^32 (reduce_row32), the others with m < 2^29. Returns (largest
    accumulator value at any point, largest output column)."""
    t, worst = [0] * 9, 0
    for i in range(9):
        for j, p in rows(i):
            t[j] += p
        m = (1 << (32 if i < m32 else 29)) - 1
        u = m * QL[0] + t[0]
        worst = max(worst, u, max(t))
        for j in range(1, 9):
            t[j] += m * QL[j]
        worst = max(worst, max(t))
        t = t[1:] + [0]
        t[0] += u >> 29
    return worst, max(t)


def _limbs_max(a):
    return [a.limb_max(j) for j in range(9)]


def _out(s):
    # (s + M q) / 2^261 with M = sum m_i 2^(29 i): m_i < 2^32 in rows 0..7 add < 2^-25 q
    out = (s >> RBITS) + Q + (Q >> 25) + 1
    assert out <= (1 << RBITS)
    return V(out, MASK)


def _mul(a, b, fused=False):
    al, bl = _limbs_max(a), _limbs_max(b)
    worst, outc = _col_bounds(lambda i: [(j, al[i] * bl[j]) for j in range(9)], _m32_rows()[0])
    assert worst < (1 << 64), "column overflow %.3f" % math.log2(worst)
    if fused:
        _fused(outc)
    return _out(a.val * b.val)


def _sqr(a, fused=False):  # fq29::sqr: row i adds a_i^2 at column 2i and 2 a_i a_j at i + j
    al = _limbs_max(a)
    worst, outc = _col_bounds(lambda i: [(i, al[i] * al[i])] + [(j, 2 * al[i] * al[j]) for j in range(i + 1, 9)],
                              _m32_rows()[0])
    assert worst < (1 << 64), "column overflow %.3f" % math.log2(worst)
    if fused:
        _fused(outc)
    return _out(a.val * a.val)


def _mul2(a, b, c, d):  # fq29::mul2: (a*b + c*d) / 2^261, one reduction
    al, bl, cl, dl = _limbs_max(a), _limbs_max(b), _limbs_max(c), _limbs_max(d)
    worst, _ = _col_bounds(lambda i: [(j, al[i] * bl[j] + cl[i] * dl[j]) for j in range(9)], _m32_rows()[1])
    assert worst < (1 << 64), "column overflow %.3f" % math.log2(worst)
    s = a.val * b.val + c.val * d.val
    assert s < (1 << RBITS) * ((1 << RBITS) - Q)
    return _out(s)


def _fused(cols_bound):
    """carry_sub folds a product's carry pass into a difference: its columns are read as int64"""
    assert cols_bound < (1 << 63), "signed column overflow %.3f" % math.log2(cols_bound)


def _mul_cols(a, b):
    return _mul(a, b, fused=True)


def _sqr_cols(a):
    return _sqr(a, fused=True)


def _add(a, b):
    return V(a.val + b.val, a.limb + b.limb)


def _sub(a, b, k, s):  # a + K - b, K = spread(k, s)
    K = _spread(k, s)
    for j in range(9):
        assert K[j] >= b.limb_max(j), (k, s, j)
    return V(a.val + k * Q, max(a.limb + K[j] for j in range(9)))


def _neg(b, k, s):
    return _sub(V(0, 0), b, k, s)


def _norm(a):
    assert a.val <= (1 << RBITS) and a.limb + 8 < (1 << 32)
    return V(a.val, MASK)


def madd_bound(vb):
    """g1_acc29::add_aff step by step (same k, s as the header); returns the output bound"""
    X1 = Y1 = ZZ1 = ZZZ1 = V(vb, MASK)
    x2 = y2 = V(Q, MASK)
    U2, S2 = _mul_cols(x2, ZZ1), _mul(y2, ZZZ1)
    P = _norm(_sub(U2, X1, 30, 1))            # carry_sub<30, 1>
    Rb = _neg(Y1, 32, 2)                      # K - Y1, then +- S2
    for j in range(9):                        # the negated branch: K_j - Y1_j - S2_j >= 0
        assert _spread(32, 2)[j] >= Y1.limb_max(j) + S2.limb_max(j)
    R = _norm(V(Rb.val + S2.val, Rb.limb + S2.limb))
    PP = _sqr(P)
    assert PP.val <= 8 * Q                    # maybe_zero8's candidate set covers PP
    PPP, Qv, R2 = _mul(P, PP), _mul(X1, PP), _sqr_cols(R)
    nX = _norm(_sub(R2, _add(PPP, _add(Qv, Qv)), 16, 3))
    T = _sub(Qv, nX, 64, 1)
    Y3 = _mul2(R, T, Y1, _neg(PPP, 3, 1))     # R*T + Y1*(3q - PPP)
    ZZ3, ZZZ3 = _mul(ZZ1, PP), _mul(ZZZ1, PPP)
    # the raw-record conversion (to_fq) and the rare-path checks multiply by C256 < q
    for c in (P, R, nX, Y3, ZZ3, ZZZ3):
        assert _mul(c, V(Q, MASK)).val <= 2 * Q
    return max(nX.val, Y3.val, ZZ3.val, ZZZ3.val)


def add_bound(vb):
    """g1_acc29::add (accumulator + accumulator, the combine / bit-sum trees) step by step"""
    X1 = Y1 = ZZ1 = ZZZ1 = X2 = Y2 = ZZ2 = ZZZ2 = V(vb, MASK)
    U1, U2, S1, S2 = _mul(X1, ZZ2), _mul_cols(X2, ZZ1), _mul(Y1, ZZZ2), _mul_cols(Y2, ZZZ1)
    P = _norm(_sub(U2, U1, 8, 1))
    R = _norm(_sub(S2, S1, 8, 1))
    PP = _sqr(P)
    assert PP.val <= 8 * Q                    # maybe_zero8's candidate set covers PP
    PPP = _mul(P, PP)
    ZZ3 = _mul(_mul(ZZ1, ZZ2), PP)
    ZZZ3 = _mul(_mul(ZZZ1, ZZZ2), PPP)
    Qv = _mul(U1, PP)
    R2 = _sqr_cols(R)
    nX = _norm(_sub(R2, _add(PPP, _add(Qv, Qv)), 16, 3))
    T = _sub(Qv, nX, 64, 1)
    Y3 = _mul2(R, T, S1, _neg(PPP, 3, 1))
    for c in (P, R, nX, Y3, ZZ3, ZZZ3):
        assert _mul(c, V(Q, MASK)).val <= 2 * Q
    return max(nX.val, Y3.val, ZZ3.val, ZZZ3.val)


def test_full_add_bounds():
    # the tree adds take two accumulators from the bucket chains (< vb) and must stay below vb;
    # from_xyzz (doubling path) yields < 2q
    vb = 2 * Q
    for _ in range(50):
        nxt = max(madd_bound(vb), vb)
        if nxt == vb:
            break
        vb = nxt
    assert add_bound(vb) <= vb
    assert 2 * Q <= vb


def test_add_aff_bounds_fixed_point():
    # initial accumulator: a table point (< q) with ZZ = ZZZ = 2^261 mod q; negated y: 2q - y
    vb = 2 * Q
    for _ in range(50):
        nxt = max(madd_bound(vb), vb)
        if nxt == vb:
            break
        vb = nxt
    assert madd_bound(vb) <= vb
    assert math.log2(vb) < 258.6  # field29.hpp: coordinates < 2^258.6


def test_spread_constants_used_by_header():
    t = _hdr()
    uses = set(re.findall(r"(?:sub|neg)<(\d+), (\d+)>", t))
    assert uses == {("30", "1"), ("32", "2"), ("16", "3"), ("64", "1"), ("2", "1"), ("3", "1"), ("8", "1")}
    for k, s in uses:
        _spread(int(k), int(s))
    # the initial negation 2q - y of a canonical y (< q) stays nonnegative per limb
    K = _spread(2, 1)
    assert all(K[j] >= (MASK if j < 8 else (Q - 1) >> 232) for j in range(9))


def test_pack_unpack_roundtrip_model():
    # python model of fq29::unpack / pack on random 256-bit values
    import random
    rnd = random.Random(7)
    for _ in range(200):
        x = rnd.getrandbits(255)
        w = [(x >> (32 * i)) & 0xffffffff for i in range(8)]
        limbs = []
        for j in range(9):
            bit = 29 * j
            i, s = bit >> 5, bit & 31
            v = w[i] >> s
            if s > 3 and i + 1 < 8:
                v |= (w[i + 1] << (32 - s)) & 0xffffffff
            limbs.append(v & MASK)
        assert _d29(limbs) == x
        out = []
        for i in range(8):
            bit = 32 * i
            j, s = bit // 29, bit % 29
            v = limbs[j] >> s
            if j + 1 < 9:
                v |= (limbs[j + 1] << (29 - s)) & 0xffffffff
            if s > 26 and j + 2 < 9:
                v |= (limbs[j + 2] << (58 - s)) & 0xffffffff
            out.append(v & 0xffffffff)
        assert out == w


def _cios(rows, m32):
    """fq29 CIOS loop of mul/sqr/mul2 on Python ints: rows(i) -> list of (absolute column offset j,
    product) pairs added in row i; rows < m32 run reduce_row32 (m = -t0/q0 mod 2^32 from the low
    word, carry = 8 x the high word of t0 + m q0), the others reduce_row; every 64-bit column
    accumulator is checked for overflow."""
    qv = [(Q >> (29 * j)) & MASK for j in range(8)] + [Q >> 232]
    inv = (-pow(Q, -1, 1 << 29)) % (1 << 29)
    inv32 = (-pow(qv[0], -1, 1 << 32)) % (1 << 32)
    t = [0] * 9
    for i in range(9):
        for j, p in rows(i):
            t[j] += p
            assert t[j] < (1 << 64)
        if i < m32:
            m = ((t[0] & 0xffffffff) * inv32) & 0xffffffff
            u = m * qv[0] + t[0]
            assert u < (1 << 64) and u % (1 << 32) == 0
            c = 8 * (u >> 32)
        else:
            m = (t[0] * inv) & MASK
            c = (m * qv[0] + t[0]) >> 29
        for j in range(1, 9):
            t[j] += m * qv[j]
            assert t[j] < (1 << 64)
        t = t[1:] + [0]
        t[0] += c
    r, c = [], 0
    for j in range(9):
        s = t[j] + c
        r.append(s & MASK)
        c = s >> 29
    r[8] += c << 29
    return _d29(r)


def _limbs(x):
    return [(x >> (29 * j)) & MASK for j in range(8)] + [x >> 232]


def test_sqr_mul2_model():
    # the exact row schedules of fq29::mul, fq29::sqr and fq29::mul2 (with the header's 32-bit-m rows)
    # on random inputs at their bound limits, and the all-limbs-maximal worst case
    import random
    rnd = random.Random(11)
    rinv = pow(2, -261, Q)
    m32, m32_mul2 = _m32_rows()
    big = (1 << 258) - 1
    for it in range(300):
        a = big if it == 0 else rnd.randrange(1 << 258)
        b0 = big if it == 0 else rnd.randrange(1 << 258)
        al, b0l = _limbs(a), _limbs(b0)
        d = [2 * x for x in al]
        sq = _cios(lambda i: [(i, al[i] * al[i])] + [(j, d[i] * al[j]) for j in range(i + 1, 9)], m32)
        assert sq % Q == a * a * rinv % Q and sq < (a * a >> 261) + Q + (Q >> 25) + 1
        mu = _cios(lambda i: [(j, al[i] * b0l[j]) for j in range(9)], m32)
        assert mu % Q == a * b0 * rinv % Q and mu < (a * b0 >> 261) + Q + (Q >> 25) + 1
        # mul2 with unnormalised second factors (limbs up to 2^30.6 / 2^29.8 as in add_aff)
        b, c, e = rnd.randrange(1 << 258), rnd.randrange(1 << 258), rnd.randrange(1 << 255)
        bl, cl, el = _limbs(b), _limbs(c), _limbs(e)
        bl = [x + (1 << 30) if j < 8 else x for j, x in enumerate(bl)]  # same value + spread carries
        bl = [bl[0]] + [bl[j] - 2 if j < 8 else bl[j] - 2 for j in range(1, 9)]
        bval = _d29(bl)
        m2 = _cios(lambda i: [(j, al[i] * bl[j]) for j in range(9)] + [(j, cl[i] * el[j]) for j in range(9)],
                   m32_mul2)
        assert m2 % Q == (a * bval + c * e) * rinv % Q
