"""BN254 arithmetic for the CPU ORACLE (test infrastructure only — never shipped, never measured).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.

Restates, from their mathematical definitions, the members of the third-party engine
`ffjavascript@0.2.59` (wasm from `wasmcurves@0.2.1`, NOT vendored in /root/reference) that the
reference calls on its hot path:

  * `curve.Fr` / `curve.F1` (Fq): Montgomery fields with R = 2^256, 32-byte little-endian storage
    (`Fr.one` = R mod r, `Fr.e`, `Fr.toRprBE`, `Fr.w[]` roots of unity with nqr = 5, s = 28);
  * `curve.G1` / `curve.G2`: short-Weierstrass y^2 = x^3 + 3 (and the D-type twist over Fq2),
    affine "LEM" storage (x||y, each 32 B LE Montgomery), `toRprUncompressed` (x||y big-endian
    standard form, infinity = 0x40 followed by zeros);
  * `curve.pairingEq`: optimal-ate pairing product check (restated in the py_ecc style: Fq12 as
    Fq[w]/(w^12 - 18 w^6 + 82), twist into Fq12, affine Miller loop, full final exponentiation).

Call sites in the reference: src/polynomial/polynomial.js:34,373,392,1109-1113,
src/polynomial/evaluations.js:18, src/grandsum/grandsum.js:41, src/Keccak256Transcript.js:37-51,
src/grandsum/mset_eq_kzg_verifier.js:119-182.
"""

# --------------------------------------------------------------------------- constants
Q = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
MONT = 1 << 256
FR_ONE_MONT = MONT % R      # ffjs Fr.one bytes (Montgomery form of 1)
FQ_ONE_MONT = MONT % Q
FR_S = 28                    # 2-adicity of r-1
FR_NQR = 5                   # first quadratic non-residue (ffjs searches upward)


def fr_inv(a):
    return pow(a % R, R - 2, R) if a % R else 0


def fq_inv(a):
    return pow(a % Q, Q - 2, Q) if a % Q else 0


def _roots():
    w = [0] * (FR_S + 1)
    w[FR_S] = pow(FR_NQR, (R - 1) >> FR_S, R)
    for k in range(FR_S - 1, -1, -1):
        w[k] = w[k + 1] * w[k + 1] % R
    return w


FR_W = _roots()               # Fr.w[k]: primitive 2^k-th root of unity (standard form)


# --------------------------------------------------------------------------- byte codecs
def fr_to_bytes(a):
    """standard-form int -> 32 B LE Montgomery (the in-memory form of every ffjs Fr element)."""
    return (a % R * MONT % R).to_bytes(32, "little")


def fr_from_bytes(b):
    """32 B LE Montgomery -> standard-form int."""
    return int.from_bytes(b, "little") * pow(MONT, -1, R) % R


def fr_std_to_bytes(a):
    """standard form, 32 B LE (what `Fr.batchFromMontgomery` produces / what callers pass in)."""
    return (a % R).to_bytes(32, "little")


def fq_to_bytes(a):
    return (a % Q * MONT % Q).to_bytes(32, "little")


def fq_from_bytes(b):
    return int.from_bytes(b, "little") * pow(MONT, -1, Q) % Q


def fr_e(v):
    """ffjs `Fr.e(bigint)`: reduce into the field (negative values wrap)."""
    return v % R


# --------------------------------------------------------------------------- G1 (affine ints, None = infinity)
B1 = 3
G1_GEN = (1, 2)


def g1_is_on_curve(p):
    if p is None:
        return True
    x, y = p
    return (y * y - x * x * x - B1) % Q == 0


def g1_neg(p):
    return None if p is None else (p[0], (-p[1]) % Q)


def g1_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2) % Q == 0:
            return None
        lam = 3 * x1 * x1 * fq_inv(2 * y1) % Q
    else:
        lam = (y2 - y1) * fq_inv(x2 - x1) % Q
    x3 = (lam * lam - x1 - x2) % Q
    return (x3, (lam * (x1 - x3) - y1) % Q)


# Jacobian helpers for speed (a = 0 curve)
def _jac_double(P):
    X, Y, Z = P
    if Z == 0:
        return P
    A = X * X % Q
    Bv = Y * Y % Q
    C = Bv * Bv % Q
    D = 2 * ((X + Bv) * (X + Bv) - A - C) % Q
    E = 3 * A % Q
    F = E * E % Q
    X3 = (F - 2 * D) % Q
    Y3 = (E * (D - X3) - 8 * C) % Q
    Z3 = 2 * Y * Z % Q
    return (X3, Y3, Z3)


def _jac_add(P, Qp):
    X1, Y1, Z1 = P
    X2, Y2, Z2 = Qp
    if Z1 == 0:
        return Qp
    if Z2 == 0:
        return P
    Z1Z1 = Z1 * Z1 % Q
    Z2Z2 = Z2 * Z2 % Q
    U1 = X1 * Z2Z2 % Q
    U2 = X2 * Z1Z1 % Q
    S1 = Y1 * Z2 * Z2Z2 % Q
    S2 = Y2 * Z1 * Z1Z1 % Q
    if U1 == U2:
        if S1 != S2:
            return (1, 1, 0)
        return _jac_double(P)
    H = (U2 - U1) % Q
    I = 4 * H * H % Q
    J = H * I % Q
    rr = 2 * (S2 - S1) % Q
    V = U1 * I % Q
    X3 = (rr * rr - J - 2 * V) % Q
    Y3 = (rr * (V - X3) - 2 * S1 * J) % Q
    Z3 = ((Z1 + Z2) * (Z1 + Z2) - Z1Z1 - Z2Z2) * H % Q
    return (X3, Y3, Z3)


def _to_jac(p):
    return (1, 1, 0) if p is None else (p[0], p[1], 1)


def _from_jac(P):
    X, Y, Z = P
    if Z == 0:
        return None
    zi = fq_inv(Z)
    zi2 = zi * zi % Q
    return (X * zi2 % Q, Y * zi2 * zi % Q)


def g1_mul(p, k):
    """ffjs `G1.timesFr` (scalar reduced mod r)."""
    k %= R
    acc = (1, 1, 0)
    base = _to_jac(p)
    while k:
        if k & 1:
            acc = _jac_add(acc, base)
        base = _jac_double(base)
        k >>= 1
    return _from_jac(acc)


def g1_sum(points):
    acc = (1, 1, 0)
    for p in points:
        acc = _jac_add(acc, _to_jac(p))
    return _from_jac(acc)


def g1_msm_pippenger(bases, scalars, c=None):
    """ffjs `G1.multiExpAffine` restated as a plain (unsigned-window) Pippenger MSM.

    bases: list of affine points (or None); scalars: standard-form ints. Result: affine or None.
    """
    n = len(scalars)
    if n == 0:
        return None
    if c is None:
        c = max(2, min(16, n.bit_length() - 2))
    nw = (254 + c - 1) // c
    total = (1, 1, 0)
    for w in range(nw - 1, -1, -1):
        for _ in range(c):
            total = _jac_double(total)
        buckets = [(1, 1, 0)] * (1 << c)
        for i in range(n):
            d = (scalars[i] >> (w * c)) & ((1 << c) - 1)
            if d and bases[i] is not None:
                buckets[d] = _jac_add(buckets[d], _to_jac(bases[i]))
        run = (1, 1, 0)
        acc = (1, 1, 0)
        for b in range((1 << c) - 1, 0, -1):
            run = _jac_add(run, buckets[b])
            acc = _jac_add(acc, run)
        total = _jac_add(total, acc)
    return _from_jac(total)


def g1_to_lem(p):
    """affine point -> 64 B LEM (ffjs affine storage; infinity = 64 zero bytes)."""
    if p is None:
        return bytes(64)
    return fq_to_bytes(p[0]) + fq_to_bytes(p[1])


def g1_from_lem(b):
    x = fq_from_bytes(b[:32])
    y = fq_from_bytes(b[32:64])
    if x == 0 and y == 0:
        return None
    return (x, y)


def g1_to_rpr_uncompressed(p):
    """ffjs `G1.toRprUncompressed`: x||y big-endian standard form; infinity -> 0x40, zeros."""
    if p is None:
        out = bytearray(64)
        out[0] = 0x40
        return bytes(out)
    return p[0].to_bytes(32, "big") + p[1].to_bytes(32, "big")


# --------------------------------------------------------------------------- Fq2 / G2
class FQ2:
    __slots__ = ("c0", "c1")

    def __init__(self, c0, c1=0):
        self.c0 = c0 % Q
        self.c1 = c1 % Q

    def __add__(self, o):
        return FQ2(self.c0 + o.c0, self.c1 + o.c1)

    def __sub__(self, o):
        return FQ2(self.c0 - o.c0, self.c1 - o.c1)

    def __neg__(self):
        return FQ2(-self.c0, -self.c1)

    def __mul__(self, o):
        if isinstance(o, int):
            return FQ2(self.c0 * o, self.c1 * o)
        return FQ2(self.c0 * o.c0 - self.c1 * o.c1, self.c0 * o.c1 + self.c1 * o.c0)

    __rmul__ = __mul__

    def inv(self):
        d = fq_inv(self.c0 * self.c0 + self.c1 * self.c1)
        return FQ2(self.c0 * d, -self.c1 * d)

    def __truediv__(self, o):
        return self * o.inv()

    def __eq__(self, o):
        return self.c0 == o.c0 and self.c1 == o.c1

    def is_zero(self):
        return self.c0 == 0 and self.c1 == 0


B2 = FQ2(3) / FQ2(9, 1)
G2_GEN = (
    FQ2(10857046999023057135944570762232829481370756359578518086990519993285655852781,
        11559732032986387107991004021392285783925812861821192530917403151452391805634),
    FQ2(8495653923123431417604973247489272438418190587263600148770280649306958101930,
        4082367875863433681332203403145435568316851327593401208105741076214120093531),
)


def g2_add(p1, p2):
    if p1 is None:
        return p2
    if p2 is None:
        return p1
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2:
        if (y1 + y2).is_zero():
            return None
        lam = (x1 * x1 * 3) / (y1 * 2)
    else:
        lam = (y2 - y1) / (x2 - x1)
    x3 = lam * lam - x1 - x2
    return (x3, lam * (x1 - x3) - y1)


def g2_mul(p, k):
    k %= R
    acc = None
    while k:
        if k & 1:
            acc = g2_add(acc, p)
        p = g2_add(p, p)
        k >>= 1
    return acc


def g2_to_lem(p):
    """128 B: x.c0 || x.c1 || y.c0 || y.c1, each 32 B LE Montgomery (ptau section 3 layout)."""
    if p is None:
        return bytes(128)
    x, y = p
    return fq_to_bytes(x.c0) + fq_to_bytes(x.c1) + fq_to_bytes(y.c0) + fq_to_bytes(y.c1)


def g2_from_lem(b):
    x = FQ2(fq_from_bytes(b[0:32]), fq_from_bytes(b[32:64]))
    y = FQ2(fq_from_bytes(b[64:96]), fq_from_bytes(b[96:128]))
    if x.is_zero() and y.is_zero():
        return None
    return (x, y)


# --------------------------------------------------------------------------- Fq12 + pairing
_FQ12_MOD = [82, 0, 0, 0, 0, 0, -18, 0, 0, 0, 0, 0]   # w^12 = 18 w^6 - 82


class FQ12:
    __slots__ = ("c",)

    def __init__(self, c):
        self.c = [x % Q for x in c]

    @staticmethod
    def one():
        return FQ12([1] + [0] * 11)

    def __add__(self, o):
        return FQ12([a + b for a, b in zip(self.c, o.c)])

    def __sub__(self, o):
        return FQ12([a - b for a, b in zip(self.c, o.c)])

    def __neg__(self):
        return FQ12([-a for a in self.c])

    def scale(self, k):
        return FQ12([a * k for a in self.c])

    def __mul__(self, o):
        if isinstance(o, int):
            return self.scale(o)
        b = [0] * 23
        for i, a in enumerate(self.c):
            if a:
                for j, bb in enumerate(o.c):
                    b[i + j] += a * bb
        for exp in range(22, 11, -1):
            top = b[exp]
            if top:
                b[exp] = 0
                b[exp - 6] += 18 * top
                b[exp - 12] -= 82 * top
        return FQ12(b[:12])

    def __pow__(self, e):
        res = FQ12.one()
        base = self
        while e:
            if e & 1:
                res = res * base
            base = base * base
            e >>= 1
        return res

    def inv(self):
        # extended Euclid over Fq[w] (py_ecc style)
        lm, hm = [1] + [0] * 12, [0] * 13
        low, high = self.c + [0], [82, 0, 0, 0, 0, 0, -18 % Q, 0, 0, 0, 0, 0, 1]

        def deg(p):
            d = len(p) - 1
            while d and p[d] % Q == 0:
                d -= 1
            return d

        def poly_rounded_div(a, b):
            dega, degb = deg(a), deg(b)
            temp = [x for x in a]
            o = [0] * len(a)
            binv = fq_inv(b[degb])
            for i in range(dega - degb, -1, -1):
                o[i] = (o[i] + temp[degb + i] * binv) % Q
                for c in range(degb + 1):
                    temp[c + i] = (temp[c + i] - o[i] * b[c]) % Q
            return o[:deg(o) + 1]

        while deg(low):
            rr = poly_rounded_div(high, low)
            rr += [0] * (13 - len(rr))
            nm = [x for x in hm]
            new = [x for x in high]
            for i in range(13):
                for j in range(13 - i):
                    nm[i + j] -= lm[i] * rr[j]
                    new[i + j] -= low[i] * rr[j]
            nm = [x % Q for x in nm]
            new = [x % Q for x in new]
            lm, low, hm, high = nm, new, lm, low
        d = fq_inv(low[0])
        return FQ12([x * d for x in lm[:12]])

    def __truediv__(self, o):
        return self * o.inv()

    def __eq__(self, o):
        return self.c == o.c

    def is_one(self):
        return self.c[0] == 1 and not any(self.c[1:])


_W12 = FQ12([0, 1] + [0] * 10)
_W2 = _W12 * _W12
_W3 = _W2 * _W12


def _twist(pt):
    x, y = pt
    xc = [x.c0 - x.c1 * 9, x.c1]
    yc = [y.c0 - y.c1 * 9, y.c1]
    nx = FQ12([xc[0]] + [0] * 5 + [xc[1]] + [0] * 5)
    ny = FQ12([yc[0]] + [0] * 5 + [yc[1]] + [0] * 5)
    return (nx * _W2, ny * _W3)


def _cast_g1(p):
    return (FQ12([p[0]] + [0] * 11), FQ12([p[1]] + [0] * 11))


def _linefunc(P1, P2, T):
    x1, y1 = P1
    x2, y2 = P2
    xt, yt = T
    if x1 != x2:
        m = (y2 - y1) / (x2 - x1)
        return m * (xt - x1) - (yt - y1)
    elif y1 == y2:
        m = (x1 * x1 * 3) / (y1 * 2)
        return m * (xt - x1) - (yt - y1)
    return xt - x1


def _add12(p1, p2):
    x1, y1 = p1
    x2, y2 = p2
    if x1 == x2 and y1 == y2:
        lam = (x1 * x1 * 3) / (y1 * 2)
    else:
        lam = (y2 - y1) / (x2 - x1)
    x3 = lam * lam - x1 - x2
    return (x3, lam * (x1 - x3) - y1)


_ATE = 29793968203157093288
_LOG_ATE = 63


def _miller(Qt, P):
    Rp = Qt
    f = FQ12.one()
    for i in range(_LOG_ATE, -1, -1):
        f = f * f * _linefunc(Rp, Rp, P)
        Rp = _add12(Rp, Rp)
        if _ATE & (1 << i):
            f = f * _linefunc(Rp, Qt, P)
            Rp = _add12(Rp, Qt)
    Q1 = (Qt[0] ** Q, Qt[1] ** Q)
    nQ2 = (Q1[0] ** Q, -(Q1[1] ** Q))
    f = f * _linefunc(Rp, Q1, P)
    Rp = _add12(Rp, Q1)
    f = f * _linefunc(Rp, nQ2, P)
    return f


def pairing_eq(a1, b1, a2, b2):
    """ffjs `curve.pairingEq(a1, b1, a2, b2)`: e(a1,b1)·e(a2,b2) == 1 (a* in G1, b* in G2)."""
    f = FQ12.one()
    for a, b in ((a1, b1), (a2, b2)):
        if a is None or b is None:
            continue
        f = f * _miller(_twist(b), _cast_g1(a))
    f = f ** ((Q ** 12 - 1) // R)
    return f.is_one()
