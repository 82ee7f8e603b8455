"""Coefficient/evaluation-form polynomials over BN254 Fr for the CPU ORACLE (test infrastructure only).

Op-for-op restatement of the reference's `Polynomial` (src/polynomial/polynomial.js) and
`Evaluations` (src/polynomial/evaluations.js), including buffer-length semantics (which decide NTT
sizes and, for `multiply`, the degenerate-degree quirk of SURVEY.md Appendix C.1). Values are kept
as standard-form Python ints; the byte representation (32 B LE Montgomery) is applied only at the
proof boundary, which is value-identical to ffjavascript's in-memory Montgomery buffers.

Two semantics (module flag QUIRKS, set per proof by `protocol.prove(..., quirks=...)`):
  * QUIRKS = True (default): the reference exactly, including three behaviours that only show on
    degenerate inputs (DESIGN.md §4 "Reference quirks"):
      Q1 `multiply` sizes each operand's FFT from its DEGREE but `Evaluations.fromPolynomial` pads
         from its buffer LENGTH (polynomial.js:352-376, evaluations.js:12-18): an operand of degree
         d >= 1 with 2^ceil(log2(d+1)) < 2^ceil(log2(length)) is evaluated on the wrong points;
      Q2 `add`/`sub` with a LONGER argument write into the argument's buffer and adopt it
         (polynomial.js:276-350): the two objects then share one buffer, and later in-place
         operations on either change both (lists are shared here exactly as buffers are there);
      Q3 `divZh` copies degree()+1 coefficients into a buffer of 0 elements when the dividend's
         degree is below the domain size (polynomial.js:857,884): V8's TypedArray `set` throws
         "RangeError: offset is out of bounds" (a zero quotient).
  * QUIRKS = False: the same operation sequence with exact products (both operands padded to the
    product's domain), no buffer sharing and a zero quotient kept — the mathematical values the
    MI355X prover computes in its default mode. On every non-degenerate input (all golden vectors)
    both semantics give the identical proof.
"""
from . import bn254 as bn

R = bn.R
QUIRKS = True


class JSRangeError(ValueError):
    """V8's RangeError from TypedArray.prototype.set (message as V8 prints it)."""


def _clog2(x):
    """Math.ceil(Math.log2(x)) for x >= 1."""
    return (x - 1).bit_length()


# --------------------------------------------------------------------------- NTT ([ffjs] Fr.fft/ifft)
def _bitrev_perm(a):
    n = len(a)
    j = 0
    for i in range(1, n):
        bit = n >> 1
        while j & bit:
            j ^= bit
            bit >>= 1
        j |= bit
        if i < j:
            a[i], a[j] = a[j], a[i]


def ntt(vals, inverse=False):
    """Natural-order DFT of size m = len(vals) over <Fr.w[log2 m]>; inverse includes 1/m.

    [ffjs] `Fr.fft` / `Fr.ifft` (called at polynomial.js:34,373,392, evaluations.js:18).
    fft: out_j = sum_i a_i w^(ij);  ifft: out_j = m^-1 sum_i a_i w^(-ij).
    """
    a = [v % R for v in vals]
    m = len(a)
    if m <= 1:
        return a
    logm = _clog2(m)
    assert 1 << logm == m
    w = bn.FR_W[logm]
    if inverse:
        w = pow(w, R - 2, R)
    _bitrev_perm(a)
    half = 1
    while half < m:
        wstep = pow(w, m // (2 * half), R)
        for start in range(0, m, 2 * half):
            wk = 1
            for k in range(half):
                u = a[start + k]
                v = a[start + k + half] * wk % R
                a[start + k] = (u + v) % R
                a[start + k + half] = (u - v) % R
                wk = wk * wstep % R
        half *= 2
    if inverse:
        minv = pow(m, R - 2, R)
        a = [x * minv % R for x in a]
    return a


def batch_inverse(vals):
    """[ffjs] `Fr.batchInverse` (grandsum.js:41): elementwise inverse; 0 maps to 0."""
    out = [0] * len(vals)
    acc = 1
    pref = []
    for v in vals:
        pref.append(acc)
        if v:
            acc = acc * v % R
    inv = pow(acc, R - 2, R)
    for i in range(len(vals) - 1, -1, -1):
        v = vals[i]
        if v:
            out[i] = inv * pref[i] % R
            inv = inv * v % R
    return out


# --------------------------------------------------------------------------- Evaluations
class Evaluations:
    """src/polynomial/evaluations.js:5-136 (values: standard-form ints, one per domain point)."""

    def __init__(self, vals):
        self.vals = list(vals)

    @staticmethod
    def from_polynomial(poly, extension):
        """evaluations.js:12-21 — zero-pads to 2^ceil(log2(buffer LENGTH)) * extension, then fft."""
        power = _clog2(poly.length())
        length = (1 << power) * extension
        buf = poly.coef + [0] * (length - poly.length())
        return Evaluations(ntt(buf, False))

    @staticmethod
    def one_evals(length):
        return Evaluations([1] * length)

    def length(self):
        return len(self.vals)

    def is_all_ones(self):
        return all(v == 1 for v in self.vals)

    def is_all_zeros(self):
        return all(v == 0 for v in self.vals)


# --------------------------------------------------------------------------- Polynomial
class Polynomial:
    """src/polynomial/polynomial.js:25-1116, hot-path subset."""

    def __init__(self, coef):
        self.coef = list(coef)

    # polynomial.js:33-37
    @staticmethod
    def from_evaluations(vals):
        return Polynomial(ntt(vals, True))

    # polynomial.js:63-66
    @staticmethod
    def zero(length):
        return Polynomial([0] * length)

    # polynomial.js:68-78
    @staticmethod
    def lagrange1(power):
        buf = [0] * (1 << power)
        buf[0] = 1
        return Polynomial.from_evaluations(buf)

    # polynomial.js:80-82
    def clone(self):
        return Polynomial(self.coef)

    def length(self):
        return len(self.coef)

    # polynomial.js:212-226
    def degree(self):
        for i in range(len(self.coef) - 1, 0, -1):
            if self.coef[i]:
                return i
        return 0

    # polynomial.js:228-238 (Horner from the top nonzero coefficient)
    def evaluate(self, x):
        res = 0
        for i in range(self.degree(), -1, -1):
            res = (res * x + self.coef[i]) % R
        return res

    # polynomial.js:276-312 / 314-350. Reference: when `other` is strictly longer the result is
    # written into other's buffer and self adopts it (Q2); otherwise into self's buffer, in place.
    def _addsub(self, other, sign, blinding):
        L = max(self.length(), other.length())
        a = self.coef + [0] * (L - self.length())
        b = other.coef + [0] * (L - other.length())
        if blinding is not None:
            b = [x * blinding % R for x in b]
        res = [(x + sign * y) % R for x, y in zip(a, b)]
        if QUIRKS and other.length() > self.length():
            other.coef[:] = res
            self.coef = other.coef
        elif self.length() == L:
            self.coef[:] = res
        else:
            self.coef = res
        return self

    def add(self, other, blinding=None):
        return self._addsub(other, 1, blinding)

    def sub(self, other, blinding=None):
        return self._addsub(other, -1, blinding)

    # polynomial.js:352-376 — sizes derived exactly as the reference does (Q1; Appendix C.1)
    def multiply(self, other):
        new_degree = self.degree() + other.degree()
        new_power = _clog2(new_degree + 1)
        new_length = 1 << new_power
        if QUIRKS:
            power1 = _clog2(self.degree() + 1)
            power2 = _clog2(other.degree() + 1)
            factor1 = 1 << (new_power - power1)
            factor2 = 1 << (new_power - power2)
            e1 = Evaluations.from_polynomial(self, factor1).vals
            e2 = Evaluations.from_polynomial(other, factor2).vals
        else:
            e1 = ntt(self.coef[:new_length] + [0] * (new_length - min(new_length, self.length())))
            e2 = ntt(other.coef[:new_length] + [0] * (new_length - min(new_length, other.length())))
        prod = [e1[i] * e2[i] % R for i in range(new_length)]
        self.coef = ntt(prod, True)
        return self

    # polynomial.js:378-393
    def shift_omega(self):
        ev = Evaluations.from_polynomial(self, 1).vals
        ev = ev[1:] + ev[:1]
        self.coef = ntt(ev, True)
        return self

    # polynomial.js:395-406
    def mul_scalar(self, v):
        self.coef[:] = [c * v % R for c in self.coef]
        return self

    # polynomial.js:408-422
    def add_scalar(self, v):
        if not self.coef:
            self.coef = [0]
        self.coef[0] = (self.coef[0] + v) % R
        return self

    def sub_scalar(self, v):
        if not self.coef:
            self.coef = [0]
        self.coef[0] = (self.coef[0] - v) % R
        return self

    # polynomial.js:814-851
    def div_by_x_sub_value(self, value):
        L = self.length()
        q = [0] * L
        q[L - 2] = self.coef[L - 1]
        for i in range(L - 3, -1, -1):
            q[i] = (self.coef[i + 1] + value * q[i + 1]) % R
        if self.coef[0] % R != (-value * q[0]) % R:
            raise ValueError("Polynomial does not divide")
        self.coef = q
        return self

    # polynomial.js:84-95 (equal up to each one's degree)
    def is_equal(self, other):
        d = self.degree()
        if d != other.degree():
            return False
        return all(self.coef[i] % R == other.coef[i] % R for i in range(d + 1))

    # polynomial.js:617-646: self <- quotient by (X^n - beta), returns the remainder polynomial (the
    # dividend's buffer with the reduced coefficients); same length as the dividend
    def div_by_vanishing(self, n, beta):
        if self.degree() < n:
            raise ValueError("divByVanishing polynomial divisor must be of degree lower than the dividend polynomial")
        rem = list(self.coef)
        q = [0] * self.length()
        for i in range(self.length() - 1, n - 1, -1):
            lead = rem[i] % R
            if lead == 0:
                continue
            rem[i] = 0
            rem[i - n] = (rem[i - n] + beta * lead) % R
            q[i - n] = (q[i - n] + lead) % R
        self.coef = q
        return Polynomial(rem)

    # polynomial.js:853-888
    def div_zh(self, domain_size):
        n = domain_size
        ext = self.length() // n
        deg = self.degree()
        length = 0 if deg < n else 1 << _clog2(deg + 1 - n)
        c = self.coef
        for i in range(n):
            c[i] = (-c[i]) % R
        for i in range(n, n * ext):
            a = (c[i - n] - c[i]) % R
            c[i] = a
            if i > n * (ext - 1) - ext and a != 0:
                raise ValueError("Polynomial is not divisible")
        d = self.degree()
        if QUIRKS and d + 1 > length:
            raise JSRangeError("offset is out of bounds")  # Q3: Uint8Array(0).set(32 bytes)
        nb = [0] * length
        nb[:d + 1] = c[:d + 1]
        self.coef = nb
        return self

    # polynomial.js:1106-1115 (N = degree()+1 bases; scalars leave Montgomery form)
    def multi_exponentiation(self, srs):
        n = self.degree() + 1
        return srs.msm(self.coef[:n])
