"""Known-answer tests that pin the CPU oracle's restatement of [ffjs] conventions
 and of the reference's polynomial.test.js KATs."""
import common  # noqa: F401
from oracle import bn254 as bn
from oracle import poly as OP
from oracle.keccak import keccak256
from oracle.protocol import Transcript, l1_eval, zh_eval

R = bn.R


def test_keccak256_kats():
    # js-sha3 keccak256 (Keccak256Transcript.js:50), legacy padding
    assert keccak256(b"").hex() == "c5d2460186f7233c927e7db2dcc703c0e500b653ca82273b7bfad8045d85a470"
    assert keccak256(b"abc").hex() == "4e03657aea45a94fc7d47ba826c8d667c0d1e6e33a64a036ec44f58fa12d6c45"
    # multi-block message (> 136 B rate)
    assert len(keccak256(b"\x00" * 300)) == 32


def test_roots_of_unity_kats():
    assert bn.FR_W[28] == 19103219067921713944291392827692070036145651957329286315305642004821462161904
    assert bn.FR_W[11] == 1120550406532664055539694724667294622065367841900378087843176726913374367458
    assert bn.FR_W[20] == 17220337697351015657950521176323262483320249231368149235373741788599650842711
    assert bn.FR_W[22] == 12143866164239048021030917283424216263377309185099704096317235600302831912062
    assert bn.FR_W[24] == 5709868443893258075976348696661355716898495876243883251619397131511003808859
    assert bn.FR_W[1] == R - 1
    for k in range(1, 29):
        assert pow(bn.FR_W[k], 1 << k, R) == 1 and pow(bn.FR_W[k], 1 << (k - 1), R) != 1


def test_montgomery_one_bytes():
    # Fr.one is the Montgomery one (R mod r)
    assert int.from_bytes(bn.fr_to_bytes(1), "little") == \
        6350874878119819312338956282401532410528162663560392320966563075034087161851
    assert int.from_bytes(bn.fq_to_bytes(1), "little") == \
        6350874878119819312338956282401532409788428879151445726012394534686998597021
    for v in (0, 1, 5, R - 1):
        assert bn.fr_from_bytes(bn.fr_to_bytes(v)) == v


def test_polynomial_evaluate_kat():
    # test/polynomial.test.js:117-124: [0,1,2,3] evaluated at 2 == 34
    assert OP.Polynomial([0, 1, 2, 3]).evaluate(2) == 34


def test_polynomial_multiply_kat():
    # test/polynomial.test.js:207-220: (2x^3 - 3x^2 + 2)(x^2 + 3x) = 2x^5 + 3x^4 - 9x^3 + 2x^2 + 6x
    p1 = OP.Polynomial([2, 0, (-3) % R, 2])
    p2 = OP.Polynomial([0, 3, 1])
    p1.multiply(p2)
    assert p1.coef[:6] == [0, 6, 2, (-9) % R, 3, 2]
    assert all(c == 0 for c in p1.coef[6:])


def test_div_by_x_sub_value():
    # (X - 6)(7X^2 - 3X + 4) = 7X^3 - 45X^2 + 22X - 24 (test/polynomial.test.js:255-262 inverse)
    p = OP.Polynomial([(-24) % R, 22, (-45) % R, 7])
    p.div_by_x_sub_value(6)
    assert p.coef == [4, (-3) % R, 7, 0]


def test_polynomial_degree_kat():
    # test/polynomial.test.js:31-70 (the degree sets the MSM length N of multiExponentiation,
    # polynomial.js:1106-1115, and the Horner start of evaluate)
    rnd = [7, 11, 13]
    assert OP.Polynomial([]).degree() == 0          # no coefficients
    assert OP.Polynomial([rnd[0]]).degree() == 0    # one coefficient
    assert OP.Polynomial([rnd[0], rnd[1]]).degree() == 1
    assert OP.Polynomial([rnd[0], 0]).degree() == 0  # the greatest is zero
    buff = [rnd[0], 0, 0]
    assert OP.Polynomial(buff).degree() == 0        # the two greatest are zero
    buff[2] = 1
    assert OP.Polynomial(buff).degree() == 2
    # degree-based equality (polynomial.js:84-95): trailing zeros do not matter
    assert OP.Polynomial([1, 2, 0, 0]).is_equal(OP.Polynomial([1, 2]))
    assert not OP.Polynomial([1, 2, 3]).is_equal(OP.Polynomial([1, 2]))


def test_div_by_vanishing_kat():
    # test/polynomial.test.js:240-253: divByVanishing(2, 2) of the 19-coefficient dividend
    e = lambda v: v % R  # noqa: E731  (Fr.e)
    dividend = OP.Polynomial([e(v) for v in (-14, -2, 3, -5, -6, -7, -8, -9, -10, -11, -12, -13, -14, -15, -16, -17,
                                             -18, 15, 16)])
    quotient = OP.Polynomial([e(v) for v in (7, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16)])
    rem = dividend.div_by_vanishing(2, e(2))
    assert dividend.is_equal(quotient)
    # and the identity dividend = q (X^2 - 2) + rem, with deg rem < 2
    assert rem.degree() < 2
    q = quotient.coef
    recon = [0] * 19
    for i, c in enumerate(q):
        recon[i + 2] = (recon[i + 2] + c) % R
        recon[i] = (recon[i] - 2 * c) % R
    recon[0] = (recon[0] + rem.coef[0]) % R
    recon[1] = (recon[1] + rem.coef[1]) % R
    assert recon == [e(v) for v in (-14, -2, 3, -5, -6, -7, -8, -9, -10, -11, -12, -13, -14, -15, -16, -17, -18, 15, 16)]
    # divZh is this division at beta = 1 (polynomial.js:853-888 specialises it): same quotient
    p = OP.Polynomial([e(v) for v in (-1, 0, 0, 0, 1, 0, 0, 0)])  # X^4 - 1 = 1 * (X^4 - 1)
    p.div_by_vanishing(4, 1)
    assert p.is_equal(OP.Polynomial([1]))
    try:
        OP.Polynomial([1, 2]).div_by_vanishing(2, 1)
        assert False, "a divisor of higher degree must throw"
    except ValueError as err:
        assert "must be of degree lower" in str(err)


def test_ntt_roundtrip_and_definition():
    vals = [(i * 7919 + 3) % R for i in range(16)]
    ev = OP.ntt(vals, False)
    w = bn.FR_W[4]
    for j in (0, 1, 5, 15):
        assert ev[j] == sum(vals[i] * pow(w, i * j, R) for i in range(16)) % R
    assert OP.ntt(ev, True) == vals


def test_batch_inverse_zero_maps_to_zero():
    out = OP.batch_inverse([3, 0, 5])
    assert out[1] == 0 and out[0] * 3 % R == 1 and out[2] * 5 % R == 1


def test_transcript_encoding():
    # Fr.toRprBE / G1.toRprUncompressed (infinity -> 0x40 || 0)
    assert bn.g1_to_rpr_uncompressed(None)[0] == 0x40
    assert bn.g1_to_rpr_uncompressed(bn.G1_GEN) == (1).to_bytes(32, "big") + (2).to_bytes(32, "big")
    t = Transcript()
    t.add_field_element(5)
    assert t.get_challenge() == int.from_bytes(keccak256((5).to_bytes(32, "big")), "big") % R


def test_zh_l1():
    xi = 123456789
    zh = zh_eval(xi, 3)
    assert zh == (pow(xi, 8, R) - 1) % R
    l1 = l1_eval(xi, zh, 3)
    # L1(X) = (X^n - 1)/(n (X - 1)) == sum_i X^i / n
    assert l1 == sum(pow(xi, i, R) for i in range(8)) * pow(8, R - 2, R) % R


def test_pairing_bilinear():
    a, b = 12345, 67890
    P1 = bn.g1_mul(bn.G1_GEN, a)
    Q1 = bn.g2_mul(bn.G2_GEN, b)
    assert bn.pairing_eq(bn.g1_neg(P1), Q1, bn.g1_mul(bn.G1_GEN, a * b), bn.G2_GEN)
    assert not bn.pairing_eq(bn.g1_neg(P1), Q1, bn.g1_mul(bn.G1_GEN, a * b + 1), bn.G2_GEN)
