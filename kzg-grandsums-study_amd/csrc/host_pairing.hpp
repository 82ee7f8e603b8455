// Host-side BN254 extension tower, G2 and the optimal-ate pairing — the `curve.pairingEq` the
// reference verifiers end with (src/grandsum/mset_eq_kzg_verifier.js:186,
// src/grandproduct/mset_eq_kzg_verifier.js:178; [ffjs] bn128 pairing). Verification is a few
// hundred field operations plus two Miller loops and one final exponentiation: host work, no GPU.
//
// Tower: Fq2 = Fq[u]/(u^2 + 1), Fq6 = Fq2[v]/(v^3 - xi), xi = 9 + u, Fq12 = Fq6[w]/(w^2 - v).
// G2 lives on the D-type twist y^2 = x^3 + 3/xi, untwisted by (x, y) -> (x w^2, y w^3).
// Miller loop over 6u+2 (u = 4965661367192848881) with affine line functions, then the two
// Frobenius lines; final exponentiation (q^12 - 1)/r = (q^6 - 1)(q^2 + 1)(q^4 - q^2 + 1)/r with the
// first factor by conjugation and the rest by square-and-multiply (exponents derived from q, r).
#pragma once
#include "host_field.hpp"

namespace kgs {
namespace host {

struct Fq2 {
  Fq a, b;  // a + b u
  static Fq2 zero() { return {Fq::zero(), Fq::zero()}; }
  static Fq2 one() { return {Fq::one(), Fq::zero()}; }
  Fq2 operator+(const Fq2& o) const { return {a + o.a, b + o.b}; }
  Fq2 operator-(const Fq2& o) const { return {a - o.a, b - o.b}; }
  Fq2 operator*(const Fq2& o) const {
    Fq t0 = a * o.a, t1 = b * o.b;
    return {t0 - t1, (a + b) * (o.a + o.b) - t0 - t1};
  }
  Fq2 mul_fq(const Fq& s) const { return {a * s, b * s}; }
  Fq2 sqr() const { return (*this) * (*this); }
  Fq2 neg() const { return {a.neg(), b.neg()}; }
  Fq2 conj() const { return {a, b.neg()}; }
  Fq2 dbl() const { return *this + *this; }
  Fq2 mul_xi() const {  // (a + b u)(9 + u) = (9a - b) + (a + 9b) u
    Fq a9 = a.dbl().dbl().dbl() + a, b9 = b.dbl().dbl().dbl() + b;
    return {a9 - b, a + b9};
  }
  Fq2 inv() const {
    Fq d = (a.sqr() + b.sqr()).inverse();
    return {a * d, b.neg() * d};
  }
  bool is_zero() const { return a.is_zero() && b.is_zero(); }
  bool operator==(const Fq2& o) const { return a == o.a && b == o.b; }
  bool operator!=(const Fq2& o) const { return !(*this == o); }
  Fq2 pow(const uint64_t* e, int nlimbs) const {
    Fq2 r = one();
    for (int i = 64 * nlimbs - 1; i >= 0; i--) {
      r = r.sqr();
      if ((e[i >> 6] >> (i & 63)) & 1) r = r * (*this);
    }
    return r;
  }
};

struct Fq6 {
  Fq2 c0, c1, c2;  // c0 + c1 v + c2 v^2
  static Fq6 zero() { return {Fq2::zero(), Fq2::zero(), Fq2::zero()}; }
  static Fq6 one() { return {Fq2::one(), Fq2::zero(), Fq2::zero()}; }
  Fq6 operator+(const Fq6& o) const { return {c0 + o.c0, c1 + o.c1, c2 + o.c2}; }
  Fq6 operator-(const Fq6& o) const { return {c0 - o.c0, c1 - o.c1, c2 - o.c2}; }
  Fq6 neg() const { return {c0.neg(), c1.neg(), c2.neg()}; }
  Fq6 operator*(const Fq6& o) const {
    Fq2 t0 = c0 * o.c0, t1 = c1 * o.c1, t2 = c2 * o.c2;
    Fq6 r;
    r.c0 = ((c1 + c2) * (o.c1 + o.c2) - t1 - t2).mul_xi() + t0;
    r.c1 = (c0 + c1) * (o.c0 + o.c1) - t0 - t1 + t2.mul_xi();
    r.c2 = (c0 + c2) * (o.c0 + o.c2) - t0 - t2 + t1;
    return r;
  }
  Fq6 mul_v() const { return {c2.mul_xi(), c0, c1}; }
  Fq6 inv() const {
    Fq2 A = c0.sqr() - (c1 * c2).mul_xi();
    Fq2 B = c2.sqr().mul_xi() - c0 * c1;
    Fq2 C = c1.sqr() - c0 * c2;
    Fq2 F = c0 * A + (c2 * B + c1 * C).mul_xi();
    Fq2 fi = F.inv();
    return {A * fi, B * fi, C * fi};
  }
  bool operator==(const Fq6& o) const { return c0 == o.c0 && c1 == o.c1 && c2 == o.c2; }
};

struct Fq12 {
  Fq6 c0, c1;  // c0 + c1 w
  static Fq12 one() { return {Fq6::one(), Fq6::zero()}; }
  Fq12 operator*(const Fq12& o) const {
    Fq6 t0 = c0 * o.c0, t1 = c1 * o.c1;
    return {t0 + t1.mul_v(), (c0 + c1) * (o.c0 + o.c1) - t0 - t1};
  }
  Fq12 sqr() const { return (*this) * (*this); }
  Fq12 conj() const { return {c0, c1.neg()}; }
  Fq12 inv() const {
    Fq6 t = (c0 * c0 - (c1 * c1).mul_v()).inv();
    return {c0 * t, (c1 * t).neg()};
  }
  bool operator==(const Fq12& o) const { return c0 == o.c0 && c1 == o.c1; }
  bool is_one() const { return *this == one(); }
  Fq12 pow(const uint64_t* e, int nlimbs) const {
    Fq12 r = one();
    for (int i = 64 * nlimbs - 1; i >= 0; i--) {
      r = r.sqr();
      if ((e[i >> 6] >> (i & 63)) & 1) r = r * (*this);
    }
    return r;
  }
};

// affine G2 point on the twist
struct G2A {
  Fq2 x, y;
  bool inf;
};

inline G2A g2_add(const G2A& p, const G2A& q) {
  if (p.inf) return q;
  if (q.inf) return p;
  Fq2 lam;
  if (p.x == q.x) {
    if ((p.y + q.y).is_zero()) return {p.x, p.y, true};
    Fq2 x2 = p.x.sqr();
    lam = (x2 + x2 + x2) * (p.y + p.y).inv();
  } else {
    lam = (q.y - p.y) * (q.x - p.x).inv();
  }
  G2A r;
  r.inf = false;
  r.x = lam.sqr() - p.x - q.x;
  r.y = lam * (p.x - r.x) - p.y;
  return r;
}

inline Fq fq_from_dec(const char* s) {
  Fq acc = Fq::zero(), ten = Fq::from_u64(10);
  for (; *s; s++) acc = acc * ten + Fq::from_u64((uint64_t)(*s - '0'));
  return acc;
}

// [1]_2 ([ffjs] bn128 G2.g)
inline G2A g2_gen() {
  G2A g;
  g.inf = false;
  g.x = {fq_from_dec("10857046999023057135944570762232829481370756359578518086990519993285655852781"),
         fq_from_dec("11559732032986387107991004021392285783925812861821192530917403151452391805634")};
  g.y = {fq_from_dec("8495653923123431417604973247489272438418190587263600148770280649306958101930"),
         fq_from_dec("4082367875863433681332203403145435568316851327593401208105741076214120093531")};
  return g;
}

// 128 B LEM: x.a || x.b || y.a || y.b (ptau section 3 layout); infinity = zeros
inline void g2_lem(const G2A& p, uint8_t out[128]) {
  if (p.inf) {
    memset(out, 0, 128);
    return;
  }
  p.x.a.to_bytes(out);
  p.x.b.to_bytes(out + 32);
  p.y.a.to_bytes(out + 64);
  p.y.b.to_bytes(out + 96);
}
inline G2A g2_from_lem(const uint8_t in[128]) {
  G2A p;
  p.x = {Fq::from_bytes(in), Fq::from_bytes(in + 32)};
  p.y = {Fq::from_bytes(in + 64), Fq::from_bytes(in + 96)};
  p.inf = p.x.is_zero() && p.y.is_zero();
  return p;
}
inline bool g2_on_curve(const G2A& p) {
  if (p.inf) return true;
  Fq2 b2 = Fq2{Fq::from_u64(3), Fq::zero()} * Fq2{Fq::from_u64(9), Fq::one()}.inv();
  return p.y.sqr() == p.x.sqr() * p.x + b2;
}

// --- exponents (functions of q and r only)
static const uint64_t E_Q2[8] = {0x3b5458a2275d69b1ull, 0xa602072d09eac101ull, 0x4a50189c6d96cadcull, 0x04689e957a1242c8ull,
                                 0x26edfa5c34c6b38dull, 0xb00b855116375606ull, 0x599a6f7c0348d21cull, 0x0925c4b8763cbf9cull};
static const uint64_t E_HARD[12] = {0xe81bb482ccdf42b1ull, 0x5abf5cc4f49c36d4ull, 0xf1154e7e1da014fdull, 0xdcc7b44c87cdbacfull,
                                    0xaaa441e3954bcf8aull, 0x6b887d56d5095f23ull, 0x79581e16f3fd90c6ull, 0x3b1b1355d189227dull,
                                    0x4e529a5861876f6bull, 0x6c0eb522d5b12278ull, 0x331ec15183177fafull, 0x01baaa710b0759adull};
static const uint64_t E_QM1_3[4] = {0x69602eb24829a9c2ull, 0xdd2b2385cd7b4384ull, 0xe81ac1e7808072c9ull, 0x10216f7ba065e00dull};
static const uint64_t E_QM1_2[4] = {0x9e10460b6c3e7ea3ull, 0xcbc0b548b438e546ull, 0xdc2822db40c0ac2eull, 0x183227397098d014ull};
static const uint64_t E_Q2M1_3[8] = {0x691c1d8b62747890ull, 0x8cab57b9adf8eb00ull, 0x18c55d8979dcee49ull, 0x56cd8a31d35b6b98ull,
                                     0xb7a4a8c966ece684ull, 0xe5592c705cbd1cacull, 0x1dde2529566d9b5eull, 0x030c96e827699534ull};
static const uint64_t E_Q2M1_2[8] = {0x9daa2c5113aeb4d8ull, 0x5301039684f56080ull, 0x25280c4e36cb656eull, 0x82344f4abd092164ull,
                                     0x1376fd2e1a6359c6ull, 0x5805c2a88b1bab03ull, 0x2ccd37be01a4690eull, 0x0492e25c3b1e5fceull};
// 6u + 2 = 29793968203157093288 (65 bits)
static const unsigned __int128 ATE_LOOP = ((unsigned __int128)0x1ull << 64) | 0x9d797039be763ba8ull;

struct FrobConsts {
  Fq2 g12, g13, g22, g23;  // xi^((q-1)/3), xi^((q-1)/2), xi^((q^2-1)/3), xi^((q^2-1)/2)
  FrobConsts() {
    Fq2 xi{Fq::from_u64(9), Fq::one()};
    g12 = xi.pow(E_QM1_3, 4);
    g13 = xi.pow(E_QM1_2, 4);
    g22 = xi.pow(E_Q2M1_3, 8);
    g23 = xi.pow(E_Q2M1_2, 8);
  }
};
inline const FrobConsts& frob() {
  static const FrobConsts f;
  return f;
}

// line through T (slope lam) evaluated at P = (xp, yp) in G1, untwisted:
// yp - lam xp w + (lam xT - yT) w^3  (w^3 = v w)
inline Fq12 line_eval(const Fq2& lam, const G2A& T, const Fq& xp, const Fq& yp) {
  Fq12 l;
  l.c0 = Fq6::zero();
  l.c1 = Fq6::zero();
  l.c0.c0 = {yp, Fq::zero()};
  l.c1.c0 = lam.mul_fq(xp).neg();
  l.c1.c1 = lam * T.x - T.y;
  return l;
}

// f *= l_{T,Q}(P); T = T + Q  (T != +-Q, both finite) or doubling when Q == T
inline void miller_step(Fq12& f, G2A& T, const G2A& Q, const Fq& xp, const Fq& yp, bool dbl) {
  Fq2 lam;
  if (dbl) {
    Fq2 x2 = T.x.sqr();
    lam = (x2 + x2 + x2) * T.y.dbl().inv();
  } else {
    // T = [m]Q with 1 < m < r (or a Frobenius image): never +-Q, so no vertical line
    lam = (Q.y - T.y) * (Q.x - T.x).inv();
  }
  f = f * line_eval(lam, T, xp, yp);
  G2A R;
  R.inf = false;
  R.x = lam.sqr() - T.x - (dbl ? T.x : Q.x);
  R.y = lam * (T.x - R.x) - T.y;
  T = R;
}

// Miller loop of the optimal ate pairing for affine P (G1, Montgomery Fq) and Q (twist)
inline Fq12 miller_loop(const Fq& xp, const Fq& yp, const G2A& Q) {
  Fq12 f = Fq12::one();
  G2A T = Q;
  int top = 127;
  while (!((ATE_LOOP >> top) & 1)) top--;
  for (int i = top - 1; i >= 0; i--) {
    f = f.sqr();
    miller_step(f, T, T, xp, yp, true);
    if ((ATE_LOOP >> i) & 1) miller_step(f, T, Q, xp, yp, false);
  }
  const FrobConsts& F = frob();
  G2A Q1{Q.x.conj() * F.g12, Q.y.conj() * F.g13, false};
  G2A Q2{Q.x * F.g22, (Q.y * F.g23).neg(), false};  // -pi^2(Q)
  miller_step(f, T, Q1, xp, yp, false);
  miller_step(f, T, Q2, xp, yp, false);
  return f;
}

inline Fq12 final_exp(const Fq12& f) {
  Fq12 f1 = f.conj() * f.inv();          // f^(q^6 - 1)
  Fq12 f2 = f1.pow(E_Q2, 8) * f1;        // ^(q^2 + 1)
  return f2.pow(E_HARD, 12);             // ^((q^4 - q^2 + 1) / r)
}

// curve.pairingEq(a1, b1, ..., an, bn): prod_k e(a_k, b_k) == 1 (one final exponentiation); G1
// points as host XYZZ, G2 affine
inline bool pairing_eq(const G1* const* as, const G2A* const* bs, int n) {
  Fq12 f = Fq12::one();
  for (int k = 0; k < n; k++) {
    if (as[k]->is_inf() || bs[k]->inf) continue;  // e(O, Q) = e(P, O) = 1
    uint8_t lem[64];
    as[k]->to_affine_lem(lem);
    f = f * miller_loop(Fq::from_bytes(lem), Fq::from_bytes(lem + 32), *bs[k]);
  }
  return final_exp(f).is_one();
}
inline bool pairing_eq2(const G1& a1, const G2A& b1, const G1& a2, const G2A& b2) {
  const G1* as[2] = {&a1, &a2};
  const G2A* bs[2] = {&b1, &b2};
  return pairing_eq(as, bs, 2);
}
// y^2 = x^3 + 3 for an affine LEM G1 point (the zero point (0, 0) is valid)
inline bool g1_lem_on_curve(const uint8_t lem[64]) {
  Fq x = Fq::from_bytes(lem), y = Fq::from_bytes(lem + 32);
  if (x.is_zero() && y.is_zero()) return true;
  return y.sqr() == x.sqr() * x + Fq::from_u64(3);
}

}  // namespace host
}  // namespace kgs
