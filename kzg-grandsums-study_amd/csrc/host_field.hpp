// Host-side BN254 arithmetic (4 x 64-bit limbs, Montgomery R = 2^256) — same bytes as the device
// representation in field.hpp. Used for Fiat-Shamir challenges, scalar evaluations (r(X)
// coefficients, Z_H(xi), L1(xi)), the last few point additions of each MSM and affine conversion.
#pragma once
#include <stdint.h>
#include <string.h>
#include <string>

namespace kgs {
namespace host {

typedef unsigned __int128 u128;

struct Mod {
  uint64_t p[4];
  uint64_t inv;  // -p^-1 mod 2^64
  uint64_t one[4];
  uint64_t r2[4];
};

inline constexpr Mod FQ_MOD = {
    {0x3c208c16d87cfd47ull, 0x97816a916871ca8dull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
    0x87d20782e4866389ull,
    {0xd35d438dc58f0d9dull, 0x0a78eb28f5c70b3dull, 0x666ea36f7879462cull, 0x0e0a77c19a07df2full},
    {0xf32cfc5b538afa89ull, 0xb5e71911d44501fbull, 0x47ab1eff0a417ff6ull, 0x06d89f71cab8351full}};
inline constexpr Mod FR_MOD = {
    {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull},
    0xc2e1f593efffffffull,
    {0xac96341c4ffffffbull, 0x36fc76959f60cd29ull, 0x666ea36f7879462eull, 0x0e0a77c19a07df2full},
    {0x1bb8e645ae216da7ull, 0x53fe3ab1e35c59e3ull, 0x8c49833d53bb8085ull, 0x0216d0b17f4e44a5ull}};

template <const Mod& M>
struct F {
  uint64_t v[4];

  static F zero() { F r; memset(r.v, 0, 32); return r; }
  static F one() { F r; memcpy(r.v, M.one, 32); return r; }
  static F from_bytes(const uint8_t* b) { F r; memcpy(r.v, b, 32); return r; }  // Montgomery LE
  void to_bytes(uint8_t* b) const { memcpy(b, v, 32); }
  bool is_zero() const { return (v[0] | v[1] | v[2] | v[3]) == 0; }
  bool operator==(const F& o) const { return memcmp(v, o.v, 32) == 0; }
  bool operator!=(const F& o) const { return !(*this == o); }

  static bool geq_p(const uint64_t* a) {
    for (int i = 3; i >= 0; i--) {
      if (a[i] != M.p[i]) return a[i] > M.p[i];
    }
    return true;
  }
  static void sub_p(uint64_t* a) {
    u128 b = 0;
    for (int i = 0; i < 4; i++) {
      u128 t = (u128)a[i] - M.p[i] - (uint64_t)b;
      a[i] = (uint64_t)t;
      b = (t >> 64) & 1;
    }
  }
  friend F operator+(const F& a, const F& b) {
    F r;
    u128 c = 0;
    for (int i = 0; i < 4; i++) {
      u128 t = (u128)a.v[i] + b.v[i] + (uint64_t)c;
      r.v[i] = (uint64_t)t;
      c = t >> 64;
    }
    if (geq_p(r.v)) sub_p(r.v);
    return r;
  }
  friend F operator-(const F& a, const F& b) {
    F r;
    u128 br = 0;
    for (int i = 0; i < 4; i++) {
      u128 t = (u128)a.v[i] - b.v[i] - (uint64_t)br;
      r.v[i] = (uint64_t)t;
      br = (t >> 64) & 1;
    }
    if (br) {
      u128 c = 0;
      for (int i = 0; i < 4; i++) {
        u128 t = (u128)r.v[i] + M.p[i] + (uint64_t)c;
        r.v[i] = (uint64_t)t;
        c = t >> 64;
      }
    }
    return r;
  }
  F neg() const { return is_zero() ? *this : zero() - *this; }
  F dbl() const { return *this + *this; }
  friend F operator*(const F& a, const F& b) {
    uint64_t t[6] = {0, 0, 0, 0, 0, 0};
    for (int i = 0; i < 4; i++) {
      u128 c = 0;
      for (int j = 0; j < 4; j++) {
        u128 x = (u128)a.v[j] * b.v[i] + t[j] + (uint64_t)c;
        t[j] = (uint64_t)x;
        c = x >> 64;
      }
      u128 s = (u128)t[4] + (uint64_t)c;
      t[4] = (uint64_t)s;
      t[5] = (uint64_t)(s >> 64);
      uint64_t m = t[0] * M.inv;
      u128 x = (u128)m * M.p[0] + t[0];
      c = x >> 64;
      for (int j = 1; j < 4; j++) {
        x = (u128)m * M.p[j] + t[j] + (uint64_t)c;
        t[j - 1] = (uint64_t)x;
        c = x >> 64;
      }
      s = (u128)t[4] + (uint64_t)c;
      t[3] = (uint64_t)s;
      t[4] = t[5] + (uint64_t)(s >> 64);
    }
    F r;
    memcpy(r.v, t, 32);
    if (t[4] || geq_p(r.v)) sub_p(r.v);
    return r;
  }
  F sqr() const { return (*this) * (*this); }
  F pow(const uint64_t e[4]) const {
    F r = one();
    for (int i = 255; i >= 0; i--) {
      r = r.sqr();
      if ((e[i >> 6] >> (i & 63)) & 1) r = r * (*this);
    }
    return r;
  }
  F pow_u64(uint64_t e) const {
    uint64_t ee[4] = {e, 0, 0, 0};
    return pow(ee);
  }
  F inverse() const {
    uint64_t e[4];
    memcpy(e, M.p, 32);
    e[0] -= 2;
    return pow(e);
  }
  // standard-form conversions
  static F from_std(const uint64_t s[4]) {
    F a; memcpy(a.v, s, 32);
    F r2; memcpy(r2.v, M.r2, 32);
    return a * r2;
  }
  static F from_u64(uint64_t x) { uint64_t s[4] = {x, 0, 0, 0}; return from_std(s); }
  void to_std(uint64_t s[4]) const {
    F o = zero(); o.v[0] = 1;
    F r = (*this) * o;
    memcpy(s, r.v, 32);
  }
  // reduce an arbitrary 256-bit big-endian integer mod p (ffjs Fr.e(Scalar.fromRprBE(h)))
  static F from_be_reduce(const uint8_t be[32]) {
    uint64_t s[4];
    for (int i = 0; i < 4; i++) {
      uint64_t w = 0;
      for (int k = 0; k < 8; k++) w = (w << 8) | be[(3 - i) * 8 + k];
      s[i] = w;
    }
    while (geq_p(s)) sub_p(s);  // h < 2^256 < 6p: at most 5 subtractions
    return from_std(s);
  }
  void to_be_std(uint8_t be[32]) const {
    uint64_t s[4];
    to_std(s);
    for (int i = 0; i < 4; i++)
      for (int k = 0; k < 8; k++) be[(3 - i) * 8 + k] = (uint8_t)(s[i] >> (56 - 8 * k));
  }
};

typedef F<FR_MOD> Fr;
typedef F<FQ_MOD> Fq;

// Fr.w[k] (standard BN254 roots: nqr = 5, s = 28) and the coset shift g = 5
inline Fr fr_w(int k) {
  // (r-1) >> 28
  uint64_t e[4];
  memcpy(e, host::FR_MOD.p, 32);
  e[0] -= 1;
  for (int s = 0; s < 28; s++) {
    e[0] = (e[0] >> 1) | (e[1] << 63);
    e[1] = (e[1] >> 1) | (e[2] << 63);
    e[2] = (e[2] >> 1) | (e[3] << 63);
    e[3] >>= 1;
  }
  Fr w = Fr::from_u64(5).pow(e);
  for (int s = 28; s > k; s--) w = w.sqr();
  return w;
}

// G1 in XYZZ on the host (matches the device layout: X,Y,ZZ,ZZZ, 128 B)
struct G1 {
  Fq X, Y, ZZ, ZZZ;
  static G1 inf() { G1 r; r.X = Fq::one(); r.Y = Fq::one(); r.ZZ = Fq::zero(); r.ZZZ = Fq::zero(); return r; }
  bool is_inf() const { return ZZ.is_zero(); }
  static G1 from_bytes128(const uint8_t* b) {
    G1 r;
    r.X = Fq::from_bytes(b); r.Y = Fq::from_bytes(b + 32);
    r.ZZ = Fq::from_bytes(b + 64); r.ZZZ = Fq::from_bytes(b + 96);
    return r;
  }
  static G1 from_affine_lem(const uint8_t* b) {
    Fq x = Fq::from_bytes(b), y = Fq::from_bytes(b + 32);
    if (x.is_zero() && y.is_zero()) return inf();
    G1 r; r.X = x; r.Y = y; r.ZZ = Fq::one(); r.ZZZ = Fq::one();
    return r;
  }
  G1 dbl() const {
    if (is_inf()) return *this;
    Fq U = Y + Y, V = U.sqr(), W = U * V, S = X * V, X2 = X.sqr();
    Fq M = X2 + X2 + X2;
    G1 r;
    r.X = M.sqr() - (S + S);
    r.Y = M * (S - r.X) - W * Y;
    r.ZZ = V * ZZ;
    r.ZZZ = W * ZZZ;
    return r;
  }
  G1 add(const G1& o) const {
    if (o.is_inf()) return *this;
    if (is_inf()) return o;
    Fq U1 = X * o.ZZ, U2 = o.X * ZZ, S1 = Y * o.ZZZ, S2 = o.Y * ZZZ;
    Fq P = U2 - U1, R = S2 - S1;
    if (P.is_zero()) return R.is_zero() ? dbl() : inf();
    Fq PP = P.sqr(), PPP = P * PP, Qv = U1 * PP;
    G1 r;
    r.X = R.sqr() - PPP - (Qv + Qv);
    r.Y = R * (Qv - r.X) - S1 * PPP;
    r.ZZ = ZZ * o.ZZ * PP;
    r.ZZZ = ZZZ * o.ZZZ * PPP;
    return r;
  }
  G1 neg() const { G1 r = *this; r.Y = Y.neg(); return r; }
  G1 mul(const Fr& k) const {  // scalar k (Montgomery Fr)
    uint64_t s[4];
    k.to_std(s);
    G1 r = inf();
    for (int i = 255; i >= 0; i--) {
      r = r.dbl();
      if ((s[i >> 6] >> (i & 63)) & 1) r = r.add(*this);
    }
    return r;
  }
  // affine LEM (x||y Montgomery LE); infinity -> 64 zero bytes (ffjs affine zero)
  void to_affine_lem(uint8_t out[64]) const {
    if (is_inf()) { memset(out, 0, 64); return; }
    Fq inv = (ZZ * ZZZ).inverse();
    Fq zzzinv = inv * ZZ;        // 1/ZZZ
    Fq zzinv = inv * ZZZ;        // 1/ZZ
    Fq x = X * zzinv, y = Y * zzzinv;
    x.to_bytes(out);
    y.to_bytes(out + 32);
  }
};

// ffjs G1.toRprUncompressed of an affine LEM point: x||y big-endian standard; infinity -> 0x40,0..
inline void g1_lem_to_rpr_uncompressed(const uint8_t lem[64], uint8_t out[64]) {
  Fq x = Fq::from_bytes(lem), y = Fq::from_bytes(lem + 32);
  if (x.is_zero() && y.is_zero()) {
    memset(out, 0, 64);
    out[0] = 0x40;
    return;
  }
  x.to_be_std(out);
  y.to_be_std(out + 32);
}

}  // namespace host
}  // namespace kgs
