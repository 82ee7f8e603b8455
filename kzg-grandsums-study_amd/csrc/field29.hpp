// BN254 Fq in 9 x 29-bit limbs for the MSM bucket accumulation (device only).
//
// Why a second representation: in the 8 x 32-bit product-scanning product every 32x32 partial
// product needs a v_mad_u64_u32 AND a v_addc_co_u32 for the column's carry word. With 29-bit limbs
// a 58-bit partial product is accumulated into a 64-bit column by the mad ALONE (a column takes 18
// products plus a carry without overflowing), so a Montgomery product is 162 mads and a handful of
// shifts: measured 145 vs 115 G products/s on MI355X (scratch micro-benchmark). Additions and
// subtractions become carry-free limb-wise adds (a - b = a + K - b with K a multiple of q whose
// limbs are "spread" above b's limbs), normalised (one carry pass) only where a value is squared
// or stored.
//
// Values are Montgomery residues with R = 2^261 (x is held as x * 2^261 mod q, NOT reduced below
// q). The bound analysis of every operation in g1_acc29::add_aff below (value bound and limb bound
// of each intermediate, column overflow of each product) is reproduced by DESIGN.md §MSM and was
// re-derived by tests/test_field29.py (interval arithmetic over the exact constants); accumulator
// coordinates stay < 2^258.6.
// Conversions: the MSM table stores affine coordinates as x * 2^261 mod q (canonical, packed into
// 8 x 32-bit words like every other field element); bucket sums leave through mul(., 2^256 mod q),
// which yields the usual 256-bit Montgomery form (< 2q, one conditional subtraction).
#pragma once
#include "field.hpp"

// CIOS rows that take the 32-bit m of fq29::reduce_row32 (at most 8: row 8 keeps the 29-bit m; the
// column bounds are re-derived by tests/test_field29.py); 0 builds the all-29-bit-m products for A/B
#ifndef KGS_M32_ROWS
#define KGS_M32_ROWS 8
#endif
#ifndef KGS_M32_ROWS_MUL2
#define KGS_M32_ROWS_MUL2 8
#endif
static_assert(KGS_M32_ROWS <= 8 && KGS_M32_ROWS_MUL2 <= 8, "column bounds of fq29::reduce_row32");

namespace kgs {
namespace f29 {

constexpr uint32_t MASK = 0x1fffffffu;
constexpr uint32_t INV = 0x04866389u;    // -q^-1 mod 2^29
constexpr uint32_t INV32 = 0x24866389u;  // -q0^-1 mod 2^32 (q0 = Q.v[0]; = INV mod 2^29)
struct L9 {
  uint32_t v[9];
};
constexpr L9 Q = {{0x187cfd47u, 0x010460b6u, 0x1c72a34fu, 0x02d522d0u, 0x1585d978u, 0x02db40c0u, 0x00a6e141u,
                   0x0e5c2634u, 0x0030644eu}};
constexpr L9 ONE = {{0x157ccc21u, 0x141c2758u, 0x185230d3u, 0x014c0419u, 0x0aa36fb9u, 0x1d4240ceu, 0x11d54c07u,
                     0x052ac7a8u, 0x000dc836u}};  // 2^261 mod q
constexpr L9 C256 = {{0x058f0d9du, 0x1aea1c6eu, 0x11c2cf74u, 0x11d651ebu, 0x1462c0a7u, 0x11b7bc3cu, 0x1cbd99bau,
                      0x183340fbu, 0x000e0a77u}};  // 2^256 mod q: mul(x*2^261, C256) = x*2^256
constexpr L9 C266 = {{0x13349ca1u, 0x1a5d84a8u, 0x0a3e5cacu, 0x100249e0u, 0x12b951e8u, 0x0e92d304u, 0x14cb95b3u,
                      0x041b9d3du, 0x00058003u}};  // 2^266 mod q: mul(x*2^256, C266) = x*2^261
// 2^261 mod q as 8 x 32-bit words: fq (R = 2^256) product t * C261W turns x*2^256 into x*2^261
constexpr uint32_t C261W[8] = {0x157ccc21u, 0x4e8384ebu, 0x0ce148c3u, 0xfb90a602u,
                               0x819caa36u, 0x5301fa84u, 0x563d4475u, 0x0dc83629u};

// K = k*q with each limb j < 8 raised by s*2^29 (borrowed from limb j+1): same value, every limb
// >= s*2^29 - s, so a - b + K never underflows a limb when b's limbs are <= s*(2^29 - 1) + ...
constexpr L9 spread(uint32_t k, uint32_t s) {
  L9 r{};
  uint64_t carry = 0;
  for (int j = 0; j < 9; j++) {
    const uint64_t t = (uint64_t)Q.v[j] * k + carry;
    r.v[j] = j < 8 ? (uint32_t)(t & MASK) : (uint32_t)t;
    carry = t >> 29;
  }
  r.v[0] += s << 29;
  for (int j = 1; j < 8; j++) r.v[j] += (s << 29) - s;
  r.v[8] -= s;
  return r;
}

}  // namespace f29

struct fq29 {
  uint32_t l[9];

  __device__ __forceinline__ static fq29 from(const f29::L9& c) {
    fq29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = c.v[j];
    return r;
  }
  // 256-bit integer (8 x 32-bit words) -> 29-bit limbs, same value
  __device__ __forceinline__ static fq29 unpack(const uint32_t* w) {
    fq29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const int bit = 29 * j, i = bit >> 5, s = bit & 31;
      uint32_t x = w[i] >> s;
      if (s > 3 && i + 1 < 8) x |= w[i + 1] << (32 - s);
      r.l[j] = x & f29::MASK;
    }
    return r;
  }
  // normalised value < 2^256 -> 8 x 32-bit words
  __device__ __forceinline__ void pack(uint32_t* w) const {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int bit = 32 * i, j = bit / 29, s = bit % 29;
      uint32_t x = l[j] >> s;
      if (j + 1 < 9) x |= l[j + 1] << (29 - s);
      if (s > 26 && j + 2 < 9) x |= l[j + 2] << (58 - s);
      w[i] = x;
    }
  }
  // one carry pass: limbs < 2^29 (value < 2^261, limbs < 2^32 - 8 on entry)
  __device__ __forceinline__ fq29 norm() const {
    fq29 r;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint32_t s = l[j] + c;
      r.l[j] = j < 8 ? (s & f29::MASK) : s;
      c = s >> 29;
    }
    return r;
  }
  __device__ __forceinline__ static fq29 add(const fq29& a, const fq29& b) {
    fq29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = a.l[j] + b.l[j];
    return r;
  }
  // a + K - b (K = spread(k, s): every limb of K >= the matching limb of b)
  template <uint32_t K, uint32_t S>
  __device__ __forceinline__ static fq29 sub(const fq29& a, const fq29& b) {
    constexpr f29::L9 Kc = f29::spread(K, S);
    fq29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = (a.l[j] + Kc.v[j]) - b.l[j];
    return r;
  }
  // K - b
  template <uint32_t K, uint32_t S>
  __device__ __forceinline__ static fq29 neg(const fq29& b) {
    constexpr f29::L9 Kc = f29::spread(K, S);
    fq29 r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = Kc.v[j] - b.l[j];
    return r;
  }

  // CIOS output: 9 64-bit columns before the final carry pass (value = sum_j t_j 2^(29 j)). The
  // consumers either run the carry pass alone (carry) or fold an addition of a spread constant into it
  // (carry_sub): one normalisation instead of two where a product feeds a sum or difference.
  struct cols {
    uint64_t t[9];
  };
  // CIOS reduction step after row i's partial products: t += m*q (m = -t0/q mod 2^29), shift down
  __device__ __forceinline__ static void reduce_row(uint64_t (&t)[9]) {
    const uint32_t m = ((uint32_t)t[0] * f29::INV) & f29::MASK;
    const uint64_t c = ((uint64_t)m * f29::Q.v[0] + t[0]) >> 29;
#pragma unroll
    for (int j = 1; j < 9; j++) t[j] = (uint64_t)m * f29::Q.v[j] + t[j];
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = t[j + 1];
    t[0] += c;
    t[8] = 0;
  }
  // The same step with a 32-bit m = -t0/q0 mod 2^32 (no mask): t0 + m*q0 then has 32 zero low bits,
  // so its carry into the next column, (t0 + m*q0) >> 29, is 8 x its high word — one v_mad_u64_u32
  // (8 comes in an SGPR the compiler cannot fold into a shift) instead of a 64-bit shift, a 64-bit add
  // and the mask: 3 instead of 5 VALU per row. m < 2^32 adds < 2^(29 i + 32) q to the reduced value in
  // row i, so rows 0..7 take it (together < 2^-25 q over the 2^261 of the division) and row 8 keeps
  // the 29-bit m (the result stays < a*b/2^261 + q(1 + 2^-25)). Columns: mul/sqr of normalised
  // operands < 2^63.0 (outputs < 2^62.6, read as int64 by carry_sub); mul2 with add_aff's / add's
  // operand limb bounds < 2^64 — tests/test_field29.py re-derives every column bound row by row and
  // runs the exact row schedule on Python integers.
  __device__ __forceinline__ static void reduce_row32(uint64_t (&t)[9], uint32_t eight) {
    const uint32_t m = (uint32_t)t[0] * f29::INV32;
    const uint64_t u = (uint64_t)m * f29::Q.v[0] + t[0];
#pragma unroll
    for (int j = 1; j < 9; j++) t[j] = (uint64_t)m * f29::Q.v[j] + t[j];
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = t[j + 1];
    t[0] = (uint64_t)(uint32_t)(u >> 32) * eight + t[0];
    t[8] = 0;
  }
  // 8 as an opaque SGPR value (keeps reduce_row32's carry a v_mad_u64_u32)
  __device__ __forceinline__ static uint32_t opaque8() {
    uint32_t e = 8;
    asm volatile("" : "+s"(e));
    return e;
  }
  template <int M32_ROWS>
  __device__ __forceinline__ static void reduce_row_at(uint64_t (&t)[9], int i, uint32_t eight) {
    if (i < M32_ROWS) reduce_row32(t, eight); else reduce_row(t);
  }

  // Montgomery product a*b*2^-261 (CIOS, 64-bit column accumulators, no carry words).
  // Needs 9*max(a_j)*max(b_j) + 2^32 * sum(q_j) + 2^36 < 2^64 (a_j, b_j < 2^29; reduce_row32 in
  // rows 0..7) and a*b < 2^261 * (2^261 - q); the result is < a*b/2^261 + q(1 + 2^-25).
  __device__ __forceinline__ static cols mul_cols(const fq29& a, const fq29& b) {
    const uint32_t eight = opaque8();
    cols r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.t[j] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int j = 0; j < 9; j++) r.t[j] = (uint64_t)a.l[i] * b.l[j] + r.t[j];
      reduce_row_at<KGS_M32_ROWS>(r.t, i, eight);
    }
    return r;
  }

  // Montgomery square a*a*2^-261: the CIOS rows of mul with the symmetric partial products taken
  // once (2a_i * a_j, j > i, and a_i^2 on the diagonal): 45 + 81 mads instead of 162. Row i adds to
  // absolute columns 2i..i+8, which sit at t[i..8] after i shifts. A column receives at most 5
  // products (<= 2 * max(a_j)^2 each), so it stays below mul's bound for a normalised a.
  __device__ __forceinline__ static cols sqr_cols(const fq29& a) {
    const uint32_t eight = opaque8();
    uint32_t d[9];
#pragma unroll
    for (int j = 0; j < 9; j++) d[j] = a.l[j] << 1;
    cols r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.t[j] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
      r.t[i] = (uint64_t)a.l[i] * a.l[i] + r.t[i];
#pragma unroll
      for (int j = i + 1; j < 9; j++) r.t[j] = (uint64_t)d[i] * a.l[j] + r.t[j];
      reduce_row_at<KGS_M32_ROWS>(r.t, i, eight);
    }
    return r;
  }

  // (a*b + c*d)*2^-261 with ONE Montgomery reduction (lazy reduction of a sum of products): each CIOS
  // row adds both rows of partial products before its reduction step, 243 mads instead of 324.
  // Needs 9*(max a_j * max b_j + max c_j * max d_j) + 9*(2^29)^2 + 2^36 < 2^64 (a and c normalised)
  // and a*b + c*d < 2^261 * (2^261 - q); the result is < (a*b + c*d)/2^261 + q.
  __device__ __forceinline__ static cols mul2_cols(const fq29& a, const fq29& b, const fq29& c2, const fq29& d2) {
    const uint32_t eight = opaque8();
    cols r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.t[j] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int j = 0; j < 9; j++) r.t[j] = (uint64_t)a.l[i] * b.l[j] + r.t[j];
#pragma unroll
      for (int j = 0; j < 9; j++) r.t[j] = (uint64_t)c2.l[i] * d2.l[j] + r.t[j];
      reduce_row_at<KGS_M32_ROWS_MUL2>(r.t, i, eight);
    }
    return r;
  }

  // final carry pass: normalised limbs
  __device__ __forceinline__ static fq29 carry(const cols& x) {
    fq29 r;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t s = x.t[j] + c;
      r.l[j] = (uint32_t)s & f29::MASK;
      c = s >> 29;
    }
    return r;
  }
  // norm(x + K - b) in ONE carry pass (K = spread(k, s): every limb of K >= b's limb; x's columns
  // < 2^63, read as int64)
  template <uint32_t K, uint32_t S>
  __device__ __forceinline__ static fq29 carry_sub(const cols& x, const fq29& b) {
    constexpr f29::L9 Kc = f29::spread(K, S);
    fq29 r;
    int64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const int64_t s = (int64_t)(Kc.v[j] - b.l[j]) + (int64_t)x.t[j] + c;
      r.l[j] = j < 8 ? ((uint32_t)s & f29::MASK) : (uint32_t)s;
      c = s >> 29;
    }
    return r;
  }

  __device__ __forceinline__ static fq29 mul(const fq29& a, const fq29& b) { return carry(mul_cols(a, b)); }
  __device__ __forceinline__ static fq29 sqr(const fq29& a) { return carry(sqr_cols(a)); }
  __device__ __forceinline__ static fq29 mul2(const fq29& a, const fq29& b, const fq29& c2, const fq29& d2) {
    return carry(mul2_cols(a, b, c2, d2));
  }

  // necessary condition for "== 0 mod q" of a normalised value < 8q: its low limb is (j*q) mod 2^29
  // for some j < 8, i.e. l0 * q0^-1 mod 2^29 < 8 (q0 is odd; q0^-1 = -INV): 3 instructions
  __device__ __forceinline__ bool maybe_zero8() const {
    return ((l[0] * (0u - f29::INV)) & f29::MASK) < 8u;
  }
  // x*2^261 -> canonical fq (x*2^256), for a normalised value with value*2^253.6 < 2^261*q
  __device__ __forceinline__ fq to_fq() const {
    fq29 m = mul(*this, from(f29::C256));  // < 2q
    fq r;
    m.pack(r.v);
    return fq::reduce_once(r);
  }
  // canonical / lazy fq (x*2^256, < 2^256 and limbs unpacked < 2^29) -> x*2^261, normalised, < 2q
  __device__ __forceinline__ static fq29 from_fq(const fq& a) { return mul(unpack(a.v), from(f29::C266)); }
};

constexpr int RAW29_WORDS = 40;  // g1_acc29::store_raw / load_raw record

// Bucket accumulator in XYZZ over fq29 (coordinates < 2^258.6, normalised); infinity is a flag.
struct g1_acc29 {
  fq29 X, Y, ZZ, ZZZ;
  bool inf;

  __device__ __forceinline__ void set_inf() { inf = true; }

  // this += (x, +-y): x, y = table coordinates (x*2^261 mod q, canonical, packed words);
  // madd-2008-s with the same special cases as g1_xyzz::add_aff
  __device__ __forceinline__ void add_aff(const uint32_t* xw, const uint32_t* yw, bool negy) {
    uint32_t z = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) z |= xw[i] | yw[i];
    if (z == 0) return;  // affine infinity
    const fq29 x2 = fq29::unpack(xw), y2 = fq29::unpack(yw);
    if (inf) {
      X = x2;
      const fq29 yn = fq29::neg<2, 1>(y2).norm();
#pragma unroll
      for (int j = 0; j < 9; j++) Y.l[j] = negy ? yn.l[j] : y2.l[j];
      ZZ = fq29::from(f29::ONE);
      ZZZ = ZZ;
      inf = false;
      return;
    }
    // P = U2 - X1 with the product's carry pass folded into the difference's normalisation
    const fq29 P = fq29::carry_sub<30, 1>(fq29::mul_cols(x2, ZZ), X);
    const fq29 S2 = fq29::mul(y2, ZZZ);
    // R = S2 - Y1, or -S2 - Y1 for a negated point: K - Y1 +- S2 (limbs of K - Y1 >= 2^30 > S2's)
    fq29 R = fq29::neg<32, 2>(Y);
#pragma unroll
    for (int j = 0; j < 9; j++) R.l[j] = negy ? R.l[j] - S2.l[j] : R.l[j] + S2.l[j];
    R = R.norm();
    const fq29 PP = fq29::sqr(P);  // < 6.8 q
    if (PP.maybe_zero8()) {  // rare: decide exactly
      if (P.to_fq().is_zero()) {
        if (R.to_fq().is_zero()) {  // same point: doubling (256-bit path, converted back)
          g1_aff a;
          a.x = x2.to_fq();
          a.y = y2.to_fq();
          if (negy) a.y = a.y.neg();
          const g1_xyzz d = g1_xyzz::dbl_aff(a);
          X = fq29::from_fq(d.X);
          Y = fq29::from_fq(d.Y);
          ZZ = fq29::from_fq(d.ZZ);
          ZZZ = fq29::from_fq(d.ZZZ);
        } else {
          inf = true;  // opposite points
        }
        return;
      }
    }
    // ordered so that P, PP, ZZ, ZZZ and Qv die early: mul2 below has four operands live, and at
    // <= 168 VGPRs the kernel keeps 3 waves per SIMD without spilling
    const fq29 PPP = fq29::mul(P, PP);
    ZZ = fq29::mul(ZZ, PP);
    const fq29 Qv = fq29::mul(X, PP);
    ZZZ = fq29::mul(ZZZ, PPP);
    X = fq29::sub<16, 3>(fq29::sqr(R), fq29::add(PPP, fq29::add(Qv, Qv))).norm();
    const fq29 T = fq29::sub<64, 1>(Qv, X);
    // Y3 = R*T - Y1*PPP = R*T + Y1*(3q - PPP) mod q, one reduction (PPP < 2.3q)
    Y = fq29::mul2(R, T, Y, fq29::neg<3, 1>(PPP));
  }

  // this += o, both accumulators (add-2008-s; coordinates < 2^258.6, normalised): the bucket
  // combine and bit-sum trees. 10 products + 2 squares + the lazily reduced Y3. The CIOS rows give
  // 9 independent column chains, so a lone wave (these trees run at low occupancy) is far less
  // latency-bound than with the 8 x 32-bit product-scanning chain. Special cases as g1_xyzz::add;
  // the doubling (equal points, never met by distinct buckets in practice) goes through the 256-bit
  // path and is converted back.
  __device__ __forceinline__ void add(const g1_acc29& o) {
    if (o.inf) return;
    if (inf) {
      *this = o;
      return;
    }
    const fq29 U1 = fq29::mul(X, o.ZZ);
    const fq29 S1 = fq29::mul(Y, o.ZZZ);
    const fq29 P = fq29::carry_sub<8, 1>(fq29::mul_cols(o.X, ZZ), U1);   // U2 - U1
    const fq29 R = fq29::carry_sub<8, 1>(fq29::mul_cols(o.Y, ZZZ), S1);  // S2 - S1
    const fq29 PP = fq29::sqr(P);
    if (PP.maybe_zero8()) {
      if (P.to_fq().is_zero()) {
        if (R.to_fq().is_zero()) {
          *this = from_xyzz(to_xyzz().dbl());
        } else {
          inf = true;
        }
        return;
      }
    }
    const fq29 PPP = fq29::mul(P, PP);
    ZZ = fq29::mul(fq29::mul(ZZ, o.ZZ), PP);
    ZZZ = fq29::mul(fq29::mul(ZZZ, o.ZZZ), PPP);
    const fq29 Qv = fq29::mul(U1, PP);
    X = fq29::carry_sub<16, 3>(fq29::sqr_cols(R), fq29::add(PPP, fq29::add(Qv, Qv)));
    const fq29 T = fq29::sub<64, 1>(Qv, X);
    Y = fq29::mul2(R, T, S1, fq29::neg<3, 1>(PPP));  // R*T - S1*PPP
  }

  // canonical 256-bit-Montgomery XYZZ -> accumulator (coordinates < 2q, normalised)
  __device__ __forceinline__ static g1_acc29 from_xyzz(const g1_xyzz& p) {
    g1_acc29 a;
    a.inf = p.is_inf();
    a.X = fq29::from_fq(p.X);
    a.Y = fq29::from_fq(p.Y);
    a.ZZ = fq29::from_fq(p.ZZ);
    a.ZZZ = fq29::from_fq(p.ZZZ);
    return a;
  }

  // raw form: 4 x 9 limbs + infinity flag, padded to 40 words (16-byte stores)
  __device__ __forceinline__ void store_raw(uint32_t* p) const {
    uint32_t w[40];
#pragma unroll
    for (int j = 0; j < 9; j++) {
      w[j] = X.l[j];
      w[9 + j] = Y.l[j];
      w[18 + j] = ZZ.l[j];
      w[27 + j] = ZZZ.l[j];
    }
    w[36] = inf ? 1u : 0u;
    w[37] = w[38] = w[39] = 0;
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int k = 0; k < 10; k++) q[k] = make_uint4(w[4 * k], w[4 * k + 1], w[4 * k + 2], w[4 * k + 3]);
  }
  __device__ __forceinline__ static g1_acc29 load_raw(const uint32_t* p) {
    uint32_t w[40];
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int k = 0; k < 10; k++) {
      const uint4 v = q[k];
      w[4 * k] = v.x; w[4 * k + 1] = v.y; w[4 * k + 2] = v.z; w[4 * k + 3] = v.w;
    }
    g1_acc29 a;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      a.X.l[j] = w[j];
      a.Y.l[j] = w[9 + j];
      a.ZZ.l[j] = w[18 + j];
      a.ZZZ.l[j] = w[27 + j];
    }
    a.inf = w[36] != 0;
    return a;
  }

  // canonical 256-bit-Montgomery XYZZ (g1_xyzz::inf() for infinity)
  __device__ __forceinline__ g1_xyzz to_xyzz() const {
    if (inf) return g1_xyzz::inf();
    g1_xyzz r;
    r.X = X.to_fq();
    r.Y = Y.to_fq();
    r.ZZ = ZZ.to_fq();
    r.ZZZ = ZZZ.to_fq();
    return r;
  }
};

}  // namespace kgs
