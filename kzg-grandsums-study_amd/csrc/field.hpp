// BN254 Fr / Fq Montgomery arithmetic for gfx950 (device) — 8 x 32-bit little-endian limbs.
//
// Representation: identical bytes to ffjavascript's in-memory form (32 B LE, Montgomery with
// R = 2^256), so ptau LEM points and caller buffers are used without conversion. Both moduli are
// < 2^254, which enables the "no-carry" CIOS variant (no t[N], t[N+1] words).
//
// Replaces the [ffjs] wasm field (`curve.Fr.*`, `curve.F1.*`) on the hot path.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kgs {

struct FqP {
  static constexpr uint32_t p[8] = {0xd87cfd47u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t inv = 0xe4866389u;  // -p^-1 mod 2^32
  static constexpr uint32_t one[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                                      0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t r2[8] = {0x538afa89u, 0xf32cfc5bu, 0xd44501fbu, 0xb5e71911u,
                                     0x0a417ff6u, 0x47ab1effu, 0xcab8351fu, 0x06d89f71u};
};

struct FrP {
  static constexpr uint32_t p[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                                    0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  static constexpr uint32_t inv = 0xefffffffu;
  static constexpr uint32_t one[8] = {0x4ffffffbu, 0xac96341cu, 0x9f60cd29u, 0x36fc7695u,
                                      0x7879462eu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
  static constexpr uint32_t r2[8] = {0xae216da7u, 0x1bb8e645u, 0xe35c59e3u, 0x53fe3ab1u,
                                     0x53bb8085u, 0x8c49833du, 0x7f4e44a5u, 0x0216d0b1u};
};

template <class P>
struct Fe {
  uint32_t v[8];

  __device__ __forceinline__ static Fe zero() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = 0;
    return r;
  }
  __device__ __forceinline__ static Fe one() {
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = P::one[i];
    return r;
  }
  __device__ __forceinline__ bool is_zero() const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i];
    return acc == 0;
  }
  __device__ __forceinline__ bool operator==(const Fe& o) const {
    uint32_t acc = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) acc |= v[i] ^ o.v[i];
    return acc == 0;
  }
  __device__ __forceinline__ bool operator!=(const Fe& o) const { return !(*this == o); }

  // Carry chains use __builtin_addc / __builtin_subc (v_add_co/v_addc_co/v_sub_co/v_subb_co with
  // VCC): ~24 VALU per modular add/sub, versus the ~37 (64-bit v_lshl_add_u64 adds + shifts +
  // moves) the compiler emits for the same limb loop written with 64-bit temporaries; measured
  // +11 % proofs/s (bucket accumulation 1.83 -> 1.64 ms per 2^20-point MSM).
  // r = a - p if a >= p (a < 2p)
  __device__ __forceinline__ static Fe reduce_once(const Fe& a) {
    Fe d;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(a.v[i], P::p[i], borrow, &borrow);
    Fe r;
#pragma unroll
    for (int i = 0; i < 8; i++) r.v[i] = borrow ? a.v[i] : d.v[i];
    return r;
  }

  __device__ __forceinline__ friend Fe operator+(const Fe& a, const Fe& b) {
    Fe s;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);
    return reduce_once(s);
  }

  __device__ __forceinline__ friend Fe operator-(const Fe& a, const Fe& b) {
    Fe d;
    uint32_t borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(a.v[i], b.v[i], borrow, &borrow);
    Fe e;
    uint32_t c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) e.v[i] = __builtin_addc(d.v[i], P::p[i], c, &c);
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = borrow ? e.v[i] : d.v[i];
    return d;
  }

  __device__ __forceinline__ Fe neg() const { return is_zero() ? *this : (zero() - *this); }
  __device__ __forceinline__ Fe dbl() const { return *this + *this; }

  // Montgomery product, product-scanning ("FIPS") order. Each 32x32 partial product is ONE
  // v_mad_u64_u32 accumulating into the running 64-bit column sum, whose carry-out feeds ONE
  // v_addc_co_u32 into the third accumulator word: 2 VALU instructions per partial product
  // (128 quarter-rate mads + 128 full-rate addc), versus ~5 when the 64-bit addends are built
  // by the compiler (measured 107.8 vs 76.5 G products/s on MI355X). Valid for p < 2^254:
  // the result is < 2p and fits 8 limbs before the final conditional subtraction.
  __device__ __forceinline__ static void mac(uint64_t& acc, uint32_t& t2, uint32_t x, uint32_t y) {
    uint64_t c;
#ifdef KGS_MAC_NOP
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\ts_nop 1\n\tv_addc_co_u32 %1, %2, 0, %1, %2"
                 : "+v"(acc), "+v"(t2), "=&s"(c)
                 : "v"(x), "v"(y));
#else
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32 %1, %2, 0, %1, %2"
                 : "+v"(acc), "+v"(t2), "=&s"(c)
                 : "v"(x), "v"(y));
#endif
  }
  // Two chained macs (a_j*b_{i-j}, then m_j*p_{i-j} into the same column) in ONE asm block: the
  // compiler pads every boundary between asm blocks after a carry-writing VALU with an s_nop, so
  // pairing halves those pads (measured: bucket reduction -10 %, single-proof latency -3.5 %).
  // Hazards: inside the block each v_addc reads the carry SGPR written by the v_mad_u64_u32 just
  // before it and the next v_mad follows an SGPR-writing v_addc without a wait state; the 8-cycle
  // quarter-rate mad covers the first, and every GPU parity test (bit-exact products inside
  // millions of MSM additions, 2^20-2^22 proofs that verify, repeated-proof determinism) runs on
  // this code. -DKGS_MAC_NOP builds the padded variant (s_nop 1 after each mad) for comparison.
  __device__ __forceinline__ static void mac2(uint64_t& acc, uint32_t& t2, uint32_t x0, uint32_t y0, uint32_t x1,
                                              uint32_t y1) {
#ifdef KGS_MAC_NOP
    mac(acc, t2, x0, y0);
    mac(acc, t2, x1, y1);
#else
    uint64_t c0, c1;
    asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_addc_co_u32 %1, %2, 0, %1, %2\n\t"
        "v_mad_u64_u32 %0, %3, %6, %7, %0\n\tv_addc_co_u32 %1, %3, 0, %1, %3"
        : "+v"(acc), "+v"(t2), "=&s"(c0), "=&s"(c1)
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
#endif
  }
  // first mac(s) of a column: the carry word is WRITTEN (0 + 0 + carry), saving its zeroing move
  __device__ __forceinline__ static void mac_init(uint64_t& acc, uint32_t& t2, uint32_t x, uint32_t y) {
    uint64_t c;
    asm("v_mad_u64_u32 %0, %2, %3, %4, %0\n\tv_addc_co_u32 %1, %2, 0, 0, %2"
        : "+v"(acc), "=v"(t2), "=&s"(c)
        : "v"(x), "v"(y));
  }
  __device__ __forceinline__ static void mac2_init(uint64_t& acc, uint32_t& t2, uint32_t x0, uint32_t y0, uint32_t x1,
                                                   uint32_t y1) {
    uint64_t c0, c1;
    asm("v_mad_u64_u32 %0, %2, %4, %5, %0\n\tv_addc_co_u32 %1, %2, 0, 0, %2\n\t"
        "v_mad_u64_u32 %0, %3, %6, %7, %0\n\tv_addc_co_u32 %1, %3, 0, %1, %3"
        : "+v"(acc), "=&v"(t2), "=&s"(c0), "=&s"(c1)
        : "v"(x0), "v"(y0), "v"(x1), "v"(y1));
  }
  // product in [0, 2p) for inputs in [0, 2p) (p < 2^254, so 4p < R = 2^256)
  __device__ __forceinline__ static Fe mul_nored(const Fe& A, const Fe& B) {
    const uint32_t* a = A.v;
    const uint32_t* b = B.v;
    uint32_t m[8];
    Fe r;
    uint64_t acc = 0;
    uint32_t t2;  // carry word of the current column: written (not accumulated) by its first mac
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (i == 0) {
        mac_init(acc, t2, a[0], b[0]);
      } else {
        mac2_init(acc, t2, a[0], b[i], m[0], P::p[i]);
#pragma unroll
        for (int j = 1; j < i; j++) mac2(acc, t2, a[j], b[i - j], m[j], P::p[i - j]);
        mac(acc, t2, a[i], b[0]);
      }
      m[i] = (uint32_t)acc * P::inv;
      mac(acc, t2, m[i], P::p[0]);
      acc = (acc >> 32) | ((uint64_t)t2 << 32);
    }
#pragma unroll
    for (int i = 8; i < 15; i++) {
      mac2_init(acc, t2, a[i - 7], b[7], m[i - 7], P::p[7]);
#pragma unroll
      for (int j = i - 6; j < 8; j++) mac2(acc, t2, a[j], b[i - j], m[j], P::p[i - j]);
      r.v[i - 8] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)t2 << 32);
    }
    r.v[7] = (uint32_t)acc;
    return r;
  }

  // Two independent products with their instruction streams interleaved: every asm block carries
  // the same two column terms of BOTH products (mad A, mad B, addc A, addc B, ...), so the serial
  // accumulator chain of one product issues between the links of the other. A single product is one
  // dependent chain (each mad reads the previous mad's 64-bit sum); at the 2 waves per SIMD of the
  // NTT passes that chain, not the issue rate, set the pace.
  __device__ __forceinline__ static void mac_x2(uint64_t& accA, uint32_t& tA, uint32_t xA, uint32_t yA, uint64_t& accB,
                                                uint32_t& tB, uint32_t xB, uint32_t yB) {
    uint64_t cA, cB;
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
        "v_addc_co_u32 %1, %4, 0, %1, %4\n\tv_addc_co_u32 %3, %5, 0, %3, %5"
        : "+v"(accA), "+v"(tA), "+v"(accB), "+v"(tB), "=&s"(cA), "=&s"(cB)
        : "v"(xA), "v"(yA), "v"(xB), "v"(yB));
  }
  __device__ __forceinline__ static void mac_x2_init(uint64_t& accA, uint32_t& tA, uint32_t xA, uint32_t yA,
                                                     uint64_t& accB, uint32_t& tB, uint32_t xB, uint32_t yB) {
    uint64_t cA, cB;
    asm("v_mad_u64_u32 %0, %4, %6, %7, %0\n\tv_mad_u64_u32 %2, %5, %8, %9, %2\n\t"
        "v_addc_co_u32 %1, %4, 0, 0, %4\n\tv_addc_co_u32 %3, %5, 0, 0, %5"
        : "+v"(accA), "=&v"(tA), "+v"(accB), "=&v"(tB), "=&s"(cA), "=&s"(cB)
        : "v"(xA), "v"(yA), "v"(xB), "v"(yB));
  }
  // two terms of one column of each product (a_j b_k and m_j p_k of A, the same of B)
  __device__ __forceinline__ static void mac2_x2(uint64_t& accA, uint32_t& tA, uint32_t xA0, uint32_t yA0, uint32_t xA1,
                                                 uint32_t yA1, uint64_t& accB, uint32_t& tB, uint32_t xB0, uint32_t yB0,
                                                 uint32_t xB1, uint32_t yB1) {
    uint64_t cA0, cB0, cA1, cB1;
    asm("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %2, %5, %12, %13, %2\n\t"
        "v_addc_co_u32 %1, %4, 0, %1, %4\n\tv_addc_co_u32 %3, %5, 0, %3, %5\n\t"
        "v_mad_u64_u32 %0, %6, %10, %11, %0\n\tv_mad_u64_u32 %2, %7, %14, %15, %2\n\t"
        "v_addc_co_u32 %1, %6, 0, %1, %6\n\tv_addc_co_u32 %3, %7, 0, %3, %7"
        : "+v"(accA), "+v"(tA), "+v"(accB), "+v"(tB), "=&s"(cA0), "=&s"(cB0), "=&s"(cA1), "=&s"(cB1)
        : "v"(xA0), "v"(yA0), "v"(xA1), "v"(yA1), "v"(xB0), "v"(yB0), "v"(xB1), "v"(yB1));
  }
  __device__ __forceinline__ static void mac2_x2_init(uint64_t& accA, uint32_t& tA, uint32_t xA0, uint32_t yA0,
                                                      uint32_t xA1, uint32_t yA1, uint64_t& accB, uint32_t& tB,
                                                      uint32_t xB0, uint32_t yB0, uint32_t xB1, uint32_t yB1) {
    uint64_t cA0, cB0, cA1, cB1;
    asm("v_mad_u64_u32 %0, %4, %8, %9, %0\n\tv_mad_u64_u32 %2, %5, %12, %13, %2\n\t"
        "v_addc_co_u32 %1, %4, 0, 0, %4\n\tv_addc_co_u32 %3, %5, 0, 0, %5\n\t"
        "v_mad_u64_u32 %0, %6, %10, %11, %0\n\tv_mad_u64_u32 %2, %7, %14, %15, %2\n\t"
        "v_addc_co_u32 %1, %6, 0, %1, %6\n\tv_addc_co_u32 %3, %7, 0, %3, %7"
        : "+v"(accA), "=&v"(tA), "+v"(accB), "=&v"(tB), "=&s"(cA0), "=&s"(cB0), "=&s"(cA1), "=&s"(cB1)
        : "v"(xA0), "v"(yA0), "v"(xA1), "v"(yA1), "v"(xB0), "v"(yB0), "v"(xB1), "v"(yB1));
  }
  // RA = A*B*R^-1, RB = C*D*R^-1, each in [0, 2p) for inputs in [0, 2p): mul_nored twice, interleaved.
  // The outputs must not alias the inputs (mul_nored_x2_ip for X *= B, Y *= D).
  __device__ __forceinline__ static void mul_nored_x2(const Fe& A, const Fe& B, const Fe& C, const Fe& D, Fe& RA,
                                                      Fe& RB) {
    const uint32_t *a = A.v, *b = B.v, *c = C.v, *d = D.v;
    uint32_t m[8], n[8];
    uint64_t acc = 0, acd = 0;
    uint32_t ta, tc;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (i == 0) {
        mac_x2_init(acc, ta, a[0], b[0], acd, tc, c[0], d[0]);
      } else {
        mac2_x2_init(acc, ta, a[0], b[i], m[0], P::p[i], acd, tc, c[0], d[i], n[0], P::p[i]);
#pragma unroll
        for (int j = 1; j < i; j++)
          mac2_x2(acc, ta, a[j], b[i - j], m[j], P::p[i - j], acd, tc, c[j], d[i - j], n[j], P::p[i - j]);
        mac_x2(acc, ta, a[i], b[0], acd, tc, c[i], d[0]);
      }
      m[i] = (uint32_t)acc * P::inv;
      n[i] = (uint32_t)acd * P::inv;
      mac_x2(acc, ta, m[i], P::p[0], acd, tc, n[i], P::p[0]);
      acc = (acc >> 32) | ((uint64_t)ta << 32);
      acd = (acd >> 32) | ((uint64_t)tc << 32);
    }
#pragma unroll
    for (int i = 8; i < 15; i++) {
      mac2_x2_init(acc, ta, a[i - 7], b[7], m[i - 7], P::p[7], acd, tc, c[i - 7], d[7], n[i - 7], P::p[7]);
#pragma unroll
      for (int j = i - 6; j < 8; j++)
        mac2_x2(acc, ta, a[j], b[i - j], m[j], P::p[i - j], acd, tc, c[j], d[i - j], n[j], P::p[i - j]);
      RA.v[i - 8] = (uint32_t)acc;
      RB.v[i - 8] = (uint32_t)acd;
      acc = (acc >> 32) | ((uint64_t)ta << 32);
      acd = (acd >> 32) | ((uint64_t)tc << 32);
    }
    RA.v[7] = (uint32_t)acc;
    RB.v[7] = (uint32_t)acd;
  }

  __device__ __forceinline__ static void mul_nored_x2_ip(Fe& X, const Fe& B, Fe& Y, const Fe& D) {
    const Fe a = X, c = Y;
    mul_nored_x2(a, B, c, D, X, Y);
  }

  __device__ __forceinline__ friend Fe operator*(const Fe& A, const Fe& B) { return reduce_once(mul_nored(A, B)); }

  __device__ __forceinline__ Fe sqr() const { return (*this) * (*this); }

  // ---- lazy reduction on [0, 2p): the bucket-accumulation chain keeps its point in this range
  // (one conditional subtraction per product saved) and canonicalises once per emitted run
  __device__ __forceinline__ static constexpr uint32_t p2(int i) {
    return (P::p[i] << 1) | (i ? P::p[i - 1] >> 31 : 0u);
  }
  __device__ __forceinline__ static Fe add_lazy(const Fe& a, const Fe& b) {
    Fe s, d;
    uint32_t c = 0, borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_addc(a.v[i], b.v[i], c, &c);  // < 4p < 2^256
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(s.v[i], p2(i), borrow, &borrow);
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = borrow ? s.v[i] : d.v[i];
    return s;
  }
  __device__ __forceinline__ static Fe sub_lazy(const Fe& a, const Fe& b) {
    Fe d, e;
    uint32_t borrow = 0, c = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = __builtin_subc(a.v[i], b.v[i], borrow, &borrow);
#pragma unroll
    for (int i = 0; i < 8; i++) e.v[i] = __builtin_addc(d.v[i], p2(i), c, &c);
#pragma unroll
    for (int i = 0; i < 8; i++) d.v[i] = borrow ? e.v[i] : d.v[i];
    return d;
  }
  // a - b + 2p in (0, 4p) for a, b in [0, 2p), no conditional correction: a multiplicand of
  // mul_nored (whose product is still < 2p when the other factor is < p: 4p * p / 2^256 < 0.76 p)
  __device__ __forceinline__ static Fe sub_2p(const Fe& a, const Fe& b) {
    Fe s;
    uint32_t c = 0, borrow = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_addc(a.v[i], p2(i), c, &c);
#pragma unroll
    for (int i = 0; i < 8; i++) s.v[i] = __builtin_subc(s.v[i], b.v[i], borrow, &borrow);
    return s;
  }
  __device__ __forceinline__ bool is_zero_lazy() const {  // == 0 mod p for a value in [0, 2p)
    uint32_t z = 0, q = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      z |= v[i];
      q |= v[i] ^ P::p[i];
    }
    return z == 0 || q == 0;
  }
  __device__ __forceinline__ Fe canon() const { return reduce_once(*this); }

  __device__ __forceinline__ Fe to_mont() const {
    Fe r2;
#pragma unroll
    for (int i = 0; i < 8; i++) r2.v[i] = P::r2[i];
    return (*this) * r2;
  }
  // a * R^-1: the Montgomery product with b = 1 (a * 1 * R^-1) without its zero partial products —
  // column i holds a_i * 1 and the m_j p_{i-j}: 72 macs instead of mul_nored's 128, the same column
  // sums, so the same result (the MSM digit passes convert every scalar twice)
  __device__ __forceinline__ Fe from_mont() const {
    const uint32_t* a = v;
    uint32_t one = 1;
    asm volatile("" : "+v"(one));  // a register operand (keeps the asm macs' operand kinds)
    uint32_t m[8];
    Fe r;
    uint64_t acc = 0;
    uint32_t t2;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      mac_init(acc, t2, a[i], one);
      int j = 0;
#pragma unroll
      for (; j + 1 < i; j += 2) mac2(acc, t2, m[j], P::p[i - j], m[j + 1], P::p[i - j - 1]);
      if (j < i) mac(acc, t2, m[j], P::p[i - j]);
      m[i] = (uint32_t)acc * P::inv;
      mac(acc, t2, m[i], P::p[0]);
      acc = (acc >> 32) | ((uint64_t)t2 << 32);
    }
#pragma unroll
    for (int i = 8; i < 15; i++) {
      int j = i - 7;
      mac_init(acc, t2, m[j], P::p[i - j]);
      j++;
#pragma unroll
      for (; j + 1 < 8; j += 2) mac2(acc, t2, m[j], P::p[i - j], m[j + 1], P::p[i - j - 1]);
      if (j < 8) mac(acc, t2, m[j], P::p[i - j]);
      r.v[i - 8] = (uint32_t)acc;
      acc = (acc >> 32) | ((uint64_t)t2 << 32);
    }
    r.v[7] = (uint32_t)acc;
    return reduce_once(r);
  }

  // a^(p-2) (Fermat); 0 -> 0. Latency-heavy: use only off the critical path / once per tile.
  // Binary extended Euclid on the integer value (branchy: meant for ONE active lane, e.g. the
  // single inversion of a batch-inversion tree; ~25 K VALU instead of Fermat's ~330 products).
  // x = this (Montgomery, aR) -> (aR)^-1 -> times R^2 twice -> a^-1 R (Montgomery). 0 -> 0.
  __device__ Fe inverse_bgcd() const {
    if (is_zero()) return *this;
    uint32_t u[8], v[8], x1[8], x2[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      u[i] = v_at(i);
      v[i] = P::p[i];
      x1[i] = i == 0 ? 1u : 0u;
      x2[i] = 0u;
    }
    auto is_one = [](const uint32_t* a) {
      uint32_t o = a[0] ^ 1u;
      for (int i = 1; i < 8; i++) o |= a[i];
      return o == 0;
    };
    auto shr1 = [](uint32_t* a, uint32_t top) {  // a = (top:a) >> 1
      for (int i = 0; i < 7; i++) a[i] = (a[i] >> 1) | (a[i + 1] << 31);
      a[7] = (a[7] >> 1) | (top << 31);
    };
    auto halve = [&](uint32_t* x) {  // x / 2 mod p (x < p)
      uint32_t c = 0;
      if (x[0] & 1u) {
        for (int i = 0; i < 8; i++) x[i] = __builtin_addc(x[i], P::p[i], c, &c);
      }
      shr1(x, c);
    };
    auto sub_mod = [&](uint32_t* a, const uint32_t* b) {  // a = a - b mod p
      uint32_t bo = 0, c = 0;
      for (int i = 0; i < 8; i++) a[i] = __builtin_subc(a[i], b[i], bo, &bo);
      if (bo)
        for (int i = 0; i < 8; i++) a[i] = __builtin_addc(a[i], P::p[i], c, &c);
    };
    while (!is_one(u) && !is_one(v)) {
      while (!(u[0] & 1u)) {
        shr1(u, 0);
        halve(x1);
      }
      while (!(v[0] & 1u)) {
        shr1(v, 0);
        halve(x2);
      }
      uint32_t d[8], bo = 0;
      for (int i = 0; i < 8; i++) d[i] = __builtin_subc(u[i], v[i], bo, &bo);
      if (!bo) {  // u >= v
        for (int i = 0; i < 8; i++) u[i] = d[i];
        sub_mod(x1, x2);
      } else {
        bo = 0;
        for (int i = 0; i < 8; i++) v[i] = __builtin_subc(v[i], u[i], bo, &bo);
        sub_mod(x2, x1);
      }
    }
    Fe r;
    for (int i = 0; i < 8; i++) r.v[i] = is_one(u) ? x1[i] : x2[i];
    Fe r2;
#pragma unroll
    for (int i = 0; i < 8; i++) r2.v[i] = P::r2[i];
    return (r * r2) * r2;
  }
  __device__ __forceinline__ uint32_t v_at(int i) const { return v[i]; }

  __device__ Fe inverse() const {
    // exponent e = p - 2, scanned from the top bit, 4-bit fixed windows
    Fe tbl[16];
    tbl[0] = one();
    tbl[1] = *this;
#pragma unroll
    for (int i = 2; i < 16; i++) tbl[i] = tbl[i - 1] * (*this);
    Fe r = one();
    for (int w = 63; w >= 0; w--) {
      const int limb = w >> 3, sh = (w & 7) * 4;
      uint32_t e = P::p[limb];
      if (limb == 0) e -= 2;  // p - 2 (no borrow: p[0] >= 2 for both moduli)
      uint32_t d = (e >> sh) & 15u;
      r = r.sqr();
      r = r.sqr();
      r = r.sqr();
      r = r.sqr();
      if (d) {
        Fe m = tbl[0];
        for (int k = 1; k < 16; k++)
          if ((uint32_t)k == d) m = tbl[k];
        r = r * m;
      }
    }
    return r;
  }

  __device__ __forceinline__ static Fe load(const uint32_t* p) {
    Fe r;
    const uint4* q = reinterpret_cast<const uint4*>(p);
    uint4 a = q[0], b = q[1];
    r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
    r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
    return r;
  }
  __device__ __forceinline__ void store(uint32_t* p) const {
    uint4* q = reinterpret_cast<uint4*>(p);
    q[0] = make_uint4(v[0], v[1], v[2], v[3]);
    q[1] = make_uint4(v[4], v[5], v[6], v[7]);
  }
};

using fr = Fe<FrP>;
using fq = Fe<FqP>;

// ------------------------------------------------------------------------------------- G1
// Affine storage: 64 B (x||y, Montgomery Fq) == ptau LEM; infinity == (0,0).
struct g1_aff {
  fq x, y;
  __device__ __forceinline__ bool is_inf() const { return x.is_zero() && y.is_zero(); }
  __device__ __forceinline__ static g1_aff load(const uint32_t* p) {
    g1_aff a;
    a.x = fq::load(p);
    a.y = fq::load(p + 8);
    return a;
  }
};

// XYZZ coordinates: x = X/ZZ, y = Y/ZZZ; infinity <=> ZZ == 0.
struct g1_xyzz {
  fq X, Y, ZZ, ZZZ;

  __device__ __forceinline__ static g1_xyzz inf() {
    g1_xyzz r;
    r.X = fq::one(); r.Y = fq::one(); r.ZZ = fq::zero(); r.ZZZ = fq::zero();
    return r;
  }
  __device__ __forceinline__ bool is_inf() const { return ZZ.is_zero(); }
  __device__ __forceinline__ static g1_xyzz from_aff(const g1_aff& a) {
    if (a.is_inf()) return inf();
    g1_xyzz r;
    r.X = a.x; r.Y = a.y; r.ZZ = fq::one(); r.ZZZ = fq::one();
    return r;
  }
  __device__ __forceinline__ static g1_xyzz load(const uint32_t* p) {
    g1_xyzz r;
    r.X = fq::load(p); r.Y = fq::load(p + 8); r.ZZ = fq::load(p + 16); r.ZZZ = fq::load(p + 24);
    return r;
  }
  __device__ __forceinline__ void store(uint32_t* p) const {
    X.store(p); Y.store(p + 8); ZZ.store(p + 16); ZZZ.store(p + 24);
  }

  // dbl-2008-s-1 (a = 0)
  __device__ __forceinline__ g1_xyzz dbl() const {
    if (is_inf()) return *this;
    fq U = Y.dbl();
    fq V = U.sqr();
    fq W = U * V;
    fq S = X * V;
    fq X2 = X.sqr();
    fq M = X2.dbl() + X2;
    g1_xyzz r;
    r.X = M.sqr() - S.dbl();
    r.Y = M * (S - r.X) - W * Y;
    r.ZZ = V * ZZ;
    r.ZZZ = W * ZZZ;
    return r;
  }

  // mdbl-2008-s-1: 2*affine
  __device__ __forceinline__ static g1_xyzz dbl_aff(const g1_aff& a) {
    fq U = a.y.dbl();
    fq V = U.sqr();
    fq W = U * V;
    fq S = a.x * V;
    fq X2 = a.x.sqr();
    fq M = X2.dbl() + X2;
    g1_xyzz r;
    r.X = M.sqr() - S.dbl();
    r.Y = M * (S - r.X) - W * a.y;
    r.ZZ = V;
    r.ZZZ = W;
    return r;
  }

  // madd-2008-s: this += affine (handles infinity / equal / opposite)
  __device__ __forceinline__ void add_aff(const g1_aff& a) {
    if (a.is_inf()) return;
    if (is_inf()) { *this = from_aff(a); return; }
    fq U2 = a.x * ZZ;
    fq S2 = a.y * ZZZ;
    fq P = U2 - X;
    fq R = S2 - Y;
    if (P.is_zero()) {
      if (R.is_zero()) { *this = dbl_aff(a); return; }
      *this = inf();
      return;
    }
    fq PP = P.sqr();
    fq PPP = P * PP;
    fq Qv = X * PP;
    fq nX = R.sqr() - PPP - Qv.dbl();
    Y = R * (Qv - nX) - Y * PPP;
    X = nX;
    ZZ = ZZ * PP;
    ZZZ = ZZZ * PPP;
  }

  // madd-2008-s with the accumulator kept lazily reduced (coordinates in [0, 2q)); the affine
  // input is canonical. Same special cases as add_aff. Call canon() before storing.
  __device__ __forceinline__ void add_aff_lazy(const g1_aff& a) {
    if (a.is_inf()) return;
    if (is_inf()) { *this = from_aff(a); return; }
    fq U2 = fq::mul_nored(a.x, ZZ);
    fq S2 = fq::mul_nored(a.y, ZZZ);
    fq P = fq::sub_lazy(U2, X);
    fq R = fq::sub_lazy(S2, Y);
    if (P.is_zero_lazy()) {
      if (R.is_zero_lazy()) { *this = dbl_aff(a); return; }
      *this = inf();
      return;
    }
    fq PP = fq::mul_nored(P, P);
    fq PPP = fq::mul_nored(P, PP);
    fq Qv = fq::mul_nored(X, PP);
    fq nX = fq::sub_lazy(fq::sub_lazy(fq::mul_nored(R, R), PPP), fq::add_lazy(Qv, Qv));
    Y = fq::sub_lazy(fq::mul_nored(R, fq::sub_lazy(Qv, nX)), fq::mul_nored(Y, PPP));
    X = nX;
    ZZ = fq::mul_nored(ZZ, PP);
    ZZZ = fq::mul_nored(ZZZ, PPP);
  }
  __device__ __forceinline__ void canon() {
    X = X.canon(); Y = Y.canon(); ZZ = ZZ.canon(); ZZZ = ZZZ.canon();
  }

  // add-2008-s: this += other
  __device__ __forceinline__ void add(const g1_xyzz& o) {
    if (o.is_inf()) return;
    if (is_inf()) { *this = o; return; }
    fq U1 = X * o.ZZ;
    fq U2 = o.X * ZZ;
    fq S1 = Y * o.ZZZ;
    fq S2 = o.Y * ZZZ;
    fq P = U2 - U1;
    fq R = S2 - S1;
    if (P.is_zero()) {
      if (R.is_zero()) { *this = dbl(); return; }
      *this = inf();
      return;
    }
    fq PP = P.sqr();
    fq PPP = P * PP;
    fq Qv = U1 * PP;
    fq nX = R.sqr() - PPP - Qv.dbl();
    Y = R * (Qv - nX) - S1 * PPP;
    X = nX;
    ZZ = ZZ * o.ZZ * PP;
    ZZZ = ZZZ * o.ZZZ * PPP;
  }
};

}  // namespace kgs
