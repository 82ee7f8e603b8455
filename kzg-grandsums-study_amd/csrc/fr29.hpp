// BN254 Fr products in 9 x 29-bit limbs for the NTT twiddle multiplications (device only).
//
// The NTT keeps its elements as 8 x 32-bit words (field.hpp `fr`, values in [0, 4p) lazily reduced,
// canonical at every pass boundary) and only its twiddle products go through this header. The 8 x 32
// product-scanning product (fr::mul_nored) is ONE dependent chain: every v_mad_u64_u32 reads the
// previous one's 64-bit sum and every mad needs a v_addc for the column's carry word (2 VALU per
// partial product). Here a CIOS product in 29-bit limbs takes one mad per partial product into 64-bit
// column accumulators with no carry words (a column's 9 products and 8 reduction terms stay below 2^64), and the 9
// columns are 9 independent chains: the same issue cycles for fewer instructions (~230 against ~300),
// and far more instruction-level parallelism for the NTT passes, which run at 2-3 waves per SIMD.
// The twiddle w comes pre-converted from the domain tables (ntt.hip k_tw29): w * 2^261 mod p,
// canonical, as 9 limbs in a 10-word record, so the product a * w * 2^261 * 2^-261 lands in the same
// Montgomery domain (R = 2^256) as a. Same reduction scheme as field29.hpp's fq29 (32-bit m in CIOS
// rows 0..7, one carry mad per row, 29-bit m in row 8); BN254's r is 1 + 2^28 mod 2^29, so
// -r^-1 mod 2^32 on the low limb is 2^28 - 1. Bounds (tests/test_fr29.py re-derives them and runs the
// exact row schedule on Python integers): for a < 2^256 (unpacked limbs < 2^29, top limb < 2^24) and
// w < p, every column stays < 2^63.14 (the m * P[j] terms dominate) and the result is < a*w/2^261 + p(1 + 2^-25) < 2p.
#pragma once
#include "field.hpp"

namespace kgs {
namespace r29 {
constexpr uint32_t MASK = 0x1fffffffu;
constexpr uint32_t P[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                           0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};  // r, 29-bit limbs
constexpr uint32_t INV = 0x0fffffffu;    // -r^-1 mod 2^29
constexpr uint32_t INV32 = 0x0fffffffu;  // -P[0]^-1 mod 2^32
constexpr int W29_WORDS = 10;            // twiddle record: 9 limbs + 1 pad (kernels.hpp TW29_WORDS)
// 32 * 2^256 mod r in 8 x 32-bit words (Montgomery form of 32): x * C32 turns x * 2^256 into x * 2^261
constexpr uint32_t C32[8] = {0x8fffff57u, 0x2fd4e156u, 0xa494b01au, 0x75bba827u,
                             0x819caa80u, 0x5301fa84u, 0x563d4475u, 0x0dc83629u};
// record of R^2 (2^517 mod r, 29-bit limbs): mul29(x, TO_MONT) = x * 2^256 mod r, the Montgomery form
constexpr uint32_t TO_MONT[9] = {0x142db4dfu, 0x19d6990eu, 0x1472f48cu, 0x06dbe7e3u, 0x0b84d579u,
                                 0x10f9faf7u, 0x121f4380u, 0x17a112deu, 0x001275c7u};
}  // namespace r29

struct W29 {
  uint32_t l[9];
};

__device__ __forceinline__ W29 w29_load(const uint32_t* p) {
  const uint4 a = *reinterpret_cast<const uint4*>(p);
  const uint4 b = *reinterpret_cast<const uint4*>(p + 4);
  W29 w;
  w.l[0] = a.x; w.l[1] = a.y; w.l[2] = a.z; w.l[3] = a.w;
  w.l[4] = b.x; w.l[5] = b.y; w.l[6] = b.z; w.l[7] = b.w;
  w.l[8] = p[8];
  return w;
}

// 8 x 32-bit words (value < 2^256) -> 9 x 29-bit limbs, same value
__device__ __forceinline__ void unpack29(const fr& a, uint32_t (&l)[9]) {
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const int bit = 29 * j, i = bit >> 5, s = bit & 31;
    uint32_t x = a.v[i] >> s;
    if (s > 3 && i + 1 < 8) x |= a.v[i + 1] << (32 - s);
    l[j] = x & r29::MASK;
  }
}

// a * w * 2^-261 mod p, in [0, 2p), for a < 2^256 (any representative) and w = a twiddle record
__device__ __forceinline__ fr mul29(const fr& A, const W29& w) {
  uint32_t a[9];
  unpack29(A, a);
  // SGPR operands the compiler cannot fold: the row carry (x 8) and m * P[0] (P[0] = 2^28 + 1) stay
  // single v_mad_u64_u32s instead of 64-bit shift-and-add sequences
  uint32_t eight = 8, p0 = r29::P[0];
  asm volatile("" : "+s"(eight), "+s"(p0));
  uint64_t t[9];
#pragma unroll
  for (int j = 0; j < 9; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j < 9; j++) t[j] = (uint64_t)a[i] * w.l[j] + t[j];
    if (i < 8) {  // 32-bit m: t0 + m P0 has 32 zero low bits, its carry is 8 x its high word
      const uint32_t m = (uint32_t)t[0] * r29::INV32;
      const uint64_t u = (uint64_t)m * p0 + t[0];
#pragma unroll
      for (int j = 1; j < 9; j++) t[j] = (uint64_t)m * r29::P[j] + t[j];
#pragma unroll
      for (int j = 0; j < 8; j++) t[j] = t[j + 1];
      t[0] = (uint64_t)(uint32_t)(u >> 32) * eight + t[0];
      t[8] = 0;
    } else {  // 29-bit m in the last row
      const uint32_t m = ((uint32_t)t[0] * r29::INV) & r29::MASK;
      const uint64_t c = ((uint64_t)m * p0 + t[0]) >> 29;
#pragma unroll
      for (int j = 1; j < 9; j++) t[j] = (uint64_t)m * r29::P[j] + t[j];
#pragma unroll
      for (int j = 0; j < 8; j++) t[j] = t[j + 1];
      t[0] += c;
      t[8] = 0;
    }
  }
  uint32_t l[9];
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const uint64_t s = t[j] + c;
    l[j] = j < 8 ? ((uint32_t)s & r29::MASK) : (uint32_t)s;
    c = s >> 29;
  }
  fr r;  // value < 2p < 2^255: pack the limbs into 8 words
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int bit = 32 * i, j = bit / 29, s = bit % 29;
    uint32_t x = l[j] >> s;
    if (j + 1 < 9) x |= l[j + 1] << (29 - s);
    if (s > 26 && j + 2 < 9) x |= l[j + 2] << (58 - s);
    r.v[i] = x;
  }
  return r;
}

}  // namespace kgs
