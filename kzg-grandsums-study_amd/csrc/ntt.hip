// BN254-Fr NTT for gfx950 — replaces [ffjs] `Fr.fft` / `Fr.ifft` (polynomial.js:34,373,392,
// evaluations.js:18).
//
// Layout: 32 B Montgomery elements, AoS. The transform is a sequence of radix-2^K passes
// (K <= 3, eight elements per thread in registers), each pass reading and writing every element
// once. Forward = decimation-in-frequency (natural in -> bit-reversed out); inverse =
// decimation-in-time (bit-reversed in -> natural out). Pointwise work between the two (coset
// quotient evaluation) runs in bit-reversed order, so no permutation pass is needed on the
// convolution path; a natural-order input to the inverse is gathered through bit reversal inside
// the first pass. Coset scaling / 1/m scaling are fused into the first / last pass.
//
// Arithmetic: butterflies run on values in [0, 2p) (lazy reduction, fr::add_lazy / sub_lazy /
// sub_2p / mul_nored): one conditional correction per sum or difference and none after a product;
// every pass stores canonical values, so the output is bit-identical to a canonical-arithmetic
// network. -DKGS_NTT_CANON builds the canonical butterflies (A/B). Since round 5 the LDS passes
// multiply by 29-bit records of their twiddles and scalings (fr29.hpp mul29: the domain's twin
// tables, same [0, 2p) contract); KGS_NTT_T29=0 selects the 8 x 32-bit products.
//
// Twiddles: per direction one resident STAGE table tw[h + t] = w_{2h}^t (t < h, h = 1..M/2; M
// entries for the largest domain M), so the butterflies of one stage read consecutive twiddles
// (coalesced: consecutive lanes have consecutive t) instead of a strided walk through w_M^j.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <utility>

#include "fr29.hpp"
#include "kernels.hpp"

namespace kgs {

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) {
  return __builtin_bitreverse32(x) >> (32 - bits);
}

#ifndef KGS_NTT_CANON
// DIF butterfly (a, b) -> (a + b, (a - b) w), t == 0: w = 1; inputs and outputs in [0, 2p)
__device__ __forceinline__ void bfly_dif(fr& x0, fr& x1, const uint32_t* w, bool tw) {
  const fr a = x0, b = x1;
  x0 = fr::add_lazy(a, b);
  x1 = tw ? fr::mul_nored(fr::sub_2p(a, b), fr::load(w)) : fr::sub_lazy(a, b);
}
// DIT butterfly (a, b) -> (a + b w, a - b w); inputs and outputs in [0, 2p)
__device__ __forceinline__ void bfly_dit(fr& x0, fr& x1, const uint32_t* w, bool tw) {
  const fr a = x0;
  const fr b = tw ? fr::mul_nored(x1, fr::load(w)) : x1;
  x0 = fr::add_lazy(a, b);
  x1 = fr::sub_lazy(a, b);
}
__device__ __forceinline__ fr canon_out(const fr& x) { return x.canon(); }
#else
__device__ __forceinline__ void bfly_dif(fr& x0, fr& x1, const uint32_t* w, bool tw) {
  const fr a = x0, b = x1;
  x0 = a + b;
  fr diff = a - b;
  if (tw) diff = diff * fr::load(w);
  x1 = diff;
}
__device__ __forceinline__ void bfly_dit(fr& x0, fr& x1, const uint32_t* w, bool tw) {
  const fr a = x0;
  fr b = x1;
  if (tw) b = b * fr::load(w);
  x0 = a + b;
  x1 = a - b;
}
__device__ __forceinline__ fr canon_out(const fr& x) { return x; }
#endif


// One pass of K DIF stages starting at global stage s0 (stage s has half-distance m >> (s+1)).
// If `in` != nullptr this is the first pass: read in[idx] (zero beyond in_len), optionally
// scaled by pre[idx], and write to `data`.
template <int K>
__global__ void __launch_bounds__(256) k_ntt_dif_pass(uint32_t* __restrict__ data,
                                                      const uint32_t* __restrict__ in, uint64_t in_len,
                                                      const uint32_t* __restrict__ pre,
                                                      const uint32_t* __restrict__ tw, int logM, int logm,
                                                      int s0) {
  KGS_AUX_PRIO();
  const uint64_t m = 1ull << logm;
  const uint64_t ngroups = m >> K;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const int logd = logm - s0 - K;  // group stride d = m >> (s0+K)
  const uint64_t d = 1ull << logd;
  const uint64_t lo = g & (d - 1), hi = g >> logd;
  const uint64_t base = (hi << (logd + K)) + lo;
  fr x[1 << K];
#pragma unroll
  for (int r = 0; r < (1 << K); r++) {
    uint64_t idx = base + ((uint64_t)r << logd);
    if (in) {
      if (idx < in_len) {
        x[r] = fr::load(in + 8 * idx);
        if (pre) x[r] = x[r] * fr::load(pre + 8 * idx);
      } else {
        x[r] = fr::zero();
      }
    } else {
      x[r] = fr::load(data + 8 * idx);
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int s = s0 + k;
    const int logh = logm - s - 1;           // half-distance h = 2^logh = d * 2^(K-1-k)
    const int dist = 1 << (K - 1 - k);       // register distance
    const uint64_t twbase = 1ull << logh;    // stage table: w_{2h}^t = tw[h + t]
#pragma unroll
    for (int j = 0; j < (1 << (K - 1)); j++) {
      // j-th butterfly of this stage: register pair (r, r + dist), r has bit (K-1-k) clear
      const int r = ((j / dist) * 2 * dist) + (j % dist);
      const uint64_t t = lo + ((uint64_t)(j % dist) << logd);
      bfly_dif(x[r], x[r + dist], tw + 8 * (twbase + t), t != 0);
    }
  }
#pragma unroll
  for (int r = 0; r < (1 << K); r++) canon_out(x[r]).store(data + 8 * (base + ((uint64_t)r << logd)));
}

// One pass of K DIT stages starting at global stage s0 (half-distance 2^s). First pass may read
// from `in` (natural order when in_bitrev == false: gathered through bit reversal). The last pass
// may multiply by post[idx] and/or the scalar `post_s` (if non-null).
template <int K>
__global__ void __launch_bounds__(256) k_ntt_dit_pass(uint32_t* __restrict__ data,
                                                      const uint32_t* __restrict__ in, int in_bitrev,
                                                      const uint32_t* __restrict__ tw, int logM, int logm,
                                                      int s0, const uint32_t* __restrict__ post,
                                                      const uint32_t* __restrict__ post_s) {
  KGS_AUX_PRIO();
  const uint64_t m = 1ull << logm;
  const uint64_t ngroups = m >> K;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= ngroups) return;
  const int logd = s0;  // group stride d = 2^s0
  const uint64_t d = 1ull << logd;
  const uint64_t lo = g & (d - 1), hi = g >> logd;
  const uint64_t base = (hi << (logd + K)) + lo;
  fr x[1 << K];
#pragma unroll
  for (int r = 0; r < (1 << K); r++) {
    uint64_t idx = base + ((uint64_t)r << logd);
    if (in) {
      uint64_t src = in_bitrev ? idx : (uint64_t)bitrev((uint32_t)idx, logm);
      x[r] = fr::load(in + 8 * src);
    } else {
      x[r] = fr::load(data + 8 * idx);
    }
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int s = s0 + k;  // half-distance h = 2^s = d * 2^k
    const int dist = 1 << k;
    const uint64_t twbase = 1ull << s;       // stage table: w_{2h}^t = tw[h + t], h = 2^s
#pragma unroll
    for (int j = 0; j < (1 << (K - 1)); j++) {
      const int r = ((j / dist) * 2 * dist) + (j % dist);
      const uint64_t t = lo + ((uint64_t)(j % dist) << logd);
      bfly_dit(x[r], x[r + dist], tw + 8 * (twbase + t), t != 0);
    }
  }
  fr ps;
  if (post_s) ps = fr::load(post_s);
#pragma unroll
  for (int r = 0; r < (1 << K); r++) {
    uint64_t idx = base + ((uint64_t)r << logd);
    fr y = x[r];
    if (post) y = y * fr::load(post + 8 * idx);
    if (post_s) y = y * ps;
    canon_out(y).store(data + 8 * idx);
  }
}

static inline unsigned nblocks(uint64_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }

// ---------------------------------------------------------------- LDS-staged passes (K1 + K2 stages)
// The same butterflies with the same stage twiddles as the radix-8 passes above (so the output is
// bit-identical), but K = K1 + K2 <= 6 stages per global read/write of the data: a block stages
// LDS_ELEMS = 2^NTT_ELOG elements in LDS, runs a radix-2^K1 register round, exchanges through LDS,
// runs a radix-2^K2 round, and writes back. An m = 2^21 transform takes 4 passes instead of 7.
// Index map of a pass (group stride d = 2^logd; DIF: logd = logm - s0 - K, DIT: logd = s0):
// idx(col, j) = (hi << (logd + K)) | (j << logd) | lo, col = (hi << logd) | lo, j < 2^K. Block b owns
// columns [b*LB, (b+1)*LB), LB = LDS_ELEMS >> K; its elements are contiguous runs of min(LB, d) (logd >=
// log2 LB) or 2^(logd+K) (otherwise) elements, loaded and stored in address order (coalesced).
// LDS layout: element e = j * LB + (col - b*LB) as two 16-byte halves in two planes, lo[e] and hi[e]:
// the lanes of a wave touch consecutive 16-byte slots, so every ds_read_b128 / ds_write_b128 is
// bank-conflict free in the DIF passes (a 32-byte element stride put two lanes of each 16-lane group on
// the same banks: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.50 -> 0.04; profiles/r03/ntt_counters.txt).
// 2^21 pair 0.625 -> 0.616 ms (same-box A/B, profiles/r03/ntt_ab.txt): LDS was never the limiter —
// the pass waves sit 37-41 % of their cycles parked on global loads and barriers at 2 blocks (8 waves)
// per CU. Tile size: 2^11 elements (64 KiB, 256 threads); 2^10-element tiles with 128 threads
// (-DKGS_NTT_ELOG=10: five blocks per CU) measured 16 % slower. A persistent grid (two blocks per CU
// walking the tiles) that prefetches the next tile's elements into registers during the rounds was
// measured too and rejected: 2^21 pair 0.609 ms (this kernel) vs 0.627 (persistent, no prefetch),
// 0.636 (2 of 8 elements prefetched), 0.655 (4 of 8: register spills), profiles/r03/ntt_pf_ab.txt.
#ifndef KGS_NTT_ELOG
#define KGS_NTT_ELOG 11
#endif
constexpr int NTT_ELOG = KGS_NTT_ELOG;
constexpr int LDS_ELEMS = 1 << NTT_ELOG;
constexpr int LDS_NT = LDS_ELEMS / 8;  // threads per block: one radix-8 column group each

__device__ __forceinline__ void lds_map(uint32_t e, int K, int logd, int lblog, uint32_t& j, uint32_t& cl) {
  if (logd >= lblog) {  // for each j a run of LB consecutive lo
    j = e >> lblog;
    cl = e & ((1u << lblog) - 1);
  } else {              // contiguous hi blocks of 2^(logd + K) elements
    const uint32_t lo = e & ((1u << logd) - 1);
    j = (e >> logd) & ((1u << K) - 1);
    cl = ((e >> (logd + K)) << logd) | lo;
  }
}

// element indices < 2^28 (logm <= 28): 32-bit index arithmetic
__device__ __forceinline__ uint32_t lds_idx(uint32_t col, uint32_t j, int K, int logd) {
  const uint32_t lo = col & ((1u << logd) - 1), hi = col >> logd;
  return (hi << (logd + K)) | (j << logd) | lo;
}

#ifndef KGS_NTT_LDS_AOS
// 16-byte slot e of a plane -> swizzled slot: the low 4 bits (the slot's bank group within a 256-byte
// LDS row) XORed with bits 4-7 and 8-11, a bijection on the tile. The contiguous pass's address-order
// staging (lanes step j, slot stride LB) and its rounds hit 2-6 slots per bank group in each 16-lane
// phase of a ds_read/write_b128 without it (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE 0.54); with it every
// access pattern of every pass plan is at most 2-way (profiles/r03/ntt_lds_swizzle.txt).
__device__ __forceinline__ uint32_t lds_swz(uint32_t e) { return e ^ ((e >> 4) & 15u) ^ ((e >> 8) & 15u); }
__device__ __forceinline__ fr lds_ld(const uint32_t* lds, uint32_t e) {
  e = lds_swz(e);
  const uint4 a = reinterpret_cast<const uint4*>(lds)[e];
  const uint4 b = reinterpret_cast<const uint4*>(lds + 4 * LDS_ELEMS)[e];
  fr r;
  r.v[0] = a.x; r.v[1] = a.y; r.v[2] = a.z; r.v[3] = a.w;
  r.v[4] = b.x; r.v[5] = b.y; r.v[6] = b.z; r.v[7] = b.w;
  return r;
}
__device__ __forceinline__ void lds_st(uint32_t* lds, uint32_t e, const fr& x) {
  e = lds_swz(e);
  reinterpret_cast<uint4*>(lds)[e] = make_uint4(x.v[0], x.v[1], x.v[2], x.v[3]);
  reinterpret_cast<uint4*>(lds + 4 * LDS_ELEMS)[e] = make_uint4(x.v[4], x.v[5], x.v[6], x.v[7]);
}
#else  // A/B: element-contiguous 32-byte slots (2-way bank conflicts on b128)
__device__ __forceinline__ fr lds_ld(const uint32_t* lds, uint32_t e) { return fr::load(lds + 8 * e); }
__device__ __forceinline__ void lds_st(uint32_t* lds, uint32_t e, const fr& x) { x.store(lds + 8 * e); }
#endif

// Where a round's elements come from / go to: the LDS tile, or global memory directly (the pass's
// first round reads its elements from HBM into registers and its last round writes them back from
// registers, with no LDS staging round trip and no barrier around them). Direct access is coalesced
// when a tile's columns are runs of LB >= 4 consecutive elements (group stride d >= LB): consecutive
// lanes then hold consecutive elements. The pass whose columns are contiguous blocks (d < LB: the
// DIF-last / DIT-first pass) stages through LDS in address order instead.
struct ntt_io {
  uint32_t* data;
  const uint32_t* in;   // first pass: source (DIF: zero beyond in_len, times pre[idx]; DIT: bit reversal)
  uint64_t in_len;
  int in_bitrev;
  const uint32_t* pre;
  const uint32_t* post;  // last pass: times post[idx] and / or the scalar *post_s
  const uint32_t* post_s;
  int logm;
  // the T29 passes: pre / post / post_s as 29-bit records (the domain's twin table, fr29.hpp)
  const uint32_t* pre29;
  const uint32_t* post29;
  const uint32_t* post_s29;
};

// values in [0, 2p) (the butterflies' range): the scalings need no reduction below p
template <bool DIT, bool T29>
__device__ __forceinline__ fr ntt_load(const ntt_io& io, uint64_t idx) {
  if (!io.in) return fr::load(io.data + 8 * idx);
  if (DIT) return fr::load(io.in + 8 * (io.in_bitrev ? idx : (uint64_t)bitrev((uint32_t)idx, io.logm)));
  if (idx >= io.in_len) return fr::zero();
  fr x = fr::load(io.in + 8 * idx);
  if (io.pre) x = T29 ? mul29(x, w29_load(io.pre29 + TW29_WORDS * idx)) : x * fr::load(io.pre + 8 * idx);
  return x;
}
template <bool T29>
__device__ __forceinline__ void ntt_store(const ntt_io& io, uint64_t idx, fr y) {
  if (io.post) y = T29 ? mul29(y, w29_load(io.post29 + TW29_WORDS * idx)) : y * fr::load(io.post + 8 * idx);
  if (io.post_s) y = T29 ? mul29(y, w29_load(io.post_s29)) : y * fr::load(io.post_s);
  canon_out(y).store(io.data + 8 * idx);
}

// Twiddles of the LDS passes: `fr` (8 x 32-bit words, fr::mul_nored_x2) or, since round 5, `W29`
// (the 29-bit records of the domain's twin tables, fr29.hpp mul29: 9 independent column chains per
// product instead of one; the two products of a pair are independent, so the compiler interleaves
// them itself). Both give a product in [0, 2p) of the same residue: the canonical pass outputs are
// bit-identical.
template <typename TW>
__device__ __forceinline__ TW tw_load(const uint32_t* tw, uint32_t idx);
template <>
__device__ __forceinline__ fr tw_load<fr>(const uint32_t* tw, uint32_t idx) { return fr::load(tw + 8 * idx); }
template <>
__device__ __forceinline__ W29 tw_load<W29>(const uint32_t* tw, uint32_t idx) {
  return w29_load(tw + TW29_WORDS * idx);
}
__device__ __forceinline__ void mul_tw_x2(const fr& a, const fr& wa, const fr& b, const fr& wb, fr& ra, fr& rb) {
  fr::mul_nored_x2(a, wa, b, wb, ra, rb);
}
__device__ __forceinline__ void mul_tw_x2(const fr& a, const W29& wa, const fr& b, const W29& wb, fr& ra, fr& rb) {
  ra = mul29(a, wa);
  rb = mul29(b, wb);
}

// for (I = 0; I < N; I++) f(integral_constant<I>) with every iteration expanded at compile time
template <typename F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// butterfly groups of lds_round: (r, r + dist) for the given register indices
__device__ __forceinline__ void bfly_pair_triv(fr* x, int r0, int r1, int dist) {  // w = 1 for both
  const fr a0 = x[r0], b0 = x[r0 + dist], a1 = x[r1], b1 = x[r1 + dist];
  x[r0] = fr::add_lazy(a0, b0);
  x[r0 + dist] = fr::sub_lazy(a0, b0);
  x[r1] = fr::add_lazy(a1, b1);
  x[r1 + dist] = fr::sub_lazy(a1, b1);
}
template <bool DIT, typename TW>
__device__ __forceinline__ void bfly_pair_x2(fr* x, int r0, int r1, int dist, const TW& w0, const TW& w1) {
  if (DIT) {
    fr b0, b1;
    mul_tw_x2(x[r0 + dist], w0, x[r1 + dist], w1, b0, b1);
    const fr a0 = x[r0], a1 = x[r1];
    x[r0] = fr::add_lazy(a0, b0);
    x[r0 + dist] = fr::sub_lazy(a0, b0);
    x[r1] = fr::add_lazy(a1, b1);
    x[r1 + dist] = fr::sub_lazy(a1, b1);
  } else {
    const fr d0 = fr::sub_2p(x[r0], x[r0 + dist]), d1 = fr::sub_2p(x[r1], x[r1 + dist]);
    x[r0] = fr::add_lazy(x[r0], x[r0 + dist]);
    x[r1] = fr::add_lazy(x[r1], x[r1 + dist]);
    mul_tw_x2(d0, w0, d1, w1, x[r0 + dist], x[r1 + dist]);
  }
}
// one register round of R stages of a pass on the 2^R elements j = jb + js * r (r < 2^R) of column
// col: stage k of the round is pass stage kp0 + k; DIF pairs (r, r + 2^(R-1-k)), DIT (r, r + 2^k)
template <int R, bool DIT, bool GIN, bool GOUT, bool PF, typename TW>
__device__ __forceinline__ void lds_round(uint32_t* lds, const uint32_t* __restrict__ tw, const ntt_io& io, uint32_t cl,
                                          uint32_t col, uint32_t jb, uint32_t js, int K, int logd, int lb, int kp0) {
  constexpr bool T29 = std::is_same<TW, W29>::value;
  fr x[1 << R];
  if (GIN && !DIT && io.in && io.pre && R >= 2) {
    // first DIF pass with a coset pre-scaling: the products two at a time. A pair past the input
    // (the zero upper half of a degree < n polynomial on a 2n coset: the top j-bit, i.e. r >= 2^(R-1)
    // for every lane) stays zero without its products. Compile-time register indices (static_for,
    // see the step loop below): with the 29-bit products the unrolled loop went to scratch
    static_for<(1 << R) / 2>([&](auto rc) {
      constexpr int r = 2 * decltype(rc)::value;
      const uint32_t i0 = lds_idx(col, jb + js * r, K, logd), i1 = lds_idx(col, jb + js * (r + 1), K, logd);
      if (__builtin_expect(__all(i0 >= io.in_len && i1 >= io.in_len), 0)) {
        x[r] = fr::zero();
        x[r + 1] = fr::zero();
        return;
      }
      const fr a0 = i0 < io.in_len ? fr::load(io.in + 8 * i0) : fr::zero();
      const fr a1 = i1 < io.in_len ? fr::load(io.in + 8 * i1) : fr::zero();
      if constexpr (T29) {
        x[r] = mul29(a0, w29_load(io.pre29 + TW29_WORDS * i0));
        x[r + 1] = mul29(a1, w29_load(io.pre29 + TW29_WORDS * i1));
      } else {
        fr::mul_nored_x2(a0, fr::load(io.pre + 8 * i0), a1, fr::load(io.pre + 8 * i1), x[r], x[r + 1]);
      }
    });
  } else {
    static_for<(1 << R)>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      x[r] = GIN ? ntt_load<DIT, T29>(io, lds_idx(col, jb + js * r, K, logd)) : lds_ld(lds, (jb + js * r) * lb + cl);
    });
  }
#ifdef KGS_NTT_SINGLE
  // A/B build: one butterfly at a time. That path reads 8 x 32-bit twiddles only, so the 29-bit
  // instantiations keep the pairs (select KGS_NTT_T29=0 to measure the single path everywhere)
  constexpr bool kPairs = T29;
#else
  constexpr bool kPairs = true;
#endif
  if constexpr (R >= 2 && kPairs) {
    // Butterflies two at a time (q, q + half), their products interleaved (fr::mul_nored_x2; four at a
    // time, fr::mul_nored_x4 at 232 VGPRs, measured 1.25x slower: profiles/r03/ntt_x2_x4.txt). A pair
    // whose twiddles are all w^0 = 1 across the wave (low stages of the contiguous pass, where t depends
    // on the register index only) skips its products; otherwise a lane with t == 0 multiplies by
    // tw[h] = 1 (a product in [0, 2p) congruent to its input: same canonical output). The twiddles of
    // the next (stage, pair) step are loaded before the current step's butterflies: each step is its
    // own basic block (the uniform w^0 branch), so the compiler issued every twiddle load right before
    // its product and waited on it there.
    constexpr int half = 1 << (R - 2);
    constexpr int NSTEP = R * half;
    uint32_t tw0[NSTEP], tw1[NSTEP];  // twiddle indices (stage table offset + t) of each step
    bool triv[NSTEP];
#pragma unroll
    for (int k = 0; k < R; k++) {
      const int kp = kp0 + k;
      const int logh = DIT ? logd + kp : logd + K - 1 - kp;
      const int dist = DIT ? 1 << k : 1 << (R - 1 - k);
      const uint32_t hm = (1u << logh) - 1;
#pragma unroll
      for (int qa = 0; qa < half; qa++) {
        const int r0 = ((qa / dist) * 2 * dist) + (qa % dist), r1 = (((qa + half) / dist) * 2 * dist) + ((qa + half) % dist);
        const uint32_t t0 = lds_idx(col, jb + js * r0, K, logd) & hm, t1 = lds_idx(col, jb + js * r1, K, logd) & hm;
        tw0[k * half + qa] = hm + 1 + t0;
        tw1[k * half + qa] = hm + 1 + t1;
        triv[k * half + qa] = __all(t0 == 0 && t1 == 0);
      }
    }
    // PF: the next step's twiddles loaded before this step's butterflies (the 2-wave build); the
    // 3-wave build (<= 168 VGPRs) loads each step's own twiddles, which saves their registers
    TW wa, wb;
    if (PF) {
      wa = tw_load<TW>(tw, tw0[0]);
      wb = tw_load<TW>(tw, tw1[0]);
    }
    // a compile-time loop: with the larger 29-bit products LLVM stopped unrolling the step loop and
    // indexed x[] dynamically, i.e. through scratch memory; here every step's register indices are
    // constants whatever the body's size
    static_for<NSTEP>([&](auto stc) {
      constexpr int st = decltype(stc)::value;
      constexpr int k = st / half, qa = st % half;
      constexpr int dist = DIT ? 1 << k : 1 << (R - 1 - k);
      constexpr int r0 = ((qa / dist) * 2 * dist) + (qa % dist), r1 = (((qa + half) / dist) * 2 * dist) + ((qa + half) % dist);
      if (PF) {
        constexpr int nx = st + 1 < NSTEP ? st + 1 : st;  // the last step reloads its own twiddles (unused)
        const TW na = tw_load<TW>(tw, tw0[nx]), nb = tw_load<TW>(tw, tw1[nx]);
        if (triv[st])
          bfly_pair_triv(x, r0, r1, dist);
        else
          bfly_pair_x2<DIT>(x, r0, r1, dist, wa, wb);
        wa = na;
        wb = nb;
      } else if (triv[st]) {
        bfly_pair_triv(x, r0, r1, dist);
      } else {
        bfly_pair_x2<DIT>(x, r0, r1, dist, tw_load<TW>(tw, tw0[st]), tw_load<TW>(tw, tw1[st]));
      }
    });
  } else {
    static_assert(sizeof(TW) == sizeof(fr), "the single-butterfly path reads 8 x 32-bit twiddles only");
#pragma unroll
    for (int k = 0; k < R; k++) {
      const int kp = kp0 + k;                                 // stage within the pass
      const int logh = DIT ? logd + kp : logd + K - 1 - kp;   // half-distance h = 2^logh
      const int dist = DIT ? 1 << k : 1 << (R - 1 - k);       // register distance
#pragma unroll
      for (int q = 0; q < (1 << (R - 1)); q++) {
        const int r = ((q / dist) * 2 * dist) + (q % dist);
        const uint32_t idx = lds_idx(col, jb + js * r, K, logd);
        const uint32_t t = idx & ((1u << logh) - 1);
        const uint32_t* w = tw + 8 * ((1u << logh) + t);  // stage table: w_{2h}^t = tw[h + t]
        if (DIT)
          bfly_dit(x[r], x[r + dist], w, t != 0);
        else
          bfly_dif(x[r], x[r + dist], w, t != 0);
      }
    }
  }
  if (GOUT && R >= 2) {
    // last pass: the post-scalings two products at a time, then canonical stores
    if (io.post) {
      static_for<(1 << R) / 2>([&](auto rc) {
        constexpr int r = 2 * decltype(rc)::value;
        const uint32_t i0 = lds_idx(col, jb + js * r, K, logd), i1 = lds_idx(col, jb + js * (r + 1), K, logd);
        if constexpr (T29) {
          x[r] = mul29(x[r], w29_load(io.post29 + TW29_WORDS * i0));
          x[r + 1] = mul29(x[r + 1], w29_load(io.post29 + TW29_WORDS * i1));
        } else {
          fr::mul_nored_x2_ip(x[r], fr::load(io.post + 8 * i0), x[r + 1], fr::load(io.post + 8 * i1));
        }
      });
    }
    if (io.post_s) {
      if constexpr (T29) {
        const W29 ps = w29_load(io.post_s29);
        static_for<(1 << R)>([&](auto rc) {
          constexpr int r = decltype(rc)::value;
          x[r] = mul29(x[r], ps);
        });
      } else {
        const fr ps = fr::load(io.post_s);
#pragma unroll
        for (int r = 0; r < (1 << R); r += 2) fr::mul_nored_x2_ip(x[r], ps, x[r + 1], ps);
      }
    }
#pragma unroll
    for (int r = 0; r < (1 << R); r++) canon_out(x[r]).store(io.data + 8 * lds_idx(col, jb + js * r, K, logd));
    return;
  }
#pragma unroll
  for (int r = 0; r < (1 << R); r++) {
    if (GOUT)
      ntt_store<T29>(io, lds_idx(col, jb + js * r, K, logd), x[r]);
    else
      lds_st(lds, (jb + js * r) * lb + cl, x[r]);
  }
}

// all groups of one round of a pass: the round covers the j-bits [b0, b0 + R) of every column of the
// tile (a thread holds the 2^R elements that differ in those bits, the other K - R bits fixed).
// DIF rounds run from the top j-bits down, DIT rounds from bit 0 up; kp0 = the round's first stage
// within the pass.
template <int R, bool DIT, bool GIN, bool GOUT, bool PF, typename TW>
__device__ __forceinline__ void lds_round_all(uint32_t* lds, const uint32_t* __restrict__ tw, const ntt_io& io,
                                              uint32_t col0, int K, int logd, int lblog, int b0) {
  const int kp0 = DIT ? b0 : K - b0 - R;
  for (uint32_t g = threadIdx.x; g < (LDS_ELEMS >> R); g += LDS_NT) {
    const uint32_t cl = g & ((1u << lblog) - 1), jq = g >> lblog;
    const uint32_t jb = (jq & ((1u << b0) - 1)) | ((jq >> b0) << (b0 + R));
    lds_round<R, DIT, GIN, GOUT, PF, TW>(lds, tw, io, cl, col0 + cl, jb, 1u << b0, K, logd, 1 << lblog, kp0);
  }
}

// K1 + K2 + K3 stages from s0 (two or three register rounds with an LDS exchange between rounds).
// DIRECT: the first round loads from and the last round stores to global memory (d >= LB); else the
// tile is loaded into / stored from LDS in address order around the rounds.
// WV = the waves per SIMD the pass is compiled for. WV = 2 (211 VGPRs for the 9-stage DIF pass): the
// fastest pass alone, but a pass wave cannot start on a SIMD that holds two accumulate waves (2 x 168
// + 211 > 512), so in flight the other proofs' NTT blocks wait for a CU's accumulate blocks to drain.
// WV = 3 (<= 168 VGPRs: 2 x 168 + 168 <= 512; the DIF passes spill 100-164 B): 9 % slower alone
// (2^21 pair 0.56 vs 0.515 ms) and +0.6 % proofs/s with four proofs in flight, higher than the
// WV = 2 build in all 5 same-box reps on two boxes (profiles/r04/coresidency/, profiles/r04/ntt/).
// Contexts proving one proof at a time (two MSM lanes, the latency mode) and every other caller
// launch WV = 2; in-flight contexts (one lane) WV = 3 (ntt_set_coresident).
// A/B knob: KGS_NTT_PF3=1 keeps the twiddle prefetch in the 3-wave build too
#ifndef KGS_NTT_PF3
#define KGS_NTT_PF3 0
#endif
// T29: the twiddle products in 9 x 29-bit limbs (tw = the domain's 29-bit twin table, fr29.hpp)
// K4 > 0 (2^12-element tiles only, -DKGS_NTT_ELOG=12): a fourth register round, up to 12 stages per pass
template <int K1, int K2, int K3, int K4, bool DIT, bool DIRECT, int WV, bool T29>
__global__ void __launch_bounds__(LDS_NT) __attribute__((amdgpu_waves_per_eu(WV, WV)))
k_ntt_lds_pass(ntt_io io, const uint32_t* __restrict__ tw, int s0) {
  using TW = typename std::conditional<T29, W29, fr>::type;
  KGS_AUX_PRIO();
  constexpr int K = K1 + K2 + K3 + K4;
  static_assert(K4 == 0 || K3 > 0, "rounds are filled in order");
  constexpr int LBLOG = NTT_ELOG - K;
  constexpr int LB = 1 << LBLOG;
  uint32_t* lds;
  if constexpr (WV >= 3) {
    // dynamic LDS: with a static 64 KiB tile the compiler takes the LDS-bound occupancy (2 blocks per
    // CU) as its target and ignores waves_per_eu
    extern __shared__ __attribute__((aligned(16))) uint32_t lds_dyn[];
    lds = lds_dyn;
  } else {
    __shared__ __attribute__((aligned(16))) uint32_t lds_tile[LDS_ELEMS * 8];
    lds = lds_tile;
  }
  const int logd = DIT ? s0 : io.logm - s0 - K;
  const uint32_t col0 = blockIdx.x * LB;
  if (!DIRECT) {  // load (address order)
    for (uint32_t e = threadIdx.x; e < LDS_ELEMS; e += LDS_NT) {
      uint32_t j, cl;
      lds_map(e, K, logd, LBLOG, j, cl);
      lds_st(lds, j * LB + cl, ntt_load<DIT, T29>(io, lds_idx(col0 + cl, j, K, logd)));
    }
    __syncthreads();
  }
  // DIF: bits [K-K1, K), [K-K1-K2, K-K1), ... down to 0; DIT: [0, K1), [K1, K1+K2), ... up to K
  constexpr bool PF = WV < 3 || KGS_NTT_PF3;
  lds_round_all<K1, DIT, DIRECT, false, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? 0 : K - K1);
  __syncthreads();
  if constexpr (K4 > 0) {
    lds_round_all<K2, DIT, false, false, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 : K3 + K4);
    __syncthreads();
    lds_round_all<K3, DIT, false, false, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 + K2 : K4);
    __syncthreads();
    lds_round_all<K4, DIT, false, DIRECT, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 + K2 + K3 : 0);
  } else if constexpr (K3 > 0) {
    lds_round_all<K2, DIT, false, false, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 : K3);
    __syncthreads();
    lds_round_all<K3, DIT, false, DIRECT, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 + K2 : 0);
  } else {
    lds_round_all<K2, DIT, false, DIRECT, PF, TW>(lds, tw, io, col0, K, logd, LBLOG, DIT ? K1 : 0);
  }
  if (!DIRECT) {  // store (address order)
    __syncthreads();
    for (uint32_t e = threadIdx.x; e < LDS_ELEMS; e += LDS_NT) {
      uint32_t j, cl;
      lds_map(e, K, logd, LBLOG, j, cl);
      ntt_store<T29>(io, lds_idx(col0 + cl, j, K, logd), lds_ld(lds, j * LB + cl));
    }
  }
}

// the calling thread's pass build (ntt_set_coresident; per thread: contexts prove on their callers' threads)
thread_local bool g_ntt_coresident = false;

// 8 x 32 element tables -> their registered 29-bit twins, record i of the twin = element i of the
// table (the shared domain tables register theirs when built, unregister when freed): a pointer
// anywhere inside a registered table (a stage table, the coset powers, one 1/m scalar) maps to its
// record. KGS_NTT_T29=0 keeps the 8 x 32 products (A/B).
struct Tw29Entry {
  uint64_t count;
  const uint32_t* twin;
};
static std::mutex g_tw29_mu;
static std::map<const uint32_t*, Tw29Entry> g_tw29;
void ntt_register_tw29(const uint32_t* base, uint64_t count, const uint32_t* twin) {
  std::lock_guard<std::mutex> lk(g_tw29_mu);
  g_tw29[base] = Tw29Entry{count, twin};
}
void ntt_unregister_tw29(const uint32_t* base) {
  std::lock_guard<std::mutex> lk(g_tw29_mu);
  g_tw29.erase(base);
}
static bool t29_off() {
  static const bool off = [] {
    const char* e = getenv("KGS_NTT_T29");
    return e && e[0] == '0';
  }();
  return off;
}
static const uint32_t* tw29_of(const uint32_t* p) {
  if (!p || t29_off()) return nullptr;
  std::lock_guard<std::mutex> lk(g_tw29_mu);
  auto it = g_tw29.upper_bound(p);
  if (it == g_tw29.begin()) return nullptr;
  --it;
  const uint64_t off = (uint64_t)(p - it->first);
  if (off % 8 || off / 8 >= it->second.count) return nullptr;
  return it->second.twin + (uint64_t)TW29_WORDS * (off / 8);
}

// the 29-bit record of a stage twiddle (fr29.hpp): w * 2^261 mod p (= its Montgomery form times the
// Montgomery form of 32), canonical, in 9 limbs + a zero pad word
__global__ void k_tw29(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, uint64_t count) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  fr c;
#pragma unroll
  for (int k = 0; k < 8; k++) c.v[k] = r29::C32[k];
  const fr x = fr::load(in + 8 * i) * c;
  uint32_t l[9];
  unpack29(x, l);
  uint32_t* o = out + (uint64_t)TW29_WORDS * i;
#pragma unroll
  for (int k = 0; k < 9; k++) o[k] = l[k];
  o[9] = 0;
}
void launch_tw29(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t count) {
  hipLaunchKernelGGL(k_tw29, dim3(nblocks(count)), dim3(256), 0, st, out, in, count);
}

#ifndef KGS_NO_NTT_LDS
// LDS passes need m >= the tile (2^NTT_ELOG elements)
constexpr int LDS_MIN_LOGM = NTT_ELOG > 11 ? NTT_ELOG : 11;
constexpr int LDS_MAX_K = NTT_ELOG - 2 < 9 ? NTT_ELOG - 2 : 9;  // >= 4 columns (128 B runs) per tile

// Pass plan of an m = 2^logm transform (logm >= LDS_MIN_LOGM), in DIF order: ceil(logm / 9) LDS passes
// of 4..9 stages; the pass whose columns are contiguous (DIF last / DIT first: group stride 1) takes up
// to 9 stages (three register rounds), the others 6 (two rounds, 1 KiB runs) unless more are needed.
// 2^20 = 6+6+8, 2^21 = 6+6+9, 2^22 = 7+6+9, 2^24 = 8+7+9: three passes where the radix-8 tail pass
// made four.
//
// 2^12-element tiles (-DKGS_NTT_ELOG=12: 128 KiB of LDS, 512 threads, one block per CU): the
// contiguous pass takes up to 12 stages (four register rounds), the others up to 10 (>= 4 columns per
// tile): 2^20 = 8+12, 2^21 = 9+12, 2^22 = 10+12, 2^24 = 6+6+12, i.e. one global round trip fewer.
static int lds_plan(int logm, int* ks) {
  if (NTT_ELOG >= 12) {
    int E = logm < NTT_ELOG ? logm : NTT_ELOG;
    int rest = logm - E;
    if (rest > 0 && rest < 4) {  // passes of >= 4 stages (two register rounds of >= 2)
      E = logm - 4;
      rest = 4;
    }
    const int maxk = NTT_ELOG - 2;
    const int P = 1 + (rest + maxk - 1) / maxk;
    for (int i = 0; i < P - 1; i++) {
      const int left = P - 1 - i;
      ks[i] = (rest + left - 1) / left;
      rest -= ks[i];
    }
    ks[P - 1] = E;
    return P;
  }
  const int P = (logm + LDS_MAX_K - 1) / LDS_MAX_K;
  int E = logm - 6 * (P - 1);
  if (E > LDS_MAX_K) E = LDS_MAX_K;
  int rest = logm - E;
  for (int i = 0; i < P - 1; i++) {
    const int left = P - 1 - i;
    ks[i] = (rest + left - 1) / left;
    rest -= ks[i];
  }
  ks[P - 1] = E;
  return P;
}

static void launch_lds_pass(hipStream_t st, int K, bool dit, uint32_t* data, const uint32_t* in, uint64_t in_len,
                            int in_bitrev, const uint32_t* pre, const uint32_t* tw, int logm, int s0,
                            const uint32_t* post, const uint32_t* post_s) {
  const unsigned blocks = (unsigned)((1ull << logm) / LDS_ELEMS);
  // the 29-bit twins of the twiddles and scalings, if the domain registered them: all or none
  const uint32_t* pre29 = tw29_of(pre);
  const uint32_t* post29 = tw29_of(post);
  const uint32_t* post_s29 = tw29_of(post_s);
  const uint32_t* tw29 = tw29_of(tw);
  if ((pre && !pre29) || (post && !post29) || (post_s && !post_s29)) tw29 = nullptr;
  const ntt_io io{data, in, in_len, in_bitrev, pre, post, post_s, logm, pre29, post29, post_s29};
  const int logd = dit ? s0 : logm - s0 - K;
  static const bool staged = getenv("KGS_NTT_STAGED") != nullptr;  // A/B: every pass staged through LDS
  // A/B: a whole-tile pass (K = NTT_ELOG, one column of consecutive elements) loads and stores its
  // rounds directly as well (lanes then step 1 or 2^R elements)
  static const bool direct_tile = getenv("KGS_NTT_DIRECT_TILE") != nullptr;
  const bool direct = logd >= NTT_ELOG - K && (NTT_ELOG - K >= 2 || direct_tile) && !staged;
#define KGS_LDS_LAUNCH2(A, B, C, F, D, E, T, TWP)                                                              \
  do {                                                                                                         \
    if (g_ntt_coresident)                                                                                      \
      hipLaunchKernelGGL((k_ntt_lds_pass<A, B, C, F, D, E, 3, T>), dim3(blocks), dim3(LDS_NT), LDS_ELEMS * 32,  \
                         st, io, TWP, s0);                                                                     \
    else                                                                                                       \
      hipLaunchKernelGGL((k_ntt_lds_pass<A, B, C, F, D, E, 2, T>), dim3(blocks), dim3(LDS_NT), 0, st, io, TWP, \
                         s0);                                                                                  \
  } while (0)
#define KGS_LDS_LAUNCH(A, B, C, F, D, E)             \
  do {                                               \
    if (tw29)                                        \
      KGS_LDS_LAUNCH2(A, B, C, F, D, E, true, tw29); \
    else                                             \
      KGS_LDS_LAUNCH2(A, B, C, F, D, E, false, tw);  \
  } while (0)
#if KGS_NTT_ELOG >= 12
#define KGS_LDS_BY_K_WIDE(D, E)                          \
  case 12: KGS_LDS_LAUNCH(3, 3, 3, 3, D, E); break;      \
  case 11: KGS_LDS_LAUNCH(3, 3, 3, 2, D, E); break;      \
  case 10: KGS_LDS_LAUNCH(3, 3, 2, 2, D, E); break;
#else
#define KGS_LDS_BY_K_WIDE(D, E)
#endif
#define KGS_LDS_BY_K(D, E)                             \
  switch (K) {                                         \
    KGS_LDS_BY_K_WIDE(D, E)                            \
    case 9: KGS_LDS_LAUNCH(3, 3, 3, 0, D, E); break;   \
    case 8: KGS_LDS_LAUNCH(3, 3, 2, 0, D, E); break;   \
    case 7: KGS_LDS_LAUNCH(3, 2, 2, 0, D, E); break;   \
    case 6: KGS_LDS_LAUNCH(3, 3, 0, 0, D, E); break;   \
    case 5: KGS_LDS_LAUNCH(3, 2, 0, 0, D, E); break;   \
    default: KGS_LDS_LAUNCH(2, 2, 0, 0, D, E); break;  \
  }
  if (dit) {
    if (direct) {
      KGS_LDS_BY_K(true, true)
    } else {
      KGS_LDS_BY_K(true, false)
    }
  } else {
    if (direct) {
      KGS_LDS_BY_K(false, true)
    } else {
      KGS_LDS_BY_K(false, false)
    }
  }
#undef KGS_LDS_BY_K
#undef KGS_LDS_BY_K_WIDE
#undef KGS_LDS_LAUNCH
#undef KGS_LDS_LAUNCH2
}
#endif

bool ntt_set_coresident(bool on) {
  const bool prev = g_ntt_coresident;
  g_ntt_coresident = on;
  return prev;
}

void ntt_dif(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t in_len, int logm,
             const uint32_t* pre, const uint32_t* tw, int logM) {
  if (logm == 0) {
    if (in_len == 0) {
      hipMemsetAsync(out, 0, 32, st);
    } else if (in != out || pre) {
      launch_scale_copy(st, out, in, 1, pre, nullptr);
    }
    return;
  }
#ifndef KGS_NO_NTT_LDS
  if (logm >= LDS_MIN_LOGM) {
    int ks[8];
    const int P = lds_plan(logm, ks);
    for (int i = 0, s0 = 0; i < P; s0 += ks[i++])
      launch_lds_pass(st, ks[i], false, out, i ? nullptr : in, in_len, 1, i ? nullptr : pre, tw, logm, s0, nullptr,
                      nullptr);
    return;
  }
#endif
  int s0 = 0;
  bool first = true;
  while (s0 < logm) {
    const uint32_t* src = first ? in : nullptr;
    const uint32_t* p = first ? pre : nullptr;
    int K = logm - s0 >= 3 ? 3 : logm - s0;
    uint64_t groups = (1ull << logm) >> K;
    if (K == 3)
      hipLaunchKernelGGL(k_ntt_dif_pass<3>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_len, p, tw, logM, logm, s0);
    else if (K == 2)
      hipLaunchKernelGGL(k_ntt_dif_pass<2>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_len, p, tw, logM, logm, s0);
    else
      hipLaunchKernelGGL(k_ntt_dif_pass<1>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_len, p, tw, logM, logm, s0);
    s0 += K;
    first = false;
  }
}

void ntt_dit(hipStream_t st, uint32_t* out, const uint32_t* in, int in_bitrev, int logm,
             const uint32_t* tw, int logM, const uint32_t* post, const uint32_t* post_s) {
  if (logm == 0) {
    launch_scale_copy(st, out, in, 1, post, post_s);
    return;
  }
#ifndef KGS_NO_NTT_LDS
  // m >= 2^11: the LDS passes of lds_plan in reverse (the contiguous, up-to-9-stage pass first)
  if (logm >= LDS_MIN_LOGM) {
    int ks[8];
    const int P = lds_plan(logm, ks);
    for (int i = 0, s0 = 0; i < P; i++) {
      const int K = ks[P - 1 - i];
      const bool last = i == P - 1;
      launch_lds_pass(st, K, true, out, i ? nullptr : in, 0, in_bitrev, nullptr, tw, logm, s0, last ? post : nullptr,
                      last ? post_s : nullptr);
      s0 += K;
    }
    return;
  }
#endif
  // radix-8/4/2 passes; the first pass handles the remainder so the last pass is a full radix-8 one
  int rem = logm % 3;
  int s0 = 0;
  bool first = true;
  while (s0 < logm) {
    const uint32_t* src = first ? in : nullptr;
    int K = first && rem ? rem : 3;
    if (K > logm - s0) K = logm - s0;
    uint64_t groups = (1ull << logm) >> K;
    bool last = s0 + K == logm;
    const uint32_t* p = last ? post : nullptr;
    const uint32_t* ps = last ? post_s : nullptr;
    if (K == 3)
      hipLaunchKernelGGL(k_ntt_dit_pass<3>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_bitrev, tw, logM, logm, s0, p, ps);
    else if (K == 2)
      hipLaunchKernelGGL(k_ntt_dit_pass<2>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_bitrev, tw, logM, logm, s0, p, ps);
    else
      hipLaunchKernelGGL(k_ntt_dit_pass<1>, dim3(nblocks(groups)), dim3(256), 0, st, out, src, in_bitrev, tw, logM, logm, s0, p, ps);
    s0 += K;
    first = false;
  }
}

// tw[j] = w^j for j < count, computed in chunks of 64 from w^(64 t) by square-and-multiply.
__global__ void k_powers(uint32_t* __restrict__ out, uint64_t count, const uint32_t* __restrict__ wp,
                         const uint32_t* __restrict__ scale) {
  KGS_AUX_PRIO();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t start = t * 64;
  if (start >= count) return;
  fr w = fr::load(wp);
  fr acc = fr::one();
  fr b = w;
  uint64_t e = start;
  while (e) {
    if (e & 1) acc = acc * b;
    b = b.sqr();
    e >>= 1;
  }
  if (scale) acc = acc * fr::load(scale);
  for (uint64_t j = start; j < start + 64 && j < count; j++) {
    acc.store(out + 8 * j);
    acc = acc * w;
  }
}

void launch_powers(hipStream_t st, uint32_t* out, uint64_t count, const uint32_t* w_dev,
                   const uint32_t* scale_dev) {
  uint64_t threads = (count + 63) / 64;
  hipLaunchKernelGGL(k_powers, dim3(nblocks(threads)), dim3(256), 0, st, out, count, w_dev, scale_dev);
}

__global__ void k_scale_copy(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, uint64_t n,
                             const uint32_t* __restrict__ tab, const uint32_t* __restrict__ sc) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr x = fr::load(in + 8 * i);
  if (tab) x = x * fr::load(tab + 8 * i);
  if (sc) x = x * fr::load(sc);
  x.store(out + 8 * i);
}

void launch_scale_copy(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n, const uint32_t* tab,
                       const uint32_t* sc) {
  hipLaunchKernelGGL(k_scale_copy, dim3(nblocks(n)), dim3(256), 0, st, out, in, n, tab, sc);
}

__global__ void k_bitrev_copy(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, int logm) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1ull << logm)) return;
  uint64_t j = logm ? bitrev((uint32_t)i, logm) : 0;
  fr::load(in + 8 * j).store(out + 8 * i);
}

void launch_bitrev_copy(hipStream_t st, uint32_t* out, const uint32_t* in, int logm) {
  hipLaunchKernelGGL(k_bitrev_copy, dim3(nblocks(1ull << logm)), dim3(256), 0, st, out, in, logm);
}

}  // namespace kgs
