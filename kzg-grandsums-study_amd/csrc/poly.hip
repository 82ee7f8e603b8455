// Per-element / scan / reduction kernels of the prover hot path (gfx950):
//   * Montgomery conversion ([ffjs] Fr.batchToMontgomery, prover.js:147-148)            — A1
//   * linear combinations (Polynomial.add/sub/mulScalar/addScalar, polynomial.js:276-422) — A9
//   * grand-sum / grand-product builder: num/den, tile Montgomery batch inverse, prefix
//     sum / product with tile carries (grandsum.js:6-62, grandproduct.js:6-57)          — A6-A8
//   * quotient on a coset + divisibility check on H (replaces the 2n/4n `multiply` chain +
//     `divZh`, prover.js:233-286, polynomial.js:352-376,853-888)                         — A4,A10
//   * tiled Horner evaluation (polynomial.js:228-238)                                    — A11
//   * synthetic division by (X - z) as a linear-recurrence scan (polynomial.js:814-851)  — A12
// Every kernel is integer arithmetic on 32 B Montgomery elements; most are VALU bound (one or
// more 254-bit Montgomery products per element), the rest HBM bound.
#include "kernels.hpp"
#include "poly_math.hpp"
#include "fr29.hpp"

namespace kgs {

static inline unsigned nb(uint64_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }

// Threads of the single-block tile scans (k_tile_inverse, k_tile_carry, k_div_carries). A/B knob: a
// 1024-thread block needs four free wave slots of its VGPR size on every SIMD of one CU at once,
// which two resident accumulate waves per SIMD (other proofs in flight) do not leave.
#ifndef KGS_SCAN_NT
#define KGS_SCAN_NT 1024
#endif
constexpr uint32_t SCAN_NT = KGS_SCAN_NT;

__device__ __forceinline__ uint32_t brev(uint32_t x, int bits) {
  return bits ? __builtin_bitreverse32(x) >> (32 - bits) : 0;
}

// ---------------------------------------------------------------------------- conversions
__global__ void k_to_mont(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, uint64_t n) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // x * R as a 29-bit product by the constant record of R^2 (any x < 2^256; canonical output)
  W29 r2;
#pragma unroll
  for (int j = 0; j < 9; j++) r2.l[j] = r29::TO_MONT[j];
  fr::reduce_once(mul29(fr::load(in + 8 * i), r2)).store(out + 8 * i);
}
void launch_to_mont(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n) {
  hipLaunchKernelGGL(k_to_mont, dim3(nb(n)), dim3(256), 0, st, out, in, n);
}
// Device -> pinned host copy by the shader (the Montgomery write-back, prover.js:147-148): 16-byte
// non-temporal stores straight into the mapped host buffer from a small grid-stride grid. The copy is
// PCIe-bound (~52 GB/s, profiles/ubench/d2h_engine.hip); hipMemcpyAsync D2H ran either on an SDMA
// engine at ~30 GB/s or, with several proofs in flight, as the runtime's __amd_rocclr_copyBuffer blit
// kernel (256 x 512 threads for 0.8 ms per 32 MiB) whose waves kept the other proofs' kernels from
// co-residing. Few blocks and few VGPRs: the waves mostly wait on their stores.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(256) k_host_store(u32x4* __restrict__ dst, const u32x4* __restrict__ src, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(src[i], &dst[i]);
}
void launch_host_store(hipStream_t st, void* dst_host_mapped, const void* src, uint64_t bytes, unsigned blocks) {
  hipLaunchKernelGGL(k_host_store, dim3(blocks), dim3(256), 0, st, (u32x4*)dst_host_mapped, (const u32x4*)src, bytes / 16);
}
// [ffjs] Fr.batchFromMontgomery (polynomial.js:1112, before G1.multiExpAffine)
__global__ void k_from_mont(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, uint64_t n) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fr::load(in + 8 * i).from_mont().store(out + 8 * i);
}
void launch_from_mont(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n) {
  hipLaunchKernelGGL(k_from_mont, dim3(nb(n)), dim3(256), 0, st, out, in, n);
}

// ---------------------------------------------------------------------------- linear combination
__global__ void k_lincomb(uint32_t* __restrict__ out, uint64_t n, LinComb lc) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // the terms accumulate on [0, 2p) (29-bit products by the uniform coefficients, lazy sums), one
  // canonicalisation at the end: the same canonical value as the term-by-term modular sum
  fr acc = fr::zero();
  for (int k = 0; k < lc.nterms; k++) {
    if (i < lc.len[k]) {
      W29 c;
#pragma unroll
      for (int j = 0; j < 9; j++) c.l[j] = lc.coef29[k][j];
      acc = fr::add_lazy(acc, mul29(fr::load(lc.src[k] + 8 * i), c));
    }
  }
  if (i == 0) {
    fr c;
#pragma unroll
    for (int j = 0; j < 8; j++) c.v[j] = lc.c0[j];
    acc = fr::add_lazy(acc, c);
  }
  fr::reduce_once(acc).store(out + 8 * i);
}
void launch_lincomb(hipStream_t st, uint32_t* out, uint64_t n, const LinComb& lc) {
  hipLaunchKernelGGL(k_lincomb, dim3(nb(n)), dim3(256), 0, st, out, n, lc);
}

// ---------------------------------------------------------------------------- block scans
// Inclusive Hillis-Steele scan of one fr per thread over a 256-thread block, operator `op`.
// lds: 256*8 u32.
template <class Op>
__device__ __forceinline__ fr block_scan_incl(fr v, uint32_t* lds, Op op) {
  const int t = threadIdx.x;
  for (int off = 1; off < 256; off <<= 1) {
    v.store(lds + 8 * t);
    __syncthreads();
    if (t >= off) v = op(fr::load(lds + 8 * (t - off)), v);
    __syncthreads();
  }
  return v;
}
// inclusive suffix scan: result_t = op(v_t, op(v_{t+1}, ...))
template <class Op>
__device__ __forceinline__ fr block_suffix_incl(fr v, uint32_t* lds, Op op) {
  const int t = threadIdx.x;
  for (int off = 1; off < 256; off <<= 1) {
    v.store(lds + 8 * t);
    __syncthreads();
    if (t + off < 256) v = op(v, fr::load(lds + 8 * (t + off)));
    __syncthreads();
  }
  return v;
}

struct OpMul { __device__ fr operator()(const fr& a, const fr& b) const { return a * b; } };
struct OpAdd { __device__ fr operator()(const fr& a, const fr& b) const { return a + b; } };

// ---------------------------------------------------------------------------- builder
// Element i of the input produces num_i/den_i stored at position (i+1) mod n.
//  grand-sum  : f'=f+g, t'=t+g, num = t'*selF - f'*selT, den = f'*t'
//  grand-prod : num = selF*(f+g-1)+1, den = selT*(t+g-1)+1
template <bool PROD, bool SEL>
__device__ __forceinline__ void numden(uint64_t i, const uint32_t* f, const uint32_t* t, const uint32_t* sf,
                                       const uint32_t* stt, const fr& g, fr& num, fr& den) {
  fr fv = fr::load(f + 8 * i) + g;
  fr tv = fr::load(t + 8 * i) + g;
  if (!PROD) {
    if (SEL) {
      num = tv * fr::load(sf + 8 * i) - fv * fr::load(stt + 8 * i);
    } else {
      num = tv - fv;
    }
    den = fv * tv;
  } else {
    if (SEL) {
      const fr one = fr::one();
      num = fr::load(sf + 8 * i) * (fv - one) + one;
      den = fr::load(stt + 8 * i) * (tv - one) + one;
    } else {
      num = fv;
      den = tv;
    }
  }
}

constexpr int BT_PER = 8;                 // elements per thread
constexpr int BT_TILE = 256 * BT_PER;     // elements per tile (block)

template <bool PROD, bool SEL>
__global__ void __launch_bounds__(256) k_builder_tileprod(uint32_t* __restrict__ tileprod, const uint32_t* f,
                                                          const uint32_t* t, const uint32_t* sf, const uint32_t* st_,
                                                          const uint32_t* gp, uint64_t n) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[256 * 8];
  const fr g = fr::load(gp);
  const uint64_t base = (uint64_t)blockIdx.x * BT_TILE + threadIdx.x * BT_PER;
  fr p = fr::one();
  for (int r = 0; r < BT_PER; r++) {
    uint64_t i = base + r;
    if (i < n) {
      fr num, den;
      numden<PROD, SEL>(i, f, t, sf, st_, g, num, den);
      if (!den.is_zero()) p = p * den;
    }
  }
  p = block_scan_incl(p, lds, OpMul());
  if (threadIdx.x == 255) p.store(tileprod + 8 * (uint64_t)blockIdx.x);
}

// Single block: inverse of every tile product via prefix/suffix products and ONE inversion.
__global__ void __launch_bounds__(SCAN_NT) k_tile_inverse(uint32_t* __restrict__ tinv, const uint32_t* __restrict__ tp,
                                                       uint32_t ntiles) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[SCAN_NT * 8];
  __shared__ uint32_t tot[8];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ntiles + SCAN_NT - 1) / SCAN_NT;
  const uint32_t lo = t * per, hi = lo + per < ntiles ? lo + per : ntiles;
  fr p = fr::one();
  for (uint32_t b = lo; b < hi; b++) p = p * fr::load(tp + 8 * b);
  // inclusive prefix over threads
  fr pre = p;
  for (uint32_t off = 1; off < SCAN_NT; off <<= 1) {
    pre.store(lds + 8 * t);
    __syncthreads();
    if (t >= off) pre = fr::load(lds + 8 * (t - off)) * pre;
    __syncthreads();
  }
  fr suf = p;
  for (uint32_t off = 1; off < SCAN_NT; off <<= 1) {
    suf.store(lds + 8 * t);
    __syncthreads();
    if (t + off < SCAN_NT) suf = suf * fr::load(lds + 8 * (t + off));
    __syncthreads();
  }
  if (t == SCAN_NT - 1) {
    fr total_inv = pre.inverse_bgcd();  // one lane: binary Euclid (~5x fewer instructions than Fermat)
    total_inv.store(tot);
  }
  __syncthreads();
  const fr total_inv = fr::load(tot);
  // exclusive prefix / suffix of this thread's group
  pre.store(lds + 8 * t);
  __syncthreads();
  fr pex = t ? fr::load(lds + 8 * (t - 1)) : fr::one();
  __syncthreads();
  suf.store(lds + 8 * t);
  __syncthreads();
  fr sex = t < SCAN_NT - 1 ? fr::load(lds + 8 * (t + 1)) : fr::one();
  // inverse of this thread's group product, then walk its tiles
  fr ginv = total_inv * pex * sex;
  // within group: inverse of tile b = ginv * (prod of other tiles in group)
  // forward prefix in group then backward
  fr run = fr::one();
  for (uint32_t b = lo; b < hi; b++) {
    run.store(tinv + 8 * b);  // prefix before b (temporary)
    run = run * fr::load(tp + 8 * b);
  }
  fr acc = ginv;
  for (uint32_t b = hi; b-- > lo;) {
    fr prefix = fr::load(tinv + 8 * b);
    fr inv_b = acc * prefix;
    acc = acc * fr::load(tp + 8 * b);
    inv_b.store(tinv + 8 * b);
  }
}

// Per tile: element inverses (Montgomery trick seeded by the tile inverse), s_i = num_i/den_i,
// local inclusive scan (sum or product) inside the tile, written to out[(i+1) mod n].
template <bool PROD, bool SEL>
__global__ void __launch_bounds__(256) k_builder_finish(uint32_t* __restrict__ out, uint32_t* __restrict__ tileacc,
                                                        const uint32_t* __restrict__ tinv, const uint32_t* f,
                                                        const uint32_t* t, const uint32_t* sf, const uint32_t* st_,
                                                        const uint32_t* gp, uint64_t n) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[256 * 8];
  const fr g = fr::load(gp);
  const uint64_t base = (uint64_t)blockIdx.x * BT_TILE + threadIdx.x * BT_PER;
  // np[r] = num_r * (product of this thread's nonzero den_k, k < r), so that the backward pass needs
  // one product per element for s_r = num_r / den_r (np[r] * inv) and one to step inv: 4 products
  // per element instead of 5, and no separate num / prefix arrays (fits 176 VGPRs: co-resides with
  // the MSM bucket accumulation of other proofs in flight)
  fr np[BT_PER], den[BT_PER];
  fr p = fr::one();
#pragma unroll
  for (int r = 0; r < BT_PER; r++) {
    uint64_t i = base + r;
    fr num;
    if (i < n) {
      numden<PROD, SEL>(i, f, t, sf, st_, g, num, den[r]);
    } else {
      num = PROD ? fr::one() : fr::zero();
      den[r] = fr::one();
    }
    np[r] = num * p;
    if (!den[r].is_zero()) p = p * den[r];
  }
  // exclusive prefix/suffix of thread products inside the tile
  fr pin = block_scan_incl(p, lds, OpMul());
  fr sin = block_suffix_incl(p, lds, OpMul());
  pin.store(lds + 8 * threadIdx.x);
  __syncthreads();
  fr pex = threadIdx.x ? fr::load(lds + 8 * (threadIdx.x - 1)) : fr::one();
  __syncthreads();
  sin.store(lds + 8 * threadIdx.x);
  __syncthreads();
  fr sex = threadIdx.x < 255 ? fr::load(lds + 8 * (threadIdx.x + 1)) : fr::one();
  __syncthreads();
  fr inv = fr::load(tinv + 8 * (uint64_t)blockIdx.x) * pex * sex;  // 1/p
  // backward: inv = 1 / (prefix_r * den_r) before step r, so num_r / den_r = np[r] * inv; s_r
  // overwrites np[r]
#pragma unroll
  for (int r = BT_PER - 1; r >= 0; r--) {
    if (den[r].is_zero()) {
      np[r] = fr::zero();  // batchInverse(0) = 0 -> term 0
    } else {
      np[r] = np[r] * inv;
      inv = inv * den[r];
    }
  }
  // local inclusive scan inside thread, then across the tile
  fr loc = np[0];
#pragma unroll
  for (int r = 1; r < BT_PER; r++) loc = PROD ? loc * np[r] : loc + np[r];
  fr excl;
  if (PROD) {
    fr inc = block_scan_incl(loc, lds, OpMul());
    inc.store(lds + 8 * threadIdx.x);
    __syncthreads();
    excl = threadIdx.x ? fr::load(lds + 8 * (threadIdx.x - 1)) : fr::one();
    if (threadIdx.x == 255) inc.store(tileacc + 8 * (uint64_t)blockIdx.x);
  } else {
    fr inc = block_scan_incl(loc, lds, OpAdd());
    inc.store(lds + 8 * threadIdx.x);
    __syncthreads();
    excl = threadIdx.x ? fr::load(lds + 8 * (threadIdx.x - 1)) : fr::zero();
    if (threadIdx.x == 255) inc.store(tileacc + 8 * (uint64_t)blockIdx.x);
  }
  fr acc = excl;
#pragma unroll
  for (int r = 0; r < BT_PER; r++) {
    uint64_t i = base + r;
    acc = PROD ? acc * np[r] : acc + np[r];
    if (i < n) {
      uint64_t j = i + 1 == n ? 0 : i + 1;
      acc.store(out + 8 * j);
    }
  }
}

// Single block: exclusive scan of tile accumulators -> carry per tile (in place).
template <bool PROD>
__global__ void __launch_bounds__(SCAN_NT) k_tile_carry(uint32_t* __restrict__ acc, uint32_t ntiles) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[SCAN_NT * 8];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ntiles + SCAN_NT - 1) / SCAN_NT;
  const uint32_t lo = t * per, hi = lo + per < ntiles ? lo + per : ntiles;
  fr s = PROD ? fr::one() : fr::zero();
  for (uint32_t b = lo; b < hi; b++) s = PROD ? s * fr::load(acc + 8 * b) : s + fr::load(acc + 8 * b);
  fr inc = s;
  for (uint32_t off = 1; off < SCAN_NT; off <<= 1) {
    inc.store(lds + 8 * t);
    __syncthreads();
    if (t >= off) inc = PROD ? fr::load(lds + 8 * (t - off)) * inc : fr::load(lds + 8 * (t - off)) + inc;
    __syncthreads();
  }
  inc.store(lds + 8 * t);
  __syncthreads();
  fr run = t ? fr::load(lds + 8 * (t - 1)) : (PROD ? fr::one() : fr::zero());
  for (uint32_t b = lo; b < hi; b++) {
    fr v = fr::load(acc + 8 * b);
    run.store(acc + 8 * b);
    run = PROD ? run * v : run + v;
  }
}

// out[(i+1) mod n] (+|*)= carry[tile(i)]; flag if out[0] != (0 | 1)
template <bool PROD>
__global__ void k_apply_carry(uint32_t* __restrict__ out, const uint32_t* __restrict__ carry, uint64_t n,
                              uint32_t* __restrict__ flag) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t tile = i / BT_TILE;
  const uint64_t j = i + 1 == n ? 0 : i + 1;
  fr v = fr::load(out + 8 * j);
  if (tile) {
    fr c = fr::load(carry + 8 * tile);
    v = PROD ? v * c : v + c;
    v.store(out + 8 * j);
  }
  if (j == 0) {
    bool ok = PROD ? v == fr::one() : v.is_zero();
    if (!ok) atomicOr(flag, 1u);
  }
}

void launch_builder(hipStream_t st, bool prod, bool sel, uint32_t* out, const uint32_t* f, const uint32_t* t,
                    const uint32_t* sf, const uint32_t* stt, const uint32_t* gamma, uint64_t n,
                    uint32_t* scratch_tp, uint32_t* scratch_ti, uint32_t* flag) {
  const uint32_t ntiles = (uint32_t)((n + BT_TILE - 1) / BT_TILE);
#define KGS_BUILD(P, S)                                                                                      \
  hipLaunchKernelGGL((k_builder_tileprod<P, S>), dim3(ntiles), dim3(256), 0, st, scratch_tp, f, t, sf, stt, gamma, n); \
  hipLaunchKernelGGL(k_tile_inverse, dim3(1), dim3(SCAN_NT), 0, st, scratch_ti, scratch_tp, ntiles);                   \
  hipLaunchKernelGGL((k_builder_finish<P, S>), dim3(ntiles), dim3(256), 0, st, out, scratch_tp, scratch_ti, f, t, sf, \
                     stt, gamma, n);                                                                                  \
  hipLaunchKernelGGL((k_tile_carry<P>), dim3(1), dim3(SCAN_NT), 0, st, scratch_tp, ntiles);                             \
  hipLaunchKernelGGL((k_apply_carry<P>), dim3(nb(n)), dim3(256), 0, st, out, scratch_tp, n, flag);
  if (prod) {
    if (sel) { KGS_BUILD(true, true) } else { KGS_BUILD(true, false) }
  } else {
    if (sel) { KGS_BUILD(false, true) } else { KGS_BUILD(false, false) }
  }
#undef KGS_BUILD
}

// ---------------------------------------------------------------------------- quotient on a coset
// Inputs: coset evaluations in bit-reversed order (size cs = 2^lcs) of S (or Z), F, T [, selF, selT].
// rot = cs/n: S(w x_i) = S_eval[natural (i+rot) mod cs]. inv_nxm1[p] = 1/(n (x_i - 1)) (bitrev).
// zinv[0|1] = 1/Z_H(x_i) for even/odd natural i (cs = 2n) or zinv[0] for all (cs = n); k_quotient reads
// alpha * zinv[0|1] as 29-bit records (slots 5-6, 7-8).
template <bool PROD, bool SEL>
__global__ void __launch_bounds__(256) k_quotient(uint32_t* __restrict__ q, const uint32_t* __restrict__ S,
                                                  const uint32_t* __restrict__ F, const uint32_t* __restrict__ T,
                                                  const uint32_t* __restrict__ SF, const uint32_t* __restrict__ ST,
                                                  const uint32_t* __restrict__ inv_nxm1, const uint32_t* __restrict__ sc,
                                                  int lcs, uint32_t rot) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t cs = 1ull << lcs;
  if (p >= cs) return;
  // scalars: alpha, gamma, zinv0, zinv1, alpha_t (selected only)
  const fr alpha = fr::load(sc), gamma = fr::load(sc + 8);
  const uint32_t i = brev((uint32_t)p, lcs);
  const uint32_t j = (i + rot) & (uint32_t)(cs - 1);
  const uint32_t pj = brev(j, lcs);
  const fr s = fr::load(S + 8 * p), sw = fr::load(S + 8 * (uint64_t)pj);
  const fr sf = SEL ? fr::load(SF + 8 * p) : fr::zero(), st = SEL ? fr::load(ST + 8 * p) : fr::zero();
  const fr acc = quotient_core_na<PROD, SEL>(s, sw, fr::load(F + 8 * p), fr::load(T + 8 * p), sf, st, alpha, gamma,
                                             SEL ? fr::load(sc + 32) : fr::zero());
  // times alpha / Z_H(x_i) in one 29-bit product (records at scalar slots 5-6 / 7-8, prover.cpp)
  const W29 az = w29_load(sc + ((rot == 2 && (i & 1)) ? 56 : 40));
  (fr::reduce_once(mul29(acc, az)) + quotient_l1<PROD>(s, fr::load(inv_nxm1 + 8 * p))).store(q + 8 * p);
}

void launch_quotient(hipStream_t st, bool prod, bool sel, uint32_t* q, const uint32_t* S, const uint32_t* F,
                     const uint32_t* T, const uint32_t* SF, const uint32_t* ST, const uint32_t* inv_nxm1,
                     const uint32_t* scalars, int lcs, uint32_t rot) {
  uint64_t cs = 1ull << lcs;
#define KGS_Q(P, S_)                                                                                          \
  hipLaunchKernelGGL((k_quotient<P, S_>), dim3(nb(cs)), dim3(256), 0, st, q, S, F, T, SF, ST, inv_nxm1, scalars, lcs, rot);
  if (prod) {
    if (sel) { KGS_Q(true, true) } else { KGS_Q(true, false) }
  } else {
    if (sel) { KGS_Q(false, true) } else { KGS_Q(false, false) }
  }
#undef KGS_Q
}

// Divisibility of the quotient numerator by Z_H, evaluated on H (natural order): N(w^i) == 0.
// S_next: S at the natural index following the last one of this array (the wrap S[0] on one GPU,
// the next rank's first element when H is BLOCK-distributed); gbase: natural index of element 0.
template <bool PROD, bool SEL>
__global__ void k_divcheck(uint32_t* __restrict__ flag, const uint32_t* __restrict__ S, const uint32_t* __restrict__ f,
                           const uint32_t* __restrict__ t, const uint32_t* __restrict__ sfp, const uint32_t* __restrict__ stp,
                           const uint32_t* __restrict__ sc, uint64_t n, const uint32_t* __restrict__ S_next,
                           uint64_t gbase) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fr alpha = fr::load(sc), gamma = fr::load(sc + 8);
  const fr s = fr::load(S + 8 * i), sw = i + 1 == n ? fr::load(S_next) : fr::load(S + 8 * (i + 1));
  const fr sf = SEL ? fr::load(sfp + 8 * i) : fr::zero(), st = SEL ? fr::load(stp + 8 * i) : fr::zero();
  const fr acc = quotient_core_na<PROD, SEL>(s, sw, fr::load(f + 8 * i), fr::load(t + 8 * i), sf, st, alpha, gamma,
                                             SEL ? fr::load(sc + 32) : fr::zero());
  // N(w^i) = alpha * acc (+ L1 S at w^0): away from w^0 it is zero iff alpha or acc is (no product)
  const bool nz = gbase + i == 0 ? !(acc * alpha + (PROD ? s - fr::one() : s)).is_zero()  // L1(w^0) = 1
                                 : !alpha.is_zero() && !acc.is_zero();
  if (nz) atomicOr(flag, 1u);
}

void launch_divcheck(hipStream_t st, bool prod, bool sel, uint32_t* flag, const uint32_t* S, const uint32_t* f,
                     const uint32_t* t, const uint32_t* sf, const uint32_t* stt, const uint32_t* scalars, uint64_t n,
                     const uint32_t* S_next, uint64_t gbase) {
  if (!S_next) S_next = S;
#define KGS_D(P, S_) hipLaunchKernelGGL((k_divcheck<P, S_>), dim3(nb(n)), dim3(256), 0, st, flag, S, f, t, sf, stt, scalars, n, S_next, gbase);
  if (prod) {
    if (sel) { KGS_D(true, true) } else { KGS_D(true, false) }
  } else {
    if (sel) { KGS_D(false, true) } else { KGS_D(false, false) }
  }
#undef KGS_D
}

// ---------------------------------------------------------------------------- Horner tiles
// part[poly][tile] = sum_{j in tile} c_j x^(j - tile_start); tile = 2048 coefficients.
// xp[l] = x^(8 * 2^l), l = 0..7 ; x itself at xp[8], its 29-bit record at xp[10..11], xp[l]'s at
// xp[12 + 2l] (prover.cpp xpowers)
__global__ void __launch_bounds__(256) k_eval_tiles(uint32_t* __restrict__ part, EvalBatch eb,
                                                    const uint32_t* __restrict__ xp, uint32_t ntiles_max) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[256 * 8];
  const int pi = blockIdx.y;
  const uint32_t* c = eb.src[pi];
  const uint64_t len = eb.len[pi];
  const uint64_t base = (uint64_t)blockIdx.x * BT_TILE + threadIdx.x * BT_PER;
  // Horner steps with x as a 29-bit record (xp[10..11]): h stays in [0, 2p), canonical after the loop
  const W29 xw = w29_load(xp + 8 * 10);
  fr h = fr::zero();
#pragma unroll
  for (int r = BT_PER - 1; r >= 0; r--) {
    uint64_t i = base + r;
    fr ci = i < len ? fr::load(c + 8 * i) : fr::zero();
    h = mul29(h, xw) + ci;
  }
  h = fr::reduce_once(h);
  // tree over the 256 partials, level l combining the previous level's pairs (2k, 2k+1) as
  // v_2k + v_2k+1 * x^(8*2^l) in threads k < 128 >> l: the active threads are contiguous, so whole
  // waves drop out (9 wave-products for the tree instead of 27 when thread t of every stride ran)
  h.store(lds + 8 * threadIdx.x);
  __syncthreads();
  // (the level multipliers as 29-bit records, xp[12 + 2l]; partials on [0, 2p), canonical at the end)
  for (int l = 0, cnt = 128; l < 8; l++, cnt >>= 1) {
    const bool on = (int)threadIdx.x < cnt;
    fr v;
    if (on)
      v = fr::add_lazy(fr::load(lds + 8 * (2 * threadIdx.x)),
                       mul29(fr::load(lds + 8 * (2 * threadIdx.x + 1)), w29_load(xp + 8 * (12 + 2 * l))));
    __syncthreads();
    if (on) v.store(lds + 8 * threadIdx.x);
    __syncthreads();
  }
  if (threadIdx.x == 0) fr::reduce_once(fr::load(lds)).store(part + 8 * ((uint64_t)pi * ntiles_max + blockIdx.x));
}

void launch_eval_tiles(hipStream_t st, uint32_t* part, const EvalBatch& eb, const uint32_t* xp, uint32_t ntiles_max) {
  hipLaunchKernelGGL(k_eval_tiles, dim3(ntiles_max, eb.npolys), dim3(256), 0, st, part, eb, xp, ntiles_max);
}

// ---------------------------------------------------------------------------- synthetic division
// r_i = a_i + z r_{i+1} (r_L = 0); quotient q_{i-1} = r_i; r_0 must be 0.
// tile carries: carry[b] = r_{start of tile b+1}, from tile Horner values h_b (part) with Z = z^2048.
__global__ void __launch_bounds__(SCAN_NT) k_div_carries(uint32_t* __restrict__ carry, const uint32_t* __restrict__ h,
                                                      uint32_t ntiles, const uint32_t* __restrict__ zT) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[SCAN_NT * 8];
  const uint32_t t = threadIdx.x;
  const uint32_t per = (ntiles + SCAN_NT - 1) / SCAN_NT;
  const uint32_t lo = t * per, hi = lo + per < ntiles ? lo + per : ntiles;
  const fr Z = fr::load(zT);
  // group value: sum_{b in [lo,hi)} h_b Z^(b-lo), and Z^(hi-lo)
  fr v = fr::zero(), zp = fr::one();
  for (uint32_t b = hi; b-- > lo;) v = v * Z + fr::load(h + 8 * b);
  for (uint32_t b = lo; b < hi; b++) zp = zp * Z;
  // suffix scan over groups: V_t = v_t + zp_t * V_{t+1}; multipliers compose by product
  fr V = v, M = zp;
  for (uint32_t off = 1; off < SCAN_NT; off <<= 1) {
    V.store(lds + 8 * t);
    __syncthreads();
    fr Vn = t + off < SCAN_NT ? fr::load(lds + 8 * (t + off)) : fr::zero();
    __syncthreads();
    M.store(lds + 8 * t);
    __syncthreads();
    fr Mn = t + off < SCAN_NT ? fr::load(lds + 8 * (t + off)) : fr::one();
    __syncthreads();
    V = V + M * Vn;
    M = M * Mn;
  }
  // V is now the inclusive suffix value at group start lo; carry-in for this group = V_{t+1}
  V.store(lds + 8 * t);
  __syncthreads();
  fr cin = t + 1 < SCAN_NT ? fr::load(lds + 8 * (t + 1)) : fr::zero();
  for (uint32_t b = hi; b-- > lo;) {
    cin.store(carry + 8 * b);                 // r at start of tile b+1
    cin = fr::load(h + 8 * b) + Z * cin;      // r at start of tile b
  }
}

// xp layout (shared with k_eval_tiles): xp[l] = z^(8*2^l) (l = 0..7), xp[8] = z, xp[9] = z^2048,
// xp[10..11] = z's 29-bit record, xp[12 + 2l] = xp[l]'s record.
__global__ void __launch_bounds__(256) k_div_finish(uint32_t* __restrict__ q, uint32_t* __restrict__ flag,
                                                    const uint32_t* __restrict__ a, uint64_t L,
                                                    const uint32_t* __restrict__ carry, const uint32_t* __restrict__ xp) {
  KGS_AUX_PRIO();
  __shared__ uint32_t lds[256 * 8];
  const W29 zw = w29_load(xp + 8 * 10);  // z as a 29-bit record
  const uint64_t base = (uint64_t)blockIdx.x * BT_TILE + threadIdx.x * BT_PER;
  fr av[BT_PER];
  fr h = fr::zero();
#pragma unroll
  for (int r = BT_PER - 1; r >= 0; r--) {
    uint64_t i = base + r;
    av[r] = i < L ? fr::load(a + 8 * i) : fr::zero();
    h = mul29(h, zw) + av[r];  // [0, 2p)
  }
  h = fr::reduce_once(h);
  const fr cin_tile = fr::load(carry + 8 * (uint64_t)blockIdx.x);
  if (threadIdx.x == 255) h = h + fr::load(xp) * cin_tile;  // z^8 * carry
  // inclusive suffix scan: V_t = h_t + z^8 V_{t+1}; at step l the multiplier is z^(8*2^l) (its
  // 29-bit record xp[12 + 2l]; partials on [0, 2p), reduced where they are used below)
  for (int l = 0; l < 8; l++) {
    const int off = 1 << l;
    h.store(lds + 8 * threadIdx.x);
    __syncthreads();
    if (threadIdx.x + off < 256)
      h = fr::add_lazy(h, mul29(fr::load(lds + 8 * (threadIdx.x + off)), w29_load(xp + 8 * (12 + 2 * l))));
    __syncthreads();
  }
  h.store(lds + 8 * threadIdx.x);
  __syncthreads();
  fr r = threadIdx.x < 255 ? fr::load(lds + 8 * (threadIdx.x + 1)) : cin_tile;
#pragma unroll
  for (int k = BT_PER - 1; k >= 0; k--) {
    uint64_t i = base + k;
    r = av[k] + fr::reduce_once(mul29(r, zw));  // r_i, canonical
    if (i < L) {
      if (i >= 1) r.store(q + 8 * (i - 1));
      else if (!r.is_zero()) atomicOr(flag, 1u);
    }
  }
}

void launch_divide(hipStream_t st, uint32_t* q, uint32_t* flag, const uint32_t* a, uint64_t L, const uint32_t* xp,
                   uint32_t* part, uint32_t* carry) {
  const uint32_t ntiles = (uint32_t)((L + BT_TILE - 1) / BT_TILE);
  EvalBatch eb;
  eb.npolys = 1;
  eb.src[0] = a;
  eb.len[0] = L;
  hipMemsetAsync(q + 8 * (L - 1), 0, 32, st);
  hipLaunchKernelGGL(k_eval_tiles, dim3(ntiles, 1), dim3(256), 0, st, part, eb, xp, ntiles);
  hipLaunchKernelGGL(k_div_carries, dim3(1), dim3(SCAN_NT), 0, st, carry, part, ntiles, xp + 8 * 9);
  hipLaunchKernelGGL(k_div_finish, dim3(ntiles), dim3(256), 0, st, q, flag, a, L, carry, xp);
}

// ---------------------------------------------------------------------------- Fr batch inverse
// out[i] = in[i]^-1 (0 -> 0), per-thread Montgomery trick over CH elements (domain setup only).
__global__ void k_fr_batch_inv(uint32_t* __restrict__ out, const uint32_t* __restrict__ in, uint64_t n, uint32_t ch) {
  KGS_AUX_PRIO();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t start = t * ch;
  if (start >= n) return;
  const uint64_t end = start + ch < n ? start + ch : n;
  fr acc = fr::one();
  for (uint64_t i = start; i < end; i++) {
    acc.store(out + 8 * i);
    fr v = fr::load(in + 8 * i);
    if (!v.is_zero()) acc = acc * v;
  }
  fr inv = acc.inverse();
  for (uint64_t i = end; i-- > start;) {
    fr v = fr::load(in + 8 * i);
    if (v.is_zero()) { fr::zero().store(out + 8 * i); continue; }
    fr pre = fr::load(out + 8 * i);
    (inv * pre).store(out + 8 * i);
    inv = inv * v;
  }
}
void launch_fr_batch_inv(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t n) {
  const uint32_t ch = 32;
  hipLaunchKernelGGL(k_fr_batch_inv, dim3(nb((n + ch - 1) / ch)), dim3(256), 0, st, out, in, n, ch);
}

// x_i = g w_cs^i (natural) -> n (x_i - 1) stored at bitrev position (domain setup only).
// tw holds w_M^j for j < M/2; w_M^(j + M/2) = -w_M^j.
__global__ void k_nxm1(uint32_t* __restrict__ out, const uint32_t* __restrict__ tw, uint64_t halfM,
                       const uint32_t* __restrict__ gp, const uint32_t* __restrict__ np, int lcs, uint64_t wstride) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1ull << lcs)) return;
  uint64_t e = i * wstride;
  fr w = e < halfM ? fr::load(tw + 8 * e) : fr::load(tw + 8 * (e - halfM)).neg();
  fr x = fr::load(gp) * w;
  fr v = fr::load(np) * (x - fr::one());
  v.store(out + 8 * (uint64_t)brev((uint32_t)i, lcs));
}
void launch_nxm1(hipStream_t st, uint32_t* out, const uint32_t* tw, uint64_t halfM, const uint32_t* gp,
                 const uint32_t* np, int lcs, uint64_t wstride) {
  hipLaunchKernelGGL(k_nxm1, dim3(nb(1ull << lcs)), dim3(256), 0, st, out, tw, halfM, gp, np, lcs, wstride);
}


// ---------------------------------------------------------------------------- reference-quirks mode
// (kgs_ctx_set_reference_quirks; prover.cpp ref_quirks_quotient). Not on the default path: these
// kernels replay the reference's own `multiply` / `shiftOmega` / `divZh` buffer semantics on the GPU.

// Polynomial.degree (polynomial.js:212-226): *out = max(*out, highest index i > 0 with a[i] != 0);
// *out is zeroed by the caller. A fixed grid of DEG_WAVES waves walks the vector downward from its
// top end in 64-element chunks (wave w takes chunks w, w + DEG_WAVES, ...); a wave stops at its first
// chunk with a nonzero element (everything it would read later is lower) or once its next chunk lies
// below the maximum already found. A polynomial of full degree thus costs one chunk per wave and at
// most one atomic each; the zero polynomial one streaming pass. (One atomic per wave over the whole
// vector serialised on the one address: ~0.2 ms per 2^20 elements, ~1 ms per proof in
// reference-quirks mode.)
constexpr unsigned DEG_WAVES = 256;
__global__ void __launch_bounds__(256) k_degree(uint32_t* __restrict__ out, const uint32_t* __restrict__ a, uint64_t len) {
  KGS_AUX_PRIO();
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t w = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  for (uint64_t c = w;; c += DEG_WAVES) {
    const uint64_t top = len - 1 - 64 * c;  // highest index of chunk c
    if (64 * c + 1 >= len) break;           // (indices >= 1 only)
    if (top <= __hip_atomic_load(out, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
    const uint64_t i = top - lane;
    uint32_t d = 0;
    if (lane <= top - 1) {  // i >= 1
      const uint4 x = *(const uint4*)(a + 8 * i);
      const uint4 y = *(const uint4*)(a + 8 * i + 4);
      if (x.x | x.y | x.z | x.w | y.x | y.y | y.z | y.w) d = (uint32_t)i;
    }
    for (int o = 32; o > 0; o >>= 1) d = max(d, (uint32_t)__shfl_xor((int)d, o));
    if (d) {
      if (lane == 0) atomicMax(out, d);
      break;
    }
  }
}
void launch_degree(hipStream_t st, uint32_t* out, const uint32_t* a, uint64_t len) {
  if (len > 1) hipLaunchKernelGGL(k_degree, dim3(DEG_WAVES / 4), dim3(256), 0, st, out, a, len);
}

// The pointwise step of Polynomial.multiply / shiftOmega (polynomial.js:366-376, 378-393) on the
// reference's own evaluation domains: a (2^loga points) and b (2^logb points) are DIF outputs
// (bit-reversed order); out[i] = a_nat[(i + rot) mod 2^loga] * b_nat[i] for i < N, natural order
// (b == nullptr: factor 1). The reference takes the FIRST N natural-order evaluations of each
// operand's transform, whatever its size (evaluations.js:12-18).
__global__ void k_ref_gather_mul(uint32_t* __restrict__ out, const uint32_t* __restrict__ a, int loga,
                                 const uint32_t* __restrict__ b, int logb, uint64_t N, uint64_t rot) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  const uint32_t ia = (uint32_t)((i + rot) & ((1ull << loga) - 1));
  fr x = fr::load(a + 8 * (uint64_t)brev(ia, loga));
  if (b) x = x * fr::load(b + 8 * (uint64_t)brev((uint32_t)i, logb));
  x.store(out + 8 * i);
}
void launch_ref_gather_mul(hipStream_t st, uint32_t* out, const uint32_t* a, int loga, const uint32_t* b, int logb,
                           uint64_t N, uint64_t rot) {
  hipLaunchKernelGGL(k_ref_gather_mul, dim3(nb(N)), dim3(256), 0, st, out, a, loga, b, logb, N, rot);
}

// Polynomial.divZh (polynomial.js:853-888) in place, one thread per residue r < n:
//   c[r] = -c[r]; c[r + t n] = c[r + (t-1) n] - c[r + t n] for t < ext,
// flagging "Polynomial is not divisible" for a nonzero value at i > n (ext - 1) - ext.
__global__ void k_ref_divzh(uint32_t* __restrict__ c, uint64_t n, uint32_t ext, uint32_t* __restrict__ flag) {
  KGS_AUX_PRIO();
  const uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n) return;
  fr acc = fr::zero() - fr::load(c + 8 * r);
  acc.store(c + 8 * r);
  const int64_t lim = (int64_t)n * (int64_t)(ext - 1) - (int64_t)ext;
  bool bad = false;
  for (uint32_t t = 1; t < ext; t++) {
    const uint64_t i = r + (uint64_t)t * n;
    acc = acc - fr::load(c + 8 * i);
    acc.store(c + 8 * i);
    if ((int64_t)i > lim && !acc.is_zero()) bad = true;
  }
  if (bad) *flag = 1;
}
void launch_ref_divzh(hipStream_t st, uint32_t* c, uint64_t n, uint32_t ext, uint32_t* flag) {
  hipLaunchKernelGGL(k_ref_divzh, dim3(nb(n)), dim3(256), 0, st, c, n, ext, flag);
}

}  // namespace kgs
