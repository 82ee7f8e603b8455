// Kernels of the distributed prover (prover_dist.cpp): the rank-local halves of the distributed
// NTT, the layout changes around the all-to-alls, and the rank-local parts of the builder scan,
// quotient and synthetic division. Layouts (tests/test_dist_layouts.py is the executable spec),
// for a vector of N elements over W ranks, M = N / W, b = M / W, rank r:
//   BLOCK  : natural indices [r M, (r+1) M)
//   CYCLIC : indices r + W j, j < N / W (any length)
//   E      : indices k1 M + r b + t (k1 < W, t < b), stored as W blocks of b (block k1 at k1 b)
// Forward DFT CYCLIC -> E: local M-point DIF (bit-reversed out) -> k_dfwd_pack (twiddle w_N^(r k2),
// chunk by k2) -> all-to-all -> k_dfwd_wdft (W-point DFT over the source rank).
// Inverse DFT E -> CYCLIC: k_dinv_wdft_pack (W-point inverse DFT over k1, twiddle w_N^-(n1 k2),
// chunk by n1) -> all-to-all -> local M-point DIT from natural order with 1/N (and coset) folded in.
// Twiddles come from the resident stage table of size N: w_N^e = tw[N/2 + e] (e < N/2),
// -tw[N/2 + e - N/2] otherwise (ntt.hip layout).
#include "kernels.hpp"
#include "poly_math.hpp"

namespace kgs {

static inline unsigned nbk(uint64_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) { return bits ? __brev(x) >> (32 - bits) : 0u; }

// w_N^e for 0 <= e < N from the stage table of size N (tw points at tw_base + 8 * N/2)
__device__ __forceinline__ fr wpow(const uint32_t* tw, uint64_t e, uint64_t halfN) {
  return e < halfN ? fr::load(tw + 8 * e) : fr::load(tw + 8 * (e - halfN)).neg();
}

// global natural index of local position p in the E layout
__device__ __forceinline__ uint64_t e_global(uint64_t p, uint64_t M, uint64_t b, uint32_t r) {
  return (p / b) * M + (uint64_t)r * b + (p % b);
}

// out[p] = in[e_global(p)] (TO_MONT: standard-form input converted to Montgomery)
template <bool TO_MONT>
__global__ void __launch_bounds__(256) k_gather_e(uint32_t* __restrict__ out, const uint32_t* __restrict__ in,
                                                  uint64_t M, uint64_t b, uint32_t r) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= M) return;
  fr x = fr::load(in + 8 * e_global(p, M, b, r));
  if (TO_MONT) x = x.to_mont();
  x.store(out + 8 * p);
}

void launch_gather_e(hipStream_t st, uint32_t* out, const uint32_t* in, uint64_t N, int W, int r, bool to_mont) {
  const uint64_t M = N / W, b = M / W;
  if (to_mont)
    hipLaunchKernelGGL(k_gather_e<true>, dim3(nbk(M)), dim3(256), 0, st, out, in, M, b, (uint32_t)r);
  else
    hipLaunchKernelGGL(k_gather_e<false>, dim3(nbk(M)), dim3(256), 0, st, out, in, M, b, (uint32_t)r);
}

// Z (local DIF output, bit-reversed over logMl bits) -> send: k2 = bitrev(p), value * w_N^(r k2),
// chunk j = k2 / b at offset k2 % b
__global__ void __launch_bounds__(256) k_dfwd_pack(uint32_t* __restrict__ send, const uint32_t* __restrict__ Z,
                                                   int logMl, uint64_t b, uint32_t r, const uint32_t* __restrict__ twN,
                                                   uint64_t halfN) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >> logMl) return;
  const uint64_t k2 = bitrev((uint32_t)p, logMl);
  fr v = fr::load(Z + 8 * p);
  const uint64_t e = (uint64_t)r * k2;  // < N
  if (e) v = v * wpow(twN, e, halfN);
  v.store(send + 8 * ((k2 / b) * b + (k2 % b)));
}

// recv chunk n1 (from rank n1) holds, at offset t, Z'_{n1}[r b + t]; out E block k1 at offset t:
// X[k1 M + r b + t] = sum_n1 Z'_{n1} w_W^(n1 k1), w_W = w_N^M
template <int W>
__global__ void __launch_bounds__(256) k_dfwd_wdft(uint32_t* __restrict__ out, const uint32_t* __restrict__ recv,
                                                   uint64_t b, uint64_t M, const uint32_t* __restrict__ twN,
                                                   uint64_t halfN) {
  KGS_AUX_PRIO();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= b) return;
  fr v[W], w[W];
#pragma unroll
  for (int n1 = 0; n1 < W; n1++) {
    v[n1] = fr::load(recv + 8 * ((uint64_t)n1 * b + t));
    w[n1] = wpow(twN, (uint64_t)n1 * M, halfN);  // w_W^n1
  }
#pragma unroll
  for (int k1 = 0; k1 < W; k1++) {
    fr acc = v[0];
#pragma unroll
    for (int n1 = 1; n1 < W; n1++) acc = acc + v[n1] * w[(n1 * k1) % W];
    acc.store(out + 8 * ((uint64_t)k1 * b + t));
  }
}

// E block k1 at offset t = X[k1 M + r b + t] -> y[n1] = sum_k1 X w_W^-(n1 k1), times w_N^-(n1 k2),
// k2 = r b + t -> send chunk n1 at offset t
template <int W>
__global__ void __launch_bounds__(256) k_dinv_wdft_pack(uint32_t* __restrict__ send, const uint32_t* __restrict__ loc,
                                                        uint64_t b, uint64_t M, uint32_t r,
                                                        const uint32_t* __restrict__ twiN, uint64_t halfN) {
  KGS_AUX_PRIO();
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= b) return;
  const uint64_t k2 = (uint64_t)r * b + t;
  fr v[W], w[W];
#pragma unroll
  for (int k1 = 0; k1 < W; k1++) {
    v[k1] = fr::load(loc + 8 * ((uint64_t)k1 * b + t));
    w[k1] = wpow(twiN, (uint64_t)k1 * M, halfN);  // w_W^-k1
  }
#pragma unroll
  for (int n1 = 0; n1 < W; n1++) {
    fr acc = v[0];
#pragma unroll
    for (int k1 = 1; k1 < W; k1++) acc = acc + v[k1] * w[(n1 * k1) % W];
    const uint64_t e = (uint64_t)n1 * k2;
    if (e) acc = acc * wpow(twiN, e, halfN);
    acc.store(send + 8 * ((uint64_t)n1 * b + t));
  }
}

#define KGS_W_SWITCH(W, CALL) \
  switch (W) {                \
    case 1: CALL(1); break;   \
    case 2: CALL(2); break;   \
    case 4: CALL(4); break;   \
    case 8: CALL(8); break;   \
    case 16: CALL(16); break; \
    default: break;           \
  }

void launch_dfwd_pack(hipStream_t st, uint32_t* send, const uint32_t* Z, int logMl, int W, int r, const uint32_t* tw,
                      int logN) {
  const uint64_t Ml = 1ull << logMl, b = Ml / W, halfN = (1ull << logN) / 2;
  hipLaunchKernelGGL(k_dfwd_pack, dim3(nbk(Ml)), dim3(256), 0, st, send, Z, logMl, b, (uint32_t)r, tw + 8 * halfN, halfN);
}

void launch_dfwd_wdft(hipStream_t st, uint32_t* out, const uint32_t* recv, int logMl, int W, const uint32_t* tw,
                      int logN) {
  const uint64_t Ml = 1ull << logMl, b = Ml / W, halfN = (1ull << logN) / 2;
#define KGS_FW(WW) hipLaunchKernelGGL(k_dfwd_wdft<WW>, dim3(nbk(b)), dim3(256), 0, st, out, recv, b, Ml, tw + 8 * halfN, halfN)
  KGS_W_SWITCH(W, KGS_FW)
#undef KGS_FW
}

void launch_dinv_wdft_pack(hipStream_t st, uint32_t* send, const uint32_t* loc, int logMl, int W, int r,
                           const uint32_t* tw_inv, int logN) {
  const uint64_t Ml = 1ull << logMl, b = Ml / W, halfN = (1ull << logN) / 2;
#define KGS_IW(WW)                                                                                             \
  hipLaunchKernelGGL(k_dinv_wdft_pack<WW>, dim3(nbk(b)), dim3(256), 0, st, send, loc, b, Ml, (uint32_t)r, \
                     tw_inv + 8 * halfN, halfN)
  KGS_W_SWITCH(W, KGS_IW)
#undef KGS_IW
}

// CYCLIC -> BLOCK receive side: out[src + W t] = recv[src c2 + t] (c2 = L / W^2)
__global__ void __launch_bounds__(256) k_unpack_c2b(uint32_t* __restrict__ out, const uint32_t* __restrict__ recv,
                                                    uint64_t Lb, uint32_t W) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // position in recv
  if (p >= Lb) return;
  const uint64_t c2 = Lb / W;
  const uint64_t src = p / c2, t = p % c2;
  fr::load(recv + 8 * p).store(out + 8 * (src + (uint64_t)W * t));
}

void launch_unpack_c2b(hipStream_t st, uint32_t* out, const uint32_t* recv, uint64_t Lb, int W) {
  hipLaunchKernelGGL(k_unpack_c2b, dim3(nbk(Lb)), dim3(256), 0, st, out, recv, Lb, (uint32_t)W);
}

// BLOCK -> CYCLIC send side (the inverse of k_unpack_c2b): send[d c2 + t] = blk[d + W t]; rank d
// receives from every source rank r the c2 = Lb / W elements r M + d + W t, i.e. its cyclic
// positions r c2 + t, so the received buffer is the cyclic slice in natural order
__global__ void __launch_bounds__(256) k_pack_b2c(uint32_t* __restrict__ send, const uint32_t* __restrict__ blk,
                                                  uint64_t Lb, uint32_t W) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;  // position in send
  if (p >= Lb) return;
  const uint64_t c2 = Lb / W;
  const uint64_t d = p / c2, t = p % c2;
  fr::load(blk + 8 * (d + (uint64_t)W * t)).store(send + 8 * p);
}

void launch_pack_b2c(hipStream_t st, uint32_t* send, const uint32_t* blk, uint64_t Lb, int W) {
  hipLaunchKernelGGL(k_pack_b2c, dim3(nbk(Lb)), dim3(256), 0, st, send, blk, Lb, (uint32_t)W);
}

// builder scan across ranks: the local builder left out[0] = local total and out[i] = local
// exclusive scan (i >= 1); with off = the op-sum of the lower ranks' totals: out[0] = off,
// out[i] = off (+|*) out[i]
template <bool PROD>
__global__ void __launch_bounds__(256) k_scan_fix(uint32_t* __restrict__ out, const uint32_t* __restrict__ offp,
                                                  uint64_t n) {
  KGS_AUX_PRIO();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fr off = fr::load(offp);
  if (i == 0) {
    off.store(out);
    return;
  }
  const fr v = fr::load(out + 8 * i);
  (PROD ? off * v : off + v).store(out + 8 * i);
}

void launch_scan_fix(hipStream_t st, bool prod, uint32_t* out, const uint32_t* off, uint64_t n) {
  if (prod)
    hipLaunchKernelGGL(k_scan_fix<true>, dim3(nbk(n)), dim3(256), 0, st, out, off, n);
  else
    hipLaunchKernelGGL(k_scan_fix<false>, dim3(nbk(n)), dim3(256), 0, st, out, off, n);
}

// first `rot` elements of each E block: halo[k1 rot + u] = S[k1 b + u]
__global__ void k_e_heads(uint32_t* __restrict__ heads, const uint32_t* __restrict__ S, uint64_t b, uint32_t W,
                          uint32_t rot) {
  KGS_AUX_PRIO();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= W * rot) return;
  fr::load(S + 8 * ((uint64_t)(i / rot) * b + (i % rot))).store(heads + 8 * (uint64_t)i);
}

void launch_e_heads(hipStream_t st, uint32_t* heads, const uint32_t* S, uint64_t Ml, int W, int rot) {
  hipLaunchKernelGGL(k_e_heads, dim3(1), dim3(64), 0, st, heads, S, Ml / W, (uint32_t)W, (uint32_t)rot);
}

// quotient on E-distributed coset evaluations (natural order inside each block). Scalars: alpha,
// gamma, zinv0, zinv1, alpha_t (selected only). S(w x_i) = S[i + rot]: the same block at p + rot, or halo[k1 rot + ...] (the
// next chunk's first elements) past the block's end. nxm1[p] = 1/(n (x_i - 1)).
template <bool PROD, bool SEL>
__global__ void __launch_bounds__(256) k_quotient_e(uint32_t* __restrict__ q, const uint32_t* __restrict__ S,
                                                    const uint32_t* __restrict__ F, const uint32_t* __restrict__ T,
                                                    const uint32_t* __restrict__ SF, const uint32_t* __restrict__ ST,
                                                    const uint32_t* __restrict__ nxm1, const uint32_t* __restrict__ sc,
                                                    const uint32_t* __restrict__ halo, uint64_t Ml, uint64_t b,
                                                    uint32_t r, uint32_t rot) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Ml) return;
  const fr alpha = fr::load(sc), gamma = fr::load(sc + 8), z0 = fr::load(sc + 16), z1 = fr::load(sc + 24);
  const uint64_t k1 = p / b, t = p % b;
  const uint64_t gi = e_global(p, Ml, b, r);
  const fr s = fr::load(S + 8 * p);
  const fr sw = t + rot < b ? fr::load(S + 8 * (p + rot)) : fr::load(halo + 8 * (k1 * rot + (t + rot - b)));
  const fr sf = SEL ? fr::load(SF + 8 * p) : fr::zero(), st = SEL ? fr::load(ST + 8 * p) : fr::zero();
  fr acc = quotient_core<PROD, SEL>(s, sw, fr::load(F + 8 * p), fr::load(T + 8 * p), sf, st, alpha, gamma,
                                            SEL ? fr::load(sc + 32) : fr::zero());
  const fr zinv = (rot == 2 && (gi & 1)) ? z1 : z0;
  acc = acc * zinv + quotient_l1<PROD>(s, fr::load(nxm1 + 8 * p));
  acc.store(q + 8 * p);
}

void launch_quotient_e(hipStream_t st, bool prod, bool sel, uint32_t* q, const uint32_t* S, const uint32_t* F,
                       const uint32_t* T, const uint32_t* SF, const uint32_t* ST, const uint32_t* nxm1,
                       const uint32_t* scalars, const uint32_t* halo, uint64_t Ml, int W, int r, int rot) {
  const uint64_t b = Ml / W;
#define KGS_QE(P, S_)                                                                                              \
  hipLaunchKernelGGL((k_quotient_e<P, S_>), dim3(nbk(Ml)), dim3(256), 0, st, q, S, F, T, SF, ST, nxm1, scalars, halo, \
                     Ml, b, (uint32_t)r, (uint32_t)rot);
  if (prod) {
    if (sel) { KGS_QE(true, true) } else { KGS_QE(true, false) }
  } else {
    if (sel) { KGS_QE(false, true) } else { KGS_QE(false, false) }
  }
#undef KGS_QE
}

// n (x_i - 1) for the E-layout coset points x_i = g w_cs^i (the caller batch-inverts)
__global__ void __launch_bounds__(256) k_nxm1_e(uint32_t* __restrict__ out, const uint32_t* __restrict__ twcs,
                                                uint64_t halfcs, const uint32_t* __restrict__ gp,
                                                const uint32_t* __restrict__ np, uint64_t Ml, uint64_t b, uint32_t r) {
  KGS_AUX_PRIO();
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= Ml) return;
  const fr x = fr::load(gp) * wpow(twcs, e_global(p, Ml, b, r), halfcs);
  (fr::load(np) * (x - fr::one())).store(out + 8 * p);
}

void launch_nxm1_e(hipStream_t st, uint32_t* out, const uint32_t* tw, int lcs, const uint32_t* gp, const uint32_t* np,
                   int W, int r) {
  const uint64_t cs = 1ull << lcs, Ml = cs / W, halfcs = cs / 2;
  hipLaunchKernelGGL(k_nxm1_e, dim3(nbk(Ml)), dim3(256), 0, st, out, tw + 8 * halfcs, halfcs, gp, np, Ml, Ml / W,
                     (uint32_t)r);
}

// division fix-up on a BLOCK slice: q[j] += z^(Lb - 1 - j) c  (pz[e] = z^e)
__global__ void __launch_bounds__(256) k_div_fix(uint32_t* __restrict__ q, const uint32_t* __restrict__ pz,
                                                 const uint32_t* __restrict__ cp, uint64_t Lb) {
  KGS_AUX_PRIO();
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Lb) return;
  const fr c = fr::load(cp);
  (fr::load(q + 8 * j) + fr::load(pz + 8 * (Lb - 1 - j)) * c).store(q + 8 * j);
}

void launch_div_fix(hipStream_t st, uint32_t* q, const uint32_t* pz, const uint32_t* c, uint64_t Lb) {
  hipLaunchKernelGGL(k_div_fix, dim3(nbk(Lb)), dim3(256), 0, st, q, pz, c, Lb);
}

}  // namespace kgs
