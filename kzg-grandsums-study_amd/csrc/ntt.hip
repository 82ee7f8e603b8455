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
// Twiddles: per direction one resident STAGE table tw[h + t] = w_{2h}^t (t < h, h = 1..M/2; M
// entries for the largest domain M), so the butterflies of one stage read consecutive twiddles
// (coalesced: consecutive lanes have consecutive t) instead of a strided walk through w_M^j.
#include "kernels.hpp"

namespace kgs {

__device__ __forceinline__ uint32_t bitrev(uint32_t x, int bits) {
  return __builtin_bitreverse32(x) >> (32 - bits);
}

// One pass of K DIF stages starting at global stage s0 (stage s has half-distance m >> (s+1)).
// If `in` != nullptr this is the first pass: read in[idx] (zero beyond in_len), optionally
// scaled by pre[idx], and write to `data`.
template <int K>
__global__ void __launch_bounds__(256) k_ntt_dif_pass(uint32_t* __restrict__ data,
                                                      const uint32_t* __restrict__ in, uint64_t in_len,
                                                      const uint32_t* __restrict__ pre,
                                                      const uint32_t* __restrict__ tw, int logM, int logm,
                                                      int s0) {
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
      fr a = x[r], b = x[r + dist];
      x[r] = a + b;
      fr diff = a - b;
      if (t) diff = diff * fr::load(tw + 8 * (twbase + t));
      x[r + dist] = diff;
    }
  }
#pragma unroll
  for (int r = 0; r < (1 << K); r++) x[r].store(data + 8 * (base + ((uint64_t)r << logd)));
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
      fr a = x[r], b = x[r + dist];
      if (t) b = b * fr::load(tw + 8 * (twbase + t));
      x[r] = a + b;
      x[r + dist] = a - b;
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
    y.store(data + 8 * idx);
  }
}

static inline unsigned nblocks(uint64_t work, unsigned bs = 256) { return (unsigned)((work + bs - 1) / bs); }

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
  int s0 = 0;
  bool first = true;
  while (s0 < logm) {
    int K = logm - s0 >= 3 ? 3 : logm - s0;
    uint64_t groups = (1ull << logm) >> K;
    const uint32_t* src = first ? in : nullptr;
    const uint32_t* p = first ? pre : nullptr;
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
  // passes: the first pass handles the remainder so the last pass is a full radix-8 one
  int rem = logm % 3;
  int s0 = 0;
  bool first = true;
  while (s0 < logm) {
    int K = first && rem ? rem : 3;
    if (K > logm - s0) K = logm - s0;
    uint64_t groups = (1ull << logm) >> K;
    const uint32_t* src = first ? in : nullptr;
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
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1ull << logm)) return;
  uint64_t j = logm ? bitrev((uint32_t)i, logm) : 0;
  fr::load(in + 8 * j).store(out + 8 * i);
}

void launch_bitrev_copy(hipStream_t st, uint32_t* out, const uint32_t* in, int logm) {
  hipLaunchKernelGGL(k_bitrev_copy, dim3(nblocks(1ull << logm)), dim3(256), 0, st, out, in, logm);
}

}  // namespace kgs
