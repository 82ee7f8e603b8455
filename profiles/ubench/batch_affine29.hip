// Microbenchmark behind DESIGN.md §3 "Batch-affine bucket accumulation: measured, rejected".
//
// Question: does replacing the XYZZ mixed add of k_accumulate (8M + 2S, 1,467 mads in 9 x 29-bit
// limbs) by affine additions whose inversions are batched with Montgomery's trick pay on gfx950?
// An affine add costs 5M + 1S per point (prefix product, two backward products, lambda, lambda^2,
// lambda*(x1 - x3)) = 936 mads, plus 1/K of one field inversion when a thread batches K
// independent chains (a bucket's points are a dependent chain, so the batch must span K chains per
// thread: SIMT lanes each pay for their own inversion, spreading one inversion over lanes costs the
// same issue slots). This file measures, register-resident like madd29.hip (no gathers, no bucket
// boundaries, synthetic operands — an upper bound for a real kernel):
//   * per-lane inversion throughput: Fermat a^(q-2) in fq29 (square-and-multiply), and the binary
//     extended Euclid of field.hpp (fq::inverse_bgcd) with all 64 lanes active (divergent);
//   * the batch-affine add rate for K = 2, 4, 8 chains per thread with either inversion;
//   * the production XYZZ mixed add (g1_acc29::add_aff) in the same harness, for reference.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../kzg-grandsums-study_amd/csrc/field29.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

// q - 2 as 8 x 32-bit words (little-endian)
__constant__ uint32_t QM2[8] = {0xd87cfd45u, 0x3c208c16u, 0x6871ca8du, 0x97816a91u,
                                0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};

// Montgomery power a^(q-2) = inverse in the x*2^261 form; square-and-multiply from the top bit
__device__ __forceinline__ fq29 inv_fermat(const fq29& a) {
  fq29 r = fq29::from(f29::ONE);
  for (int b = 253; b >= 0; b--) {
    r = fq29::sqr(r);
    if ((QM2[b >> 5] >> (b & 31)) & 1u) r = fq29::mul(r, a);  // uniform branch (same exponent)
  }
  return r;
}

// binary extended Euclid on the canonical 256-bit form (field.hpp), converted in and out
__device__ __forceinline__ fq29 inv_bgcd(const fq29& a) {
  const fq c = a.to_fq();
  return fq29::from_fq(c.inverse_bgcd());
}

template <int MODE>
__device__ __forceinline__ fq29 inv_of(const fq29& a) {
  return MODE == 0 ? inv_fermat(a) : inv_bgcd(a);
}

__device__ __forceinline__ fq29 load29(const uint32_t* p) {
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) w[k] = p[k];
  w[7] &= 0x0fffffffu;
  return fq29::unpack(w);
}

// inversion throughput; writes a * a^-1 (must be the Montgomery one) for the host check
template <int MODE>
__global__ void __launch_bounds__(256) k_inv(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fq29 a = load29(io + 16 * tid);
  fq29 x = a;
  for (int it = 0; it < iters; it++) {
    x = inv_of<MODE>(x);
    x.l[0] ^= 1;  // next input (keeps the chain live; still a field element)
  }
  const fq29 chk = fq29::mul(a, inv_of<MODE>(a));
  fq r = chk.to_fq();
  r.store(io + 16 * tid);
  fq29 s = x.norm();
  io[16 * tid + 8] = s.l[0];
}

// K chains per thread, one batch of K affine adds per iteration sharing ONE inversion
template <int K, int MODE>
__global__ void __launch_bounds__(256) k_batch(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fq29 X[K], Y[K];
  const fq29 px = load29(io + 16 * tid), py = load29(io + 16 * tid + 8);
#pragma unroll
  for (int i = 0; i < K; i++) {
    X[i] = px;
    X[i].l[1] += i + 1;
    Y[i] = py;
  }
  for (int it = 0; it < iters; it++) {
    fq29 pref[K];
    fq29 acc = fq29::from(f29::ONE);
#pragma unroll
    for (int i = 0; i < K; i++) {
      fq29 x2 = px;
      x2.l[0] += it + 3 * i;
      const fq29 d = fq29::sub<64, 1>(x2, X[i]).norm();
      pref[i] = acc;
      acc = fq29::mul(acc, d);
    }
    fq29 inv = inv_of<MODE>(acc);
#pragma unroll
    for (int i = K - 1; i >= 0; i--) {
      fq29 x2 = px, y2 = py;
      x2.l[0] += it + 3 * i;
      y2.l[2] += it;
      const fq29 d = fq29::sub<64, 1>(x2, X[i]).norm();
      const fq29 inv_i = fq29::mul(inv, pref[i]);
      inv = fq29::mul(inv, d);
      const fq29 lam = fq29::mul(fq29::sub<64, 1>(y2, Y[i]).norm(), inv_i);
      const fq29 x3 = fq29::sub<128, 2>(fq29::sqr(lam), fq29::add(X[i], x2)).norm();
      Y[i] = fq29::sub<64, 1>(fq29::mul(lam, fq29::sub<64, 1>(X[i], x3).norm()), Y[i]).norm();
      X[i] = x3;
    }
  }
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < K; i++) o ^= X[i].l[0] ^ Y[i].l[3];
  io[16 * tid] = o;
}

// Round 6 (VERDICT r5 Next #4): the CROSS-LANE wave batch. K chains per lane whose pending state
// (accumulator X, Y and the forward prefix products) lives in LDS; per step ONE inversion per wave:
// each lane's K-chain product t_l, an inclusive and an exclusive-suffix product scan of t_l over the
// 64 lanes (shuffles, 6 levels each), the wave total inverted once, 1/t_l = inv * prefix_excl *
// suffix_excl, then each lane's backward pass and affine adds. Fq products per entry:
//   forward 1 + backward 2 + affine add 3 (lambda, lambda^2, lambda * (x1 - x3)) = 6 per entry,
//   + (12 scan + 2 + inversion) per lane per step = (14 + INV) / K per entry,
// INV = 253 squarings + 120 multiplies (q - 2 has 121 set bits) = 373 products by the whole wave.
__device__ __forceinline__ fq29 shfl_fq29(const fq29& a, int src_lane) {
  fq29 r;
#pragma unroll
  for (int j = 0; j < 9; j++) r.l[j] = __shfl(a.l[j], src_lane);
  return r;
}

template <int K>
__global__ void __launch_bounds__(64) k_xlane(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x, lane = threadIdx.x;
  __shared__ fq29 sX[K][64], sY[K][64], sP[K][64];
  const fq29 px = load29(io + 16 * tid), py = load29(io + 16 * tid + 8);
#pragma unroll
  for (int i = 0; i < K; i++) {
    fq29 x = px;
    x.l[1] += i + 1;
    sX[i][lane] = x;
    sY[i][lane] = py;
  }
  const fq29 one = fq29::from(f29::ONE);
  for (int it = 0; it < iters; it++) {
    fq29 acc = one;
    for (int i = 0; i < K; i++) {  // forward: prefix products of this lane's K differences
      fq29 x2 = px;
      x2.l[0] += it + 3 * i;
      const fq29 d = fq29::sub<64, 1>(x2, sX[i][lane]).norm();
      sP[i][lane] = acc;
      acc = fq29::mul(acc, d);
    }
    // inclusive prefix and exclusive suffix products of the lane totals over the wave
    fq29 pre = acc, suf = one;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const fq29 y = shfl_fq29(pre, lane >= off ? lane - off : lane);
      if (lane >= off) pre = fq29::mul(pre, y);
    }
    fq29 sacc = acc;  // inclusive suffix
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const fq29 y = shfl_fq29(sacc, lane + off < 64 ? lane + off : lane);
      if (lane + off < 64) sacc = fq29::mul(sacc, y);
    }
    const fq29 pre_ex = lane ? shfl_fq29(pre, lane - 1) : one;
    const fq29 pre_excl = lane ? pre_ex : one;
    suf = shfl_fq29(sacc, lane < 63 ? lane + 1 : lane);
    if (lane == 63) suf = one;
    const fq29 total = shfl_fq29(pre, 63);
    fq29 inv = inv_fermat(total);                                  // one inversion per wave
    inv = fq29::mul(fq29::mul(inv, pre_excl), suf);                // 1 / (this lane's K-product)
    for (int i = K - 1; i >= 0; i--) {  // backward pass + affine adds
      fq29 x2 = px, y2 = py;
      x2.l[0] += it + 3 * i;
      y2.l[2] += it;
      const fq29 X = sX[i][lane], Y = sY[i][lane];
      const fq29 d = fq29::sub<64, 1>(x2, X).norm();
      const fq29 inv_i = fq29::mul(inv, sP[i][lane]);
      inv = fq29::mul(inv, d);
      const fq29 lam = fq29::mul(fq29::sub<64, 1>(y2, Y).norm(), inv_i);
      const fq29 x3 = fq29::sub<128, 2>(fq29::sqr(lam), fq29::add(X, x2)).norm();
      sY[i][lane] = fq29::sub<64, 1>(fq29::mul(lam, fq29::sub<64, 1>(X, x3).norm()), Y).norm();
      sX[i][lane] = x3;
    }
  }
  uint32_t o = 0;
  for (int i = 0; i < K; i++) o ^= sX[i][lane].l[0] ^ sY[i][lane].l[3];
  io[16 * tid] = o;
}

// production XYZZ mixed add in the same harness (as madd29.hip)
__global__ void __launch_bounds__(256) k_xyzz(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t xw[8], yw[8];
  for (int k = 0; k < 8; k++) {
    xw[k] = io[16 * tid + k];
    yw[k] = io[16 * tid + 8 + k];
  }
  xw[7] &= 0x0fffffff;
  yw[7] &= 0x0fffffff;
  g1_acc29 acc;
  acc.set_inf();
  for (int it = 0; it < iters; it++) {
    xw[0] += it;
    acc.add_aff(xw, yw, it & 1);
  }
  acc.to_xyzz().store(io + 32 * tid);
}

int main() {
  const int blocks = 256 * 8;
  const size_t words = (size_t)blocks * 256 * 32;
  std::vector<uint32_t> h(words);
  uint64_t s = 0x243f6a8885a308d3ull;
  for (auto& w : h) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    w = (uint32_t)(s >> 32);
  }
  uint32_t* d;
  CHECK(hipMalloc(&d, words * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  auto timed = [&](auto launch, double units, const char* what, const char* unit) -> int {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      if (hipMemcpy(d, h.data(), words * 4, hipMemcpyHostToDevice) != hipSuccess) return 1;
      if (hipEventRecord(e0) != hipSuccess) return 1;
      launch();
      if (hipEventRecord(e1) != hipSuccess || hipEventSynchronize(e1) != hipSuccess) return 1;
      if (hipEventElapsedTime(&ms, e0, e1) != hipSuccess) return 1;
    }
    printf("%-34s %8.3f ms  %8.3f G %s/s\n", what, ms, units / ms / 1e6, unit);
    return 0;
  };
  const double threads = (double)blocks * 256;
  // inversions (fewer threads: the binary Euclid is long)
  const int ib = 256 * 2, iit = 4;
  if (timed([&] { hipLaunchKernelGGL(k_inv<0>, dim3(ib), dim3(256), 0, 0, d, iit); }, (double)ib * 256 * (iit + 1),
            "fq29 Fermat inversion", "inv")) return 1;
  {
    std::vector<uint32_t> o((size_t)ib * 256 * 16);
    CHECK(hipMemcpy(o.data(), d, o.size() * 4, hipMemcpyDeviceToHost));
    // Montgomery one (2^256 mod q) words
    const uint32_t one[8] = {0xc58f0d9du, 0xd35d438du, 0xf5c70b3du, 0x0a78eb28u,
                             0x7879462cu, 0x666ea36fu, 0x9a07df2fu, 0x0e0a77c1u};
    int bad = 0;
    for (int t = 0; t < ib * 256; t++)
      for (int k = 0; k < 8; k++) bad += o[16 * (size_t)t + k] != one[k];
    printf("fq29 Fermat inversion check: %s\n", bad ? "BAD" : "a * a^-1 == 1 for every lane");
  }
  if (timed([&] { hipLaunchKernelGGL(k_inv<1>, dim3(ib), dim3(256), 0, 0, d, iit); }, (double)ib * 256 * (iit + 1),
            "binary Euclid inversion (64 lanes)", "inv")) return 1;
  const int iters = 16;
  if (timed([&] { hipLaunchKernelGGL(k_xyzz, dim3(blocks), dim3(256), 0, 0, d, 4 * iters); }, threads * 4 * iters,
            "XYZZ mixed add (production)", "adds")) return 1;
#define BA(KK, MM, name)                                                                                      \
  if (timed([&] { hipLaunchKernelGGL((k_batch<KK, MM>), dim3(blocks), dim3(256), 0, 0, d, iters); },           \
            threads * KK * iters, name, "adds")) return 1;
  BA(2, 0, "batch-affine K=2, Fermat")
  BA(4, 0, "batch-affine K=4, Fermat")
  BA(8, 0, "batch-affine K=8, Fermat")
#define XL(KK, name)                                                                                          \
  if (timed([&] { hipLaunchKernelGGL((k_xlane<KK>), dim3(blocks * 4), dim3(64), 0, 0, d, iters); },            \
            threads * KK * iters, name, "adds")) return 1;
  XL(8, "cross-lane wave batch K=8, Fermat")
  XL(16, "cross-lane wave batch K=16, Fermat")
  // K = 32 does not compile: 3 x 32 x 64 x 36 B = 221 KB of pending state exceeds the CU's 160 KB LDS
  BA(2, 1, "batch-affine K=2, binary Euclid")
  BA(4, 1, "batch-affine K=4, binary Euclid")
  BA(8, 1, "batch-affine K=8, binary Euclid")
  return 0;
}
