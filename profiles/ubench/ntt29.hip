// Microbenchmark: one radix-8 NTT round (3 stages, 12 butterflies, every twiddle nontrivial) in
// registers: the production 8 x 32-bit canonical Fr arithmetic (field.hpp: modular add / sub with a
// conditional correction, Montgomery product + reduce_once) against BN254 Fr in 9 x 29-bit limbs
// with lazy, carry-free additions (values grow inside the round, one carry pass per element at its
// end; differences a + K - b with K a spread multiple of r). DIF and DIT forms. Timing only (random
// operands; the two variants use different Montgomery radices).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include "../../kzg-grandsums-study_amd/csrc/field.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

namespace r29 {
constexpr uint32_t MASK = 0x1fffffffu;
constexpr uint32_t INV = 0x0fffffffu;  // -r^-1 mod 2^29
constexpr uint32_t Q[9] = {0x10000001u, 0x1f0fac9fu, 0x0e5c2450u, 0x07d090f3u, 0x1585d283u,
                           0x02db40c0u, 0x00a6e141u, 0x0e5c2634u, 0x0030644eu};
struct L9 { uint32_t v[9]; };
constexpr L9 spread(uint32_t k, uint32_t s) {
  L9 r{};
  uint64_t carry = 0;
  for (int j = 0; j < 9; j++) {
    const uint64_t t = (uint64_t)Q[j] * k + carry;
    r.v[j] = j < 8 ? (uint32_t)(t & MASK) : (uint32_t)t;
    carry = t >> 29;
  }
  r.v[0] += s << 29;
  for (int j = 1; j < 8; j++) r.v[j] += (s << 29) - s;
  r.v[8] -= s;
  return r;
}
struct e {
  uint32_t l[9];
  __device__ __forceinline__ static e unpack(const uint32_t* w) {
    e r;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const int bit = 29 * j, i = bit >> 5, s = bit & 31;
      uint32_t x = w[i] >> s;
      if (s > 3 && i + 1 < 8) x |= w[i + 1] << (32 - s);
      r.l[j] = x & MASK;
    }
    return r;
  }
  __device__ __forceinline__ e norm() const {
    e r;
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint32_t s = l[j] + c;
      r.l[j] = j < 8 ? (s & MASK) : s;
      c = s >> 29;
    }
    return r;
  }
  __device__ __forceinline__ friend e operator+(const e& a, const e& b) {
    e r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = a.l[j] + b.l[j];
    return r;
  }
  template <uint32_t K, uint32_t S>
  __device__ __forceinline__ static e sub(const e& a, const e& b) {
    constexpr L9 Kc = spread(K, S);
    e r;
#pragma unroll
    for (int j = 0; j < 9; j++) r.l[j] = (a.l[j] + Kc.v[j]) - b.l[j];
    return r;
  }
  // a * b * 2^-261 (CIOS rows, 64-bit columns, final carry pass): < a*b/2^261 + r, normalised
  __device__ __forceinline__ static e mul(const e& a, const e& b) {
    uint64_t t[9];
#pragma unroll
    for (int j = 0; j < 9; j++) t[j] = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
#pragma unroll
      for (int j = 0; j < 9; j++) t[j] = (uint64_t)a.l[i] * b.l[j] + t[j];
      const uint32_t m = ((uint32_t)t[0] * INV) & MASK;
      const uint64_t c = ((uint64_t)m * Q[0] + t[0]) >> 29;
#pragma unroll
      for (int j = 1; j < 9; j++) t[j] = (uint64_t)m * Q[j] + t[j];
#pragma unroll
      for (int j = 0; j < 8; j++) t[j] = t[j + 1];
      t[0] += c;
      t[8] = 0;
    }
    e r;
    uint64_t c = 0;
#pragma unroll
    for (int j = 0; j < 9; j++) {
      const uint64_t s = t[j] + c;
      r.l[j] = (uint32_t)s & MASK;
      c = s >> 29;
    }
    return r;
  }
};
}  // namespace r29

// V = 0: production fr DIF round; 1: r29 lazy DIF round; 2: production DIT; 3: r29 lazy DIT
template <int V>
__global__ void __launch_bounds__(256) k_round(uint32_t* io, const uint32_t* tw, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (V == 0 || V == 2) {
    fr x[8], w[7];
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = fr::load(io + 8 * (8 * tid + r));
#pragma unroll
    for (int k = 0; k < 7; k++) w[k] = fr::load(tw + 8 * k);
    for (int it = 0; it < iters; it++) {
#pragma unroll
      for (int k = 0; k < 3; k++) {
        const int dist = V == 0 ? 4 >> k : 1 << k;
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const int r = ((q / dist) * 2 * dist) + (q % dist);
          const fr& ww = w[(k * 3 + q) % 7];
          fr a = x[r], b = x[r + dist];
          if (V == 2) {
            b = b * ww;
            x[r] = a + b;
            x[r + dist] = a - b;
          } else {
            x[r] = a + b;
            x[r + dist] = (a - b) * ww;
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < 8; r++) x[r].store(io + 8 * (8 * tid + r));
  } else {
    r29::e x[8], w[7];
#pragma unroll
    for (int r = 0; r < 8; r++) x[r] = r29::e::unpack(io + 8 * (8 * tid + r));
#pragma unroll
    for (int k = 0; k < 7; k++) w[k] = r29::e::unpack(tw + 8 * k);
    for (int it = 0; it < iters; it++) {
      if (V == 1) {
        // DIF: x path grows by 2x per stage; the difference a + K - b needs K's limbs >= b's
#pragma unroll
        for (int q = 0; q < 4; q++) {  // stage 0, dist 4: inputs normalised (< 2^29 limbs)
          const r29::e a = x[q], b = x[q + 4];
          x[q] = a + b;
          x[q + 4] = r29::e::mul(r29::e::sub<2, 1>(a, b), w[q % 7]);
        }
        // stage 1, dist 2: (0,2),(1,3) inputs <= 2^30 limbs; (4,6),(5,7) normalised
#pragma unroll
        for (int q = 0; q < 2; q++) {
          const r29::e a = x[q], b = x[q + 2];
          x[q] = a + b;
          x[q + 2] = r29::e::mul(r29::e::sub<4, 2>(a, b), w[(3 + q) % 7]);
          const r29::e c = x[q + 4], d = x[q + 6];
          x[q + 4] = c + d;
          x[q + 6] = r29::e::mul(r29::e::sub<2, 1>(c, d), w[(5 + q) % 7]);
        }
        // stage 2, dist 1: (0,1) inputs <= 2^31 limbs: normalise the pair first
        x[0] = x[0].norm();
        x[1] = x[1].norm();
#pragma unroll
        for (int q = 0; q < 4; q++) {
          const r29::e a = x[2 * q], b = x[2 * q + 1];
          x[2 * q] = a + b;
          x[2 * q + 1] = r29::e::mul(r29::e::sub<4, 2>(a, b), w[(6 + q) % 7]);
        }
      } else {
        // DIT: b*w normalised (< 2r); a grows by one 2^30-limb term per stage
#pragma unroll
        for (int k = 0; k < 3; k++) {
          const int dist = 1 << k;
#pragma unroll
          for (int q = 0; q < 4; q++) {
            const int r = ((q / dist) * 2 * dist) + (q % dist);
            const r29::e a = x[r];
            const r29::e bw = r29::e::mul(x[r + dist], w[(k * 3 + q) % 7]);
            x[r] = a + bw;
            x[r + dist] = r29::e::sub<2, 1>(a, bw);
          }
        }
      }
      // end of the round: every element back to normalised limbs
#pragma unroll
      for (int r = 0; r < 8; r++) x[r] = x[r].norm();
    }
    // out: raw limbs (value < 2^261), canonicalised on the host
#pragma unroll
    for (int r = 0; r < 8; r++)
#pragma unroll
      for (int j = 0; j < 8; j++) io[8 * (8 * tid + r) + j] = x[r].l[j] | (j == 7 ? (x[r].l[8] << 29) : 0u);
  }
}

int main() {
  const int blocks = 256 * 8, threads = 256, nthr = blocks * threads, iters = 32;
  const size_t words = (size_t)nthr * 64;
  uint32_t *d, *dw;
  CHECK(hipMalloc(&d, words * 4));
  CHECK(hipMalloc(&dw, 7 * 32));
  uint32_t tw[56];
  for (int i = 0; i < 56; i++) tw[i] = 0x9e3779b9u * (i + 1);
  for (int k = 0; k < 7; k++) tw[8 * k + 7] &= 0x0fffffff;
  CHECK(hipMemcpy(dw, tw, sizeof(tw), hipMemcpyHostToDevice));
  uint32_t* h = (uint32_t*)malloc(words * 4);
  for (size_t i = 0; i < words; i++) h[i] = (uint32_t)(i * 2654435761u) ^ 0x5bd1e995u;
  for (size_t i = 7; i < words; i += 8) h[i] &= 0x0fffffff;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"fr 8x32 canonical, DIF", "r29 lazy, DIF", "fr 8x32 canonical, DIT", "r29 lazy, DIT"};
  for (int v = 0; v < 4; v++) {
    float best = 1e9;
    for (int rep = 0; rep < 4; rep++) {
      CHECK(hipMemcpy(d, h, words * 4, hipMemcpyHostToDevice));
      float ms = 0;
      CHECK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_round<0>, dim3(blocks), dim3(threads), 0, 0, d, dw, iters);
      if (v == 1) hipLaunchKernelGGL(k_round<1>, dim3(blocks), dim3(threads), 0, 0, d, dw, iters);
      if (v == 2) hipLaunchKernelGGL(k_round<2>, dim3(blocks), dim3(threads), 0, 0, d, dw, iters);
      if (v == 3) hipLaunchKernelGGL(k_round<3>, dim3(blocks), dim3(threads), 0, 0, d, dw, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double bfly = (double)nthr * iters * 12;
    printf("%-26s %.3f ms  %.2f G butterflies/s\n", names[v], best, bfly / best / 1e6);
  }
  return 0;
}
