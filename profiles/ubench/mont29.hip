// Microbenchmark: BN254 Fq Montgomery product in 9 x 29-bit limbs with 64-bit column accumulators
// (R = 2^261, no carry words) versus the production 8 x 32-bit product-scanning product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include "../../kzg-grandsums-study_amd/csrc/field.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

constexpr uint32_t M29 = 0x1fffffffu;
constexpr uint32_t Q29[9] = {0x187cfd47u, 0x10460b6u, 0x1c72a34fu, 0x2d522d0u, 0x1585d978u,
                             0x2db40c0u, 0xa6e141u, 0xe5c2634u, 0x30644eu};
constexpr uint32_t INV29 = 0x4866389u;

struct F29 { uint32_t l[9]; };

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

// a: limbs < 2^29; b: limbs < 2^31; values < 2^259 -> result < 2^258, limbs < 2^29
__device__ __forceinline__ F29 mul29(const F29& a, const F29& b) {
  uint64_t t[9];
#pragma unroll
  for (int j = 0; j < 9; j++) t[j] = 0;
#pragma unroll
  for (int i = 0; i < 9; i++) {
#pragma unroll
    for (int j = 0; j < 9; j++) t[j] = mad64(a.l[i], b.l[j], t[j]);
    const uint32_t m = ((uint32_t)t[0] * INV29) & M29;
    const uint64_t c = mad64(m, Q29[0], t[0]) >> 29;
#pragma unroll
    for (int j = 1; j < 9; j++) t[j] = mad64(m, Q29[j], t[j]);
#pragma unroll
    for (int j = 0; j < 8; j++) t[j] = t[j + 1];
    t[0] += c;
    t[8] = 0;
  }
  F29 r;
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const uint64_t s = t[j] + c;
    r.l[j] = (uint32_t)s & M29;
    c = s >> 29;
  }
  return r;
}

__device__ __forceinline__ F29 to29(const fq& a) {
  F29 r;
#pragma unroll
  for (int j = 0; j < 9; j++) {
    const int bit = 29 * j, w = bit >> 5, s = bit & 31;
    uint32_t lo = a.v[w] >> s;
    if (s > 3 && w + 1 < 8) lo |= a.v[w + 1] << (32 - s);
    r.l[j] = lo & M29;
  }
  return r;
}

__global__ void k_check(uint32_t* out, const uint32_t* in, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fq a = fq::load(in + 16 * i), b = fq::load(in + 16 * i + 8);
  fq c = a * b;
  F29 c29 = mul29(to29(a), to29(b));
  for (int j = 0; j < 8; j++) out[17 * i + j] = c.v[j];
  for (int j = 0; j < 9; j++) out[17 * i + 8 + j] = c29.l[j];
}

template <int V>
__global__ void __launch_bounds__(256) k_thr(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  fq a = fq::load(io + 16 * tid), b = fq::load(io + 16 * tid + 8);
  if (V == 0) {
    for (int it = 0; it < iters; it++) {
      fq c = a * b;
      b = c * a;
      a = c;
    }
    a.store(io + 16 * tid);
    b.store(io + 16 * tid + 8);
  } else {
    F29 x = to29(a), y = to29(b);
    for (int it = 0; it < iters; it++) {
      F29 z = mul29(x, y);
      y = mul29(z, x);
      x = z;
    }
    for (int j = 0; j < 9; j++) io[16 * tid + j] = x.l[j] ^ y.l[j];
  }
}

int main() {
  const int n = 4096;
  std::vector<uint32_t> h(16 * n);
  uint64_t s = 0x12345678abcdefull;
  for (auto& x : h) { s = s * 6364136223846793005ull + 1442695040888963407ull; x = (uint32_t)(s >> 33); }
  for (int i = 0; i < 2 * n; i++) h[8 * i + 7] &= 0x0fffffffu;  // < 2^252 < q
  uint32_t *din, *dout;
  CHECK(hipMalloc(&din, h.size() * 4));
  CHECK(hipMalloc(&dout, (size_t)17 * n * 4));
  CHECK(hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_check, dim3(n / 256), dim3(256), 0, 0, dout, din, n);
  std::vector<uint32_t> o(17 * n);
  CHECK(hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost));
  FILE* f = fopen("gpurun_out/mont29_check.bin", "wb");
  fwrite(h.data(), 4, h.size(), f);
  fwrite(o.data(), 4, o.size(), f);
  fclose(f);

  const int blocks = 256 * 8, iters = 256;
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 256 * 64));
  std::vector<uint32_t> hh((size_t)blocks * 256 * 16);
  for (auto& x : hh) { s = s * 6364136223846793005ull + 1442695040888963407ull; x = (uint32_t)(s >> 33); }
  for (size_t i = 0; i < hh.size() / 8; i++) hh[8 * i + 7] &= 0x0fffffffu;
  CHECK(hipMemcpy(d, hh.data(), hh.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int v = 0; v < 2; v++) {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_thr<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
      else hipLaunchKernelGGL(k_thr<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double mults = (double)blocks * 256 * iters * 2;
    printf("%s: %.3f ms  %.1f G products/s\n", v ? "9x29 (R=2^261)" : "8x32 production", ms, mults / ms / 1e6);
  }
  return 0;
}
