// Microbenchmark: the fq29 XYZZ mixed add with product-scanning Montgomery products (FIPS: the
// reduction interleaved column by column, the carry of each column the addend of the next, limbs
// leaving normalised) against the production CIOS products + carry pass (field29.hpp).
// Register-resident operands, no memory traffic; the two accumulators must agree bit for bit.
// Result (profiles/ubench/madd29_fips_r02.txt): 16.6 vs 14.6 G adds/s here, bit-identical — but at
// this launch bound the CIOS kernel spills (168 VGPRs + 236 B scratch) while the FIPS one fits in
// 127 VGPRs at 4 waves/SIMD. Ported into field29.hpp, the production k_accumulate compiled to the
// same column schedule and instruction mix from both source forms (the compiler already turns the
// CIOS rows into product scanning) and measured neutral (profiles/r02/ab_fips_vs_cios.txt); at a
// 4-wave register bound the production loop spills and runs 37 % slower. Not adopted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../kzg-grandsums-study_amd/csrc/field29.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

namespace fips {
using f29::MASK;
using f29::INV;
// column k < 9: m_k from the column's low bits, add m_k q_0, carry out
#define KGS_FIPS_LOW(k)                                               \
  m[k] = ((uint32_t)acc * INV) & MASK;                                \
  acc = (uint64_t)m[k] * f29::Q.v[0] + acc;                           \
  acc >>= 29;

__device__ __forceinline__ fq29 mul(const fq29& a, const fq29& b) {
  uint32_t m[9];
  fq29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc = (uint64_t)a.l[i] * b.l[k - i] + acc;
#pragma unroll
    for (int i = 0; i < k; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    KGS_FIPS_LOW(k)
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)a.l[i] * b.l[k - i] + acc;
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    r.l[k - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// a*b + c*d, one reduction
__device__ __forceinline__ fq29 mul2(const fq29& a, const fq29& b, const fq29& c, const fq29& d) {
  uint32_t m[9];
  fq29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc = (uint64_t)a.l[i] * b.l[k - i] + acc;
#pragma unroll
    for (int i = 0; i <= k; i++) acc = (uint64_t)c.l[i] * d.l[k - i] + acc;
#pragma unroll
    for (int i = 0; i < k; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    KGS_FIPS_LOW(k)
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)a.l[i] * b.l[k - i] + acc;
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)c.l[i] * d.l[k - i] + acc;
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    r.l[k - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

__device__ __forceinline__ fq29 sqr(const fq29& a) {
  uint32_t m[9], d[9];
#pragma unroll
  for (int j = 0; j < 9; j++) d[j] = a.l[j] << 1;
  fq29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; 2 * i < k; i++) acc = (uint64_t)d[i] * a.l[k - i] + acc;
    if ((k & 1) == 0) acc = (uint64_t)a.l[k / 2] * a.l[k / 2] + acc;
#pragma unroll
    for (int i = 0; i < k; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    KGS_FIPS_LOW(k)
  }
#pragma unroll
  for (int k = 9; k < 17; k++) {
#pragma unroll
    for (int i = k - 8; 2 * i < k; i++) acc = (uint64_t)d[i] * a.l[k - i] + acc;
    if ((k & 1) == 0) acc = (uint64_t)a.l[k / 2] * a.l[k / 2] + acc;
#pragma unroll
    for (int i = k - 8; i < 9; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    r.l[k - 9] = (uint32_t)acc & MASK;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// mul(a, b) + K - c, the difference folded into the scan (K = spread(k, s))
template <uint32_t K, uint32_t S>
__device__ __forceinline__ fq29 mul_sub(const fq29& a, const fq29& b, const fq29& c) {
  constexpr f29::L9 Kc = f29::spread(K, S);
  uint32_t m[9];
  fq29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; k++) {
#pragma unroll
    for (int i = 0; i <= k; i++) acc = (uint64_t)a.l[i] * b.l[k - i] + acc;
#pragma unroll
    for (int i = 0; i < k; i++) acc = (uint64_t)m[i] * f29::Q.v[k - i] + acc;
    KGS_FIPS_LOW(k)
  }
  int64_t sacc = (int64_t)acc;
#pragma unroll
  for (int k = 9; k < 17; k++) {
    sacc += (int64_t)(Kc.v[k - 9] - c.l[k - 9]);
#pragma unroll
    for (int i = k - 8; i < 9; i++) sacc = (int64_t)((uint64_t)a.l[i] * b.l[k - i] + (uint64_t)sacc);
#pragma unroll
    for (int i = k - 8; i < 9; i++) sacc = (int64_t)((uint64_t)m[i] * f29::Q.v[k - i] + (uint64_t)sacc);
    r.l[k - 9] = (uint32_t)sacc & MASK;
    sacc >>= 29;
  }
  r.l[8] = (uint32_t)(sacc + (int64_t)(Kc.v[8] - c.l[8]));
  return r;
}
#undef KGS_FIPS_LOW

struct acc {
  fq29 X, Y, ZZ, ZZZ;
  bool inf;
  // same formula, operand order and special cases as g1_acc29::add_aff (the doubling / opposite
  // cases are not reached by the benchmark's inputs and are left to the production path)
  __device__ __forceinline__ void add_aff(const uint32_t* xw, const uint32_t* yw, bool negy) {
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
    const fq29 P = mul_sub<30, 1>(x2, ZZ, X);
    const fq29 S2 = mul(y2, ZZZ);
    fq29 R = fq29::neg<32, 2>(Y);
#pragma unroll
    for (int j = 0; j < 9; j++) R.l[j] = negy ? R.l[j] - S2.l[j] : R.l[j] + S2.l[j];
    R = R.norm();
    const fq29 PP = sqr(P);
    const fq29 PPP = mul(P, PP);
    ZZ = mul(ZZ, PP);
    const fq29 Qv = mul(X, PP);
    ZZZ = mul(ZZZ, PPP);
    X = fq29::sub<16, 3>(sqr(R), fq29::add(PPP, fq29::add(Qv, Qv))).norm();
    const fq29 T = fq29::sub<64, 1>(Qv, X);
    Y = mul2(R, T, Y, fq29::neg<3, 1>(PPP));
  }
};
}  // namespace fips

template <int V>
__global__ void __launch_bounds__(256, 3) k_add(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t xw[8], yw[8];
  for (int k = 0; k < 8; k++) {
    xw[k] = io[16 * tid + k];
    yw[k] = io[16 * tid + 8 + k];
  }
  xw[7] &= 0x0fffffff;
  yw[7] &= 0x0fffffff;
  uint32_t out[36];
  if (V == 0) {
    g1_acc29 a;
    a.set_inf();
    for (int it = 0; it < iters; it++) {
      xw[0] += it;
      a.add_aff(xw, yw, it & 1);
    }
    for (int j = 0; j < 9; j++) {
      out[j] = a.X.l[j];
      out[9 + j] = a.Y.l[j];
      out[18 + j] = a.ZZ.l[j];
      out[27 + j] = a.ZZZ.l[j];
    }
  } else {
    fips::acc a;
    a.inf = true;
    for (int it = 0; it < iters; it++) {
      xw[0] += it;
      a.add_aff(xw, yw, it & 1);
    }
    for (int j = 0; j < 9; j++) {
      out[j] = a.X.l[j];
      out[9 + j] = a.Y.l[j];
      out[18 + j] = a.ZZ.l[j];
      out[27 + j] = a.ZZZ.l[j];
    }
  }
  const size_t N = (size_t)gridDim.x * blockDim.x;
  uint32_t* o = io + 16 * N + V * 36 * N + 36 * (size_t)tid;
  for (int j = 0; j < 36; j++) o[j] = out[j];
}

int main() {
  const int blocks = 256 * 6, iters = 64, nthr = blocks * 256;
  uint32_t* d;
  const size_t words = (size_t)nthr * 16 + 2 * (size_t)nthr * 36 + 64;
  CHECK(hipMalloc(&d, words * 4));
  CHECK(hipMemset(d, 0x5a, words * 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const char* names[] = {"CIOS + carry pass (production)", "FIPS product scanning"};
  for (int v = 0; v < 2; v++) {
    float best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
      float ms = 0;
      CHECK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_add<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
      else hipLaunchKernelGGL(k_add<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double adds = (double)nthr * iters;
    printf("%-32s %.3f ms  %.2f G adds/s\n", names[v], best, adds / best / 1e6);
  }
  uint32_t* h = (uint32_t*)malloc(2 * (size_t)nthr * 36 * 4);
  CHECK(hipMemcpy(h, d + (size_t)nthr * 16 + 0, 2 * (size_t)nthr * 36 * 4, hipMemcpyDeviceToHost));
  // outputs: V = 0 at io + 16 N, V = 1 at io + 52 N (36 words per lane each)
  size_t bad = 0;
  for (size_t t = 0; t < (size_t)nthr; t++)
    for (int j = 0; j < 36; j++) bad += h[t * 36 + j] != h[(size_t)nthr * 36 + t * 36 + j];
  printf("accumulators compared: %d lanes, %zu differing words\n", nthr, bad);
  return 0;
}
