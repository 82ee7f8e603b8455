// Microbenchmark: the production fq29 XYZZ mixed add (field29.hpp, register-resident operands) at a
// fixed number of waves per SIMD (W blocks of 256 threads per CU, __launch_bounds__(256, W)), with
// one accumulator per thread (NACC = 1, production add_aff) or two independent accumulators whose
// adds share one basic block (NACC = 2, the rare-case branch hoisted out): does the add issue faster
// when the scheduler has two independent product chains to interleave?
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../kzg-grandsums-study_amd/csrc/field29.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

// add_aff's common path (no infinity / P == 0 handling): acc += (x2, y2)
__device__ __forceinline__ void add_common(g1_acc29& a, const fq29& x2, const fq29& y2) {
  const fq29 P = fq29::carry_sub<30, 1>(fq29::mul_cols(x2, a.ZZ), a.X);
  const fq29 S2 = fq29::mul(y2, a.ZZZ);
  fq29 R = fq29::neg<32, 2>(a.Y);
#pragma unroll
  for (int j = 0; j < 9; j++) R.l[j] = R.l[j] + S2.l[j];
  R = R.norm();
  const fq29 PP = fq29::sqr(P);
  const fq29 PPP = fq29::mul(P, PP);
  a.ZZ = fq29::mul(a.ZZ, PP);
  const fq29 Qv = fq29::mul(a.X, PP);
  a.ZZZ = fq29::mul(a.ZZZ, PPP);
  a.X = fq29::sub<16, 3>(fq29::sqr(R), fq29::add(PPP, fq29::add(Qv, Qv))).norm();
  const fq29 T = fq29::sub<64, 1>(Qv, a.X);
  a.Y = fq29::mul2(R, T, a.Y, fq29::neg<3, 1>(PPP));
}

template <int W, int NACC>
__global__ void __launch_bounds__(256, W) k_add(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t xw[8], yw[8];
  for (int k = 0; k < 8; k++) {
    xw[k] = io[16 * tid + k];
    yw[k] = io[16 * tid + 8 + k];
  }
  xw[7] &= 0x0fffffff;
  yw[7] &= 0x0fffffff;
  if (NACC == 1) {
    g1_acc29 acc;
    acc.set_inf();
    for (int it = 0; it < iters; it++) {
      xw[0] += it;
      acc.add_aff(xw, yw, it & 1);
    }
    acc.to_xyzz().store(io + 32 * tid);
  } else {
    g1_acc29 a0, a1;
    const fq29 x2 = fq29::unpack(xw), y2 = fq29::unpack(yw);
    a0.X = x2; a0.Y = y2; a0.ZZ = fq29::from(f29::ONE); a0.ZZZ = a0.ZZ; a0.inf = false;
    a1 = a0;
    a1.X.l[0] ^= 1;
    for (int it = 0; it < iters; it++) {
      fq29 xa = x2, xb = x2;
      xa.l[0] += it;
      xb.l[1] += it;
      add_common(a0, xa, y2);
      add_common(a1, xb, y2);
    }
    a0.add(a1);
    a0.to_xyzz().store(io + 32 * tid);
  }
}

template <int W, int NACC>
int run(int cus, uint32_t* d, hipEvent_t e0, hipEvent_t e1) {
  const int blocks = cus * W, iters = 256;
  float ms = 0;
  for (int rep = 0; rep < 3; rep++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL((k_add<W, NACC>), dim3(blocks), dim3(256), 0, 0, d, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    CHECK(hipEventElapsedTime(&ms, e0, e1));
  }
  const double adds = (double)blocks * 256 * iters * NACC;
  printf("waves/SIMD %d  accumulators/thread %d: %.3f ms  %.2f G adds/s\n", W, NACC, ms, adds / ms / 1e6);
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)cus * 4 * 256 * 128));
  CHECK(hipMemset(d, 0x5a, (size_t)cus * 4 * 256 * 128));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  run<1, 1>(cus, d, e0, e1);
  run<2, 1>(cus, d, e0, e1);
  run<3, 1>(cus, d, e0, e1);
  run<1, 2>(cus, d, e0, e1);
  run<2, 2>(cus, d, e0, e1);
  return 0;
}
