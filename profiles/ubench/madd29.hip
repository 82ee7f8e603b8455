// Microbenchmark: XYZZ mixed-add throughput, fq29 accumulator vs the 8x32-bit lazy accumulator
// (register-resident operands, no memory traffic).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include "../../kzg-grandsums-study_amd/csrc/field29.hpp"
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)
using namespace kgs;

template <int V>
__global__ void __launch_bounds__(256) k_add(uint32_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t xw[8], yw[8];
  for (int k = 0; k < 8; k++) {
    xw[k] = io[16 * tid + k];
    yw[k] = io[16 * tid + 8 + k];
  }
  xw[7] &= 0x0fffffff;
  yw[7] &= 0x0fffffff;
  if (V == 1) {
    g1_acc29 acc;
    acc.set_inf();
    for (int it = 0; it < iters; it++) {
      xw[0] += it;
      acc.add_aff(xw, yw, it & 1);
    }
    acc.to_xyzz().store(io + 32 * tid);
  } else {
    g1_xyzz acc = g1_xyzz::inf();
    for (int it = 0; it < iters; it++) {
      xw[0] += it;
      g1_aff p;
      for (int k = 0; k < 8; k++) {
        p.x.v[k] = xw[k];
        p.y.v[k] = yw[k];
      }
      if (it & 1) p.y = p.y.neg();
      acc.add_aff_lazy(p);
    }
    acc.canon();
    acc.store(io + 32 * tid);
  }
}

int main() {
  const int blocks = 256 * 8, iters = 64;
  uint32_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 256 * 128));
  CHECK(hipMemset(d, 0x5a, (size_t)blocks * 256 * 128));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int v = 0; v < 2; v++) {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipEventRecord(e0));
      if (v == 0) hipLaunchKernelGGL(k_add<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
      else hipLaunchKernelGGL(k_add<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    const double adds = (double)blocks * 256 * iters;
    printf("%s: %.3f ms  %.2f G adds/s\n", v ? "fq29 acc" : "8x32 lazy", ms, adds / ms / 1e6);
  }
  return 0;
}
