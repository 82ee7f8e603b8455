// Microbenchmark: v_mad_u64_u32 issue cost when the mads form C independent accumulator chains per
// wave and W waves share a SIMD (W blocks of 256 threads per CU). The field products compile to
// product-scanning columns, i.e. ONE serial accumulator chain at a time: this measures what that
// costs at the 2-3 waves per SIMD the bucket accumulation runs at.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

template <int C>
__global__ void __launch_bounds__(256) k_chain(uint64_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = tid * 2654435761u, b = tid ^ 0x9e3779b9u;
  uint64_t u[C];
#pragma unroll
  for (int k = 0; k < C; k++) u[k] = tid + k;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 64 / C; r++) {
#pragma unroll
      for (int k = 0; k < C; k++) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(u[k]) : "v"(a), "v"(b) : "s40", "s41");
    }
  }
  uint64_t r = 0;
#pragma unroll
  for (int k = 0; k < C; k++) r ^= u[k];
  io[tid] = r;
}

template <int C>
int run(int cus, double clk, uint64_t* d, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 2048;
  for (int W = 1; W <= 4; W++) {
    const int blocks = cus * W;
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_chain<C>, dim3(blocks), dim3(256), 0, 0, d, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    // per SIMD: W waves x iters x 64 mads
    const double cyc = ms * 1e-3 * clk / ((double)W * iters * 64);
    printf("chains %d  waves/SIMD %d  %.3f ms  %.2f SIMD-cycles per mad (nominal clock)\n", C, W, ms, cyc);
  }
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %.0f MHz\n", prop.gcnArchName, cus, clk / 1e6);
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)cus * 4 * 256 * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  run<1>(cus, clk, d, e0, e1);
  run<2>(cus, clk, d, e0, e1);
  run<4>(cus, clk, d, e0, e1);
  run<8>(cus, clk, d, e0, e1);
  return 0;
}
