// Microbenchmark: does the (dead) carry-out SGPR pair of v_mad_u64_u32 serialise a wave's mads?
// 8 independent accumulator chains per wave, 1 or 2 waves per SIMD; every mad writes the same SGPR
// pair (what the compiler emits), or the mads rotate over 2 / 4 / 8 pairs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

#define MAD(U, S) asm volatile("v_mad_u64_u32 %0, " S ", %1, %2, %0" : "+v"(U) : "v"(a), "v"(b) : "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "s48", "s49", "s50", "s51", "s52", "s53", "s54", "s55");
template <int NS>
__global__ void __launch_bounds__(256) k_sd(uint64_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t a = tid * 2654435761u, b = tid ^ 0x9e3779b9u;
  uint64_t u0 = tid, u1 = tid + 1, u2 = tid + 2, u3 = tid + 3, u4 = tid + 4, u5 = tid + 5, u6 = tid + 6, u7 = tid + 7;
  for (int i = 0; i < iters; i++) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      if (NS == 1) {
        MAD(u0, "s[40:41]") MAD(u1, "s[40:41]") MAD(u2, "s[40:41]") MAD(u3, "s[40:41]")
        MAD(u4, "s[40:41]") MAD(u5, "s[40:41]") MAD(u6, "s[40:41]") MAD(u7, "s[40:41]")
      } else if (NS == 2) {
        MAD(u0, "s[40:41]") MAD(u1, "s[42:43]") MAD(u2, "s[40:41]") MAD(u3, "s[42:43]")
        MAD(u4, "s[40:41]") MAD(u5, "s[42:43]") MAD(u6, "s[40:41]") MAD(u7, "s[42:43]")
      } else if (NS == 4) {
        MAD(u0, "s[40:41]") MAD(u1, "s[42:43]") MAD(u2, "s[44:45]") MAD(u3, "s[46:47]")
        MAD(u4, "s[40:41]") MAD(u5, "s[42:43]") MAD(u6, "s[44:45]") MAD(u7, "s[46:47]")
      } else {
        MAD(u0, "s[40:41]") MAD(u1, "s[42:43]") MAD(u2, "s[44:45]") MAD(u3, "s[46:47]")
        MAD(u4, "s[48:49]") MAD(u5, "s[50:51]") MAD(u6, "s[52:53]") MAD(u7, "s[54:55]")
      }
    }
  }
  io[tid] = u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7;
}

template <int NS>
int run(int cus, double clk, uint64_t* d, hipEvent_t e0, hipEvent_t e1) {
  const int iters = 2048;
  for (int W = 1; W <= 2; W++) {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      CHECK(hipEventRecord(e0));
      hipLaunchKernelGGL(k_sd<NS>, dim3(cus * W), dim3(256), 0, 0, d, iters);
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      CHECK(hipEventElapsedTime(&ms, e0, e1));
    }
    printf("sdst pairs %d  waves/SIMD %d  %.3f ms  %.2f SIMD-cycles per mad (nominal clock)\n", NS, W, ms,
           ms * 1e-3 * clk / ((double)W * iters * 64));
  }
  return 0;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;
  const int cus = prop.multiProcessorCount;
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)cus * 2 * 256 * 8));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  run<1>(cus, clk, d, e0, e1);
  run<2>(cus, clk, d, e0, e1);
  run<4>(cus, clk, d, e0, e1);
  run<8>(cus, clk, d, e0, e1);
  return 0;
}
