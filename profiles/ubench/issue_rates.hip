// Microbenchmark: issue cost (SIMD cycles per wave64 instruction) of candidate bignum instructions on gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

#define R8(X) X X X X X X X X
template <int OP>
__global__ void __launch_bounds__(256) k_op(uint64_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  double d0 = tid * 1.0, d1 = d0 + 1, d2 = d0 + 2, d3 = d0 + 3, d4 = d0 + 4, d5 = d0 + 5, d6 = d0 + 6, d7 = d0 + 7;
  double ma = 1.0000001, mb = 3.0e-9;
  uint64_t u0 = tid, u1 = tid + 1, u2 = tid + 2, u3 = tid + 3, u4 = tid + 4, u5 = tid + 5, u6 = tid + 6, u7 = tid + 7;
  uint32_t a = tid * 2654435761u, b = tid ^ 0x9e3779b9u;
  uint32_t w0 = tid, w1 = tid + 1, w2 = tid + 2, w3 = tid + 3, w4 = tid + 4, w5 = tid + 5, w6 = tid + 6, w7 = tid + 7;
  for (int i = 0; i < iters; i++) {
    if (OP == 0) {  // v_fma_f64
#define F(D) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(D) : "v"(ma), "v"(mb));
      R8(F(d0) F(d1) F(d2) F(d3) F(d4) F(d5) F(d6) F(d7))
    } else if (OP == 1) {  // v_mad_u64_u32
#define M(U) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %0" : "+v"(U) : "v"(a), "v"(b) : "vcc");
      R8(M(u0) M(u1) M(u2) M(u3) M(u4) M(u5) M(u6) M(u7))
    } else if (OP == 2) {  // v_lshl_add_u64
#define L(U) asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(U) : "v"(u7));
      R8(L(u0) L(u1) L(u2) L(u3) L(u4) L(u5) L(u6) L(u0))
    } else if (OP == 3) {  // v_add_co_u32
#define A(W) asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(W) : "v"(a) : "vcc");
      R8(A(w0) A(w1) A(w2) A(w3) A(w4) A(w5) A(w6) A(w7))
    } else if (OP == 4) {  // v_add_u32 (no carry)
#define A2(W) asm volatile("v_add_u32 %0, %0, %1" : "+v"(W) : "v"(a));
      R8(A2(w0) A2(w1) A2(w2) A2(w3) A2(w4) A2(w5) A2(w6) A2(w7))
    } else if (OP == 5) {  // v_mul_hi_u32
#define H(W) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(W) : "v"(a));
      R8(H(w0) H(w1) H(w2) H(w3) H(w4) H(w5) H(w6) H(w7))
    } else if (OP == 6) {  // v_mad_u32_u24
#define U24(W) asm volatile("v_mad_u32_u24 %0, %1, %2, %0" : "+v"(W) : "v"(a), "v"(b));
      R8(U24(w0) U24(w1) U24(w2) U24(w3) U24(w4) U24(w5) U24(w6) U24(w7))
    } else if (OP == 7) {  // v_mul_f64
#define FM(D) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(D) : "v"(ma));
      R8(FM(d0) FM(d1) FM(d2) FM(d3) FM(d4) FM(d5) FM(d6) FM(d7))
    } else if (OP == 8) {  // v_add_f64
#define FA(D) asm volatile("v_add_f64 %0, %0, %1" : "+v"(D) : "v"(mb));
      R8(FA(d0) FA(d1) FA(d2) FA(d3) FA(d4) FA(d5) FA(d6) FA(d7))
    } else if (OP == 9) {  // v_pk_fma_f32 (packed, for reference)
#define PF(D) asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(D) : "v"(ma), "v"(mb));
      R8(PF(d0) PF(d1) PF(d2) PF(d3) PF(d4) PF(d5) PF(d6) PF(d7))
    } else if (OP == 10) {  // v_addc_co_u32
#define AC(W) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(W) : "v"(a) : "vcc");
      R8(AC(w0) AC(w1) AC(w2) AC(w3) AC(w4) AC(w5) AC(w6) AC(w7))
    } else if (OP == 11) {  // v_cvt_f64_u32
#define CV(D, W) asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(D) : "v"(W));
      R8(CV(d0, w0) CV(d1, w1) CV(d2, w2) CV(d3, w3) CV(d4, w4) CV(d5, w5) CV(d6, w6) CV(d7, w7))
    } else if (OP == 12) {  // v_mul_lo_u32
#define ML(W) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(W) : "v"(a));
      R8(ML(w0) ML(w1) ML(w2) ML(w3) ML(w4) ML(w5) ML(w6) ML(w7))
    } else if (OP == 13) {  // v_mul_hi_u32_u24
#define MH24(W) asm volatile("v_mul_hi_u32_u24 %0, %0, %1" : "+v"(W) : "v"(a));
      R8(MH24(w0) MH24(w1) MH24(w2) MH24(w3) MH24(w4) MH24(w5) MH24(w6) MH24(w7))
    }
  }
  uint64_t r = u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7 ^ w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^ w6 ^ w7;
  double s = d0 + d1 + d2 + d3 + d4 + d5 + d6 + d7;
  io[tid] = r ^ __double_as_longlong(s);
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %.0f MHz\n", prop.gcnArchName, cus, clk / 1e6);
  const int blocks = cus * 8, threads = 256, iters = 4096;
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * threads * 8));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_fma_f64", "v_mad_u64_u32", "v_lshl_add_u64", "v_add_co_u32", "v_add_u32", "v_mul_hi_u32",
                         "v_mad_u32_u24", "v_mul_f64", "v_add_f64", "v_pk_fma_f32", "v_addc_co_u32", "v_cvt_f64_u32",
                         "v_mul_lo_u32", "v_mul_hi_u32_u24"};
  void (*ks[])(uint64_t*, int) = {k_op<0>, k_op<1>, k_op<2>, k_op<3>, k_op<4>, k_op<5>, k_op<6>,
                                  k_op<7>, k_op<8>, k_op<9>, k_op<10>, k_op<11>, k_op<12>, k_op<13>};
  for (int op = 0; op < 14; op++) {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[op], dim3(blocks), dim3(threads), 0, 0, d, iters);
      hipEventRecord(e1);
      CHECK(hipEventSynchronize(e1));
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double waves = (double)blocks * threads / 64;
    const double instrs = waves * iters * 64;  // 64 asm instrs per iteration
    const double cyc = ms * 1e-3 * clk * cus * 4 / instrs;
    printf("%-18s %.3f ms  %.2f SIMD-cycles per wave64 instr\n", names[op], ms, cyc);
  }
  return 0;
}
