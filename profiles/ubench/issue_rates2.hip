// Microbenchmark: issue cost (real SIMD cycles per wave64 instruction, at the event-timed clock the
// driver reports) of the 32-bit helper instructions a 29-bit-limb carry pass can be built from, next
// to the 64-bit forms the compiler uses today (round 3: which ops issue at the doubled rate that
// v_add_u32 shows in issue_rates.hip).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CHECK(x) do{hipError_t e=(x); if(e!=hipSuccess){printf("HIP error %s at %d\n",hipGetErrorString(e),__LINE__); return 1;}}while(0)

#define R8(X) X X X X X X X X
#define BODY(INSN, ...)                                                                         \
  R8(asm volatile(INSN : "+v"(w0) : __VA_ARGS__); asm volatile(INSN : "+v"(w1) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(w2) : __VA_ARGS__); asm volatile(INSN : "+v"(w3) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(w4) : __VA_ARGS__); asm volatile(INSN : "+v"(w5) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(w6) : __VA_ARGS__); asm volatile(INSN : "+v"(w7) : __VA_ARGS__);)
#define BODY64(INSN, ...)                                                                       \
  R8(asm volatile(INSN : "+v"(u0) : __VA_ARGS__); asm volatile(INSN : "+v"(u1) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(u2) : __VA_ARGS__); asm volatile(INSN : "+v"(u3) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(u4) : __VA_ARGS__); asm volatile(INSN : "+v"(u5) : __VA_ARGS__);                 \
     asm volatile(INSN : "+v"(u6) : __VA_ARGS__); asm volatile(INSN : "+v"(u7) : __VA_ARGS__);)

template <int OP>
__global__ void __launch_bounds__(256) k_op(uint64_t* io, int iters) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t u0 = tid, u1 = tid + 1, u2 = tid + 2, u3 = tid + 3, u4 = tid + 4, u5 = tid + 5, u6 = tid + 6, u7 = tid + 7;
  uint32_t a = tid * 2654435761u, b = tid ^ 0x9e3779b9u;
  uint64_t a64 = ((uint64_t)b << 32) | a;
  uint32_t w0 = tid, w1 = tid + 1, w2 = tid + 2, w3 = tid + 3, w4 = tid + 4, w5 = tid + 5, w6 = tid + 6, w7 = tid + 7;
  for (int i = 0; i < iters; i++) {
    if (OP == 0) { BODY("v_add_u32 %0, %0, %1", "v"(a)) }
    else if (OP == 1) { BODY("v_and_b32 %0, %0, %1", "v"(a)) }
    else if (OP == 2) { BODY("v_or_b32 %0, %0, %1", "v"(a)) }
    else if (OP == 3) { BODY("v_lshrrev_b32 %0, 29, %0", "v"(a)) }
    else if (OP == 4) { BODY("v_lshrrev_b32 %0, %1, %0", "v"(a)) }
    else if (OP == 5) { BODY("v_alignbit_b32 %0, %1, %0, 29", "v"(a)) }
    else if (OP == 6) { BODY("v_bfe_u32 %0, %0, 3, 29", "v"(a)) }
    else if (OP == 7) { BODY("v_add3_u32 %0, %0, %1, %2", "v"(a), "v"(b)) }
    else if (OP == 8) { BODY("v_lshl_add_u32 %0, %1, 3, %0", "v"(a)) }
    else if (OP == 9) { BODY("v_sub_u32 %0, %0, %1", "v"(a)) }
    else if (OP == 10) { BODY("v_and_or_b32 %0, %0, %1, %2", "v"(a), "v"(b)) }
    else if (OP == 11) { BODY("v_cndmask_b32 %0, %0, %1, vcc", "v"(a)) }
    else if (OP == 12) { BODY("v_mul_u32_u24 %0, %0, %1", "v"(a)) }
    else if (OP == 13) { BODY("v_xor_b32 %0, %0, %1", "v"(a)) }
    else if (OP == 14) { BODY64("v_lshrrev_b64 %0, 29, %0", "v"(a)) }
    else if (OP == 15) { BODY64("v_lshl_add_u64 %0, %0, 0, %1", "v"(a64)) }
    else if (OP == 16) { BODY64("v_mad_u64_u32 %0, s[40:41], %1, %2, %0", "v"(a), "v"(b)) }
    else if (OP == 17) { BODY("v_mul_lo_u32 %0, %0, %1", "v"(a)) }
    else if (OP == 18) { BODY("v_lshl_or_b32 %0, %1, 3, %0", "v"(a)) }
    else if (OP == 19) { BODY("v_xad_u32 %0, %0, %1, %2", "v"(a), "v"(b)) }
    else if (OP == 20) { BODY("v_bfi_b32 %0, %1, %0, %2", "v"(a), "v"(b)) }
    else if (OP == 21) { BODY("v_mov_b32 %0, %1", "v"(a)) }
    else if (OP == 22) { BODY("v_add_lshl_u32 %0, %0, %1, 3", "v"(a)) }
    else if (OP == 23) { BODY("v_mad_u32_u16 %0, %0, %1, %2", "v"(a), "v"(b)) }
  }
  uint64_t r = u0 ^ u1 ^ u2 ^ u3 ^ u4 ^ u5 ^ u6 ^ u7 ^ w0 ^ w1 ^ w2 ^ w3 ^ w4 ^ w5 ^ w6 ^ w7;
  io[tid] = r;
}

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const double clk = prop.clockRate * 1e3;
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %.0f MHz (cycles below at this nominal clock)\n", prop.gcnArchName, cus, clk / 1e6);
  const int blocks = cus * 8, threads = 256, iters = 4096;
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * threads * 8));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const char* names[] = {"v_add_u32", "v_and_b32", "v_or_b32", "v_lshrrev_b32 imm", "v_lshrrev_b32 reg",
                         "v_alignbit_b32", "v_bfe_u32", "v_add3_u32", "v_lshl_add_u32", "v_sub_u32",
                         "v_and_or_b32", "v_cndmask_b32", "v_mul_u32_u24", "v_xor_b32", "v_lshrrev_b64",
                         "v_lshl_add_u64", "v_mad_u64_u32", "v_mul_lo_u32", "v_lshl_or_b32", "v_xad_u32",
                         "v_bfi_b32", "v_mov_b32", "v_add_lshl_u32", "v_mad_u32_u16"};
  void (*ks[])(uint64_t*, int) = {k_op<0>,  k_op<1>,  k_op<2>,  k_op<3>,  k_op<4>,  k_op<5>,  k_op<6>,  k_op<7>,
                                  k_op<8>,  k_op<9>,  k_op<10>, k_op<11>, k_op<12>, k_op<13>, k_op<14>, k_op<15>,
                                  k_op<16>, k_op<17>, k_op<18>, k_op<19>, k_op<20>, k_op<21>, k_op<22>, k_op<23>};
  for (int op = 0; op < 24; op++) {
    float ms = 0;
    for (int rep = 0; rep < 3; rep++) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(ks[op], dim3(blocks), dim3(threads), 0, 0, d, iters);
      hipEventRecord(e1);
      CHECK(hipEventSynchronize(e1));
      hipEventElapsedTime(&ms, e0, e1);
    }
    const double waves = (double)blocks * threads / 64;
    const double instrs = waves * iters * 64;
    const double cyc = ms * 1e-3 * clk * cus * 4 / instrs;
    printf("%-22s %.3f ms  %.2f SIMD-cycles per wave64 instr\n", names[op], ms, cyc);
  }
  return 0;
}
