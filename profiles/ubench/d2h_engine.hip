// Which engine carries a 32 MiB device -> host copy, per kind of host destination, and how fast:
// hipMemcpyAsync D2H on a non-blocking stream into hipHostMalloc (default / non-coherent / write-
// combined / numa-user), into malloc'd memory registered with hipHostRegister, and the same through
// hipMemcpyDtoHAsync; H2D for comparison. Run under rocprofv3 --kernel-trace --memory-copy-trace:
// a copy done by a blit kernel shows as __amd_rocclr_copyBuffer, an SDMA copy as MEMORY_COPY_*.
// Also a zero-copy kernel that stores straight into mapped pinned memory (k_store_host).
// build: hipcc --offload-arch=gfx950 -O2 d2h_engine.hip -o d2h_engine
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__global__ void k_store_host(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n16) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(src[i], &dst[i]);
}

int main() {
  const size_t E = (size_t)32 << 20;
  const int reps = 8;
  void* dev;
  CK(hipMalloc(&dev, E));
  CK(hipMemset(dev, 1, E));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b, evx;
  hipStream_t st2;
  CK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
  CK(hipEventCreateWithFlags(&evx, hipEventDisableTiming));
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Dst {
    const char* name;
    void* p;
  } dsts[6];
  int nd = 0;
  void* p;
  CK(hipHostMalloc(&p, E, hipHostMallocDefault));
  dsts[nd++] = {"hipHostMalloc(default)", p};
  CK(hipHostMalloc(&p, E, hipHostMallocNonCoherent));
  dsts[nd++] = {"hipHostMalloc(non-coherent)", p};
  CK(hipHostMalloc(&p, E, hipHostMallocWriteCombined));
  dsts[nd++] = {"hipHostMalloc(write-combined)", p};
  CK(hipHostMalloc(&p, E, hipHostMallocNumaUser));
  dsts[nd++] = {"hipHostMalloc(numa-user)", p};
  p = aligned_alloc(4096, E);
  memset(p, 0, E);
  CK(hipHostRegister(p, E, hipHostRegisterDefault));
  dsts[nd++] = {"malloc + hipHostRegister", p};
  for (int d = 0; d < nd; d++) {
    for (int mode = 0; mode < 6; mode++) {
      // 0: hipMemcpyAsync D2H, 1: hipMemcpyDtoHAsync, 2: H2D, 3: zero-copy store kernel
      CK(hipStreamSynchronize(st));
      CK(hipEventRecord(a, st));
      for (int r = 0; r < reps; r++) {
        if (mode == 0) CK(hipMemcpyAsync(dsts[d].p, dev, E, hipMemcpyDeviceToHost, st));
        if (mode == 1) CK(hipMemcpyDtoHAsync(dsts[d].p, (hipDeviceptr_t)dev, E, st));
        if (mode == 2) CK(hipMemcpyAsync(dev, dsts[d].p, E, hipMemcpyHostToDevice, st));
        if (mode == 4 || mode == 5) {
          // D2H ordered after work on another stream through an event (as the prover's write-back on
          // its own stream after the conversion kernel); mode 5 also puts a kernel before it there
          if (mode == 5) k_store_host<<<1, 64, 0, st2>>>((u32x4*)dev, (const u32x4*)dev, 1024);
          CK(hipEventRecord(evx, st2));
          CK(hipStreamWaitEvent(st, evx, 0));
          CK(hipMemcpyAsync(dsts[d].p, dev, E, hipMemcpyDeviceToHost, st));
        }
        if (mode == 3) {
          void* dp = nullptr;
          if (hipHostGetDevicePointer(&dp, dsts[d].p, 0) != hipSuccess) {
            (void)hipGetLastError();
            dp = dsts[d].p;  // unified addressing: the host pointer itself
          }
          k_store_host<<<256, 256, 0, st>>>((u32x4*)dp, (const u32x4*)dev, E / 16);
        }
      }
      CK(hipEventRecord(b, st));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      static const char* mn[] = {"hipMemcpyAsync D2H", "hipMemcpyDtoHAsync", "hipMemcpyAsync H2D", "store kernel D2H",
                                 "D2H after event wait", "D2H after kernel+event"};
      printf("%-32s %-20s %7.3f ms per 32 MiB  %6.1f GB/s\n", dsts[d].name, mn[mode], ms / reps, E / (ms / reps * 1e-3) / 1e9);
    }
  }
  return 0;
}
