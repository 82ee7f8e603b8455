// Host-side cost of enqueuing pinned host -> device copies, the way kgs_prove feeds F_0 (2 MiB
// pieces on the context's stream) and the other vectors (8 MiB pieces on a low-priority copy
// stream): wall time of the hipMemcpyAsync calls alone, then of the copies' completion.
// build: hipcc --offload-arch=gfx950 -O2 h2d_enqueue.hip -o h2d_enqueue
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e = (x);                                                                \
    if (e != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

int main() {
  const size_t E = (size_t)32 << 20;
  void *h, *d;
  CK(hipHostMalloc(&h, E, hipHostMallocDefault));
  CK(hipMalloc(&d, E));
  for (size_t i = 0; i < E; i += 4096) ((char*)h)[i] = 1;
  hipStream_t st_norm, st_low;
  CK(hipStreamCreateWithFlags(&st_norm, hipStreamNonBlocking));
  int lo = 0, hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
  CK(hipStreamCreateWithPriority(&st_low, hipStreamNonBlocking, lo));
  struct Case {
    const char* name;
    hipStream_t st;
    size_t piece;
  } cases[] = {{"normal stream, 2 MiB pieces", st_norm, 2u << 20}, {"normal stream, 8 MiB pieces", st_norm, 8u << 20},
               {"normal stream, 32 MiB", st_norm, 32u << 20},       {"low-priority, 2 MiB pieces", st_low, 2u << 20},
               {"low-priority, 8 MiB pieces", st_low, 8u << 20},    {"low-priority, 32 MiB", st_low, 32u << 20}};
  for (int rep = 0; rep < 3; rep++) {
    for (const auto& c : cases) {
      CK(hipDeviceSynchronize());
      const auto t0 = clk::now();
      int calls = 0;
      for (size_t o = 0; o < E; o += c.piece, calls++)
        CK(hipMemcpyAsync((char*)d + o, (char*)h + o, c.piece, hipMemcpyHostToDevice, c.st));
      const auto t1 = clk::now();
      CK(hipStreamSynchronize(c.st));
      const auto t2 = clk::now();
      printf("rep %d %-30s %2d calls: enqueue %.3f ms (%.1f us per call), done after %.3f ms (%.1f GB/s)\n", rep, c.name,
             calls, ms(t0, t1), 1e3 * ms(t0, t1) / calls, ms(t0, t2), E / ms(t0, t2) / 1e6);
    }
  }
  return 0;
}
