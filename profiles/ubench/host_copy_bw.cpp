// Host copy bandwidth of the boundary's staging copy (VERDICT r5 Next #5): one 32 MiB vector (an
// n = 2^20 Fr evaluation buffer) copied from a pageable, already-touched source into
//   pinned  - hipHostMalloc'd staging (what kgs_prove copies into, context.hpp io_in)
//   pinwc   - hipHostMalloc write-combined staging
//   page    - an ordinary touched pageable buffer (the upper bound of the host itself)
// with 1..16 threads, plain memcpy and 16 B non-temporal stores. Best of 9 per cell (ms, GB/s).
// Build: hipcc -O3 -std=c++17 host_copy_bw.cpp -o host_copy_bw -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <algorithm>
#include <chrono>
#include <thread>
#include <vector>

static void copy_nt(uint8_t* d, const uint8_t* s, size_t n) {
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    __m128i a = _mm_loadu_si128((const __m128i*)(s + i)), b = _mm_loadu_si128((const __m128i*)(s + i + 16));
    __m128i c = _mm_loadu_si128((const __m128i*)(s + i + 32)), e = _mm_loadu_si128((const __m128i*)(s + i + 48));
    _mm_stream_si128((__m128i*)(d + i), a);
    _mm_stream_si128((__m128i*)(d + i + 16), b);
    _mm_stream_si128((__m128i*)(d + i + 32), c);
    _mm_stream_si128((__m128i*)(d + i + 48), e);
  }
  memcpy(d + i, s + i, n - i);
  _mm_sfence();
}

static double run(uint8_t* dst, const uint8_t* src, size_t bytes, int nth, bool nt) {
  double best = 1e30;
  for (int rep = 0; rep < 9; rep++) {
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    const size_t piece = (bytes / nth + 4095) & ~(size_t)4095;
    for (int t = 0; t < nth; t++) {
      const size_t o = (size_t)t * piece;
      if (o >= bytes) break;
      const size_t len = std::min(piece, bytes - o);
      th.emplace_back([=] {
        if (nt) copy_nt(dst + o, src + o, len);
        else memcpy(dst + o, src + o, len);
      });
    }
    for (auto& x : th) x.join();
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    best = std::min(best, ms);
  }
  return best;
}

int main() {
  const size_t bytes = (size_t)32 << 20;
  cpu_set_t cs;
  sched_getaffinity(0, sizeof(cs), &cs);
  printf("cpus in affinity mask: %d, hardware_concurrency %u\n", CPU_COUNT(&cs), std::thread::hardware_concurrency());
  uint8_t* src = (uint8_t*)aligned_alloc(4096, bytes);
  uint8_t* page = (uint8_t*)aligned_alloc(4096, bytes);
  memset(src, 1, bytes);
  memset(page, 2, bytes);
  uint8_t *pin = nullptr, *pinwc = nullptr;
  if (hipHostMalloc((void**)&pin, bytes, hipHostMallocDefault) != hipSuccess) return 1;
  if (hipHostMalloc((void**)&pinwc, bytes, hipHostMallocWriteCombined) != hipSuccess) return 1;
  memset(pin, 3, bytes);
  memset(pinwc, 4, bytes);
  struct D {
    const char* name;
    uint8_t* p;
  } dsts[] = {{"page", page}, {"pinned", pin}, {"pinwc", pinwc}};
  printf("%-7s %-6s %s\n", "dst", "store", "threads: ms (GB/s) for 32 MiB, best of 9");
  for (const D& d : dsts)
    for (int nt = 0; nt < 2; nt++) {
      printf("%-7s %-6s", d.name, nt ? "nt" : "memcpy");
      for (int th : {1, 2, 4, 8, 12, 16}) {
        const double ms = run(d.p, src, bytes, th, nt);
        printf(" %2d: %.3f (%.1f)", th, ms, bytes / ms / 1e6);
      }
      printf("\n");
      fflush(stdout);
    }
  hipHostFree(pin);
  hipHostFree(pinwc);
  return 0;
}
