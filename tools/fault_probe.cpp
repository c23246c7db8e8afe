#include <sys/mman.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>
#include <cstdlib>
using clk = std::chrono::steady_clock;
int main() {
  const size_t N = 32u << 20;
  std::vector<char> src(N, 7);
  for (int mode = 0; mode < 4; mode++)
  for (int T : {1, 2, 4, 8}) {
    double best = 1e9;
    for (int rep = 0; rep < 5; rep++) {
      char* p = (char*)mmap(nullptr, N, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (mode == 2 || mode == 3) madvise(p, N, MADV_HUGEPAGE);
      auto t0 = clk::now();
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++) th.emplace_back([&, t] {
        size_t lo = N * t / T, hi = N * (t + 1) / T;
        if (mode == 0 || mode == 2) memcpy(p + lo, src.data() + lo, hi - lo);
        else { madvise(p + (lo & ~4095ul), hi - (lo & ~4095ul), 23 /*MADV_POPULATE_WRITE*/); memcpy(p + lo, src.data() + lo, hi - lo); }
      });
      for (auto& x : th) x.join();
      double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
      if (ms < best) best = ms;
      munmap(p, N);
    }
    printf("mode %d (%s) T=%d: %.3f ms  %.1f GB/s\n", mode, mode==0?"memcpy":mode==1?"populate+memcpy":mode==2?"hugepage memcpy":"hugepage populate+memcpy", T, best, N / best / 1e6);
  }
  // warm
  char* p = (char*)malloc(N); memset(p, 1, N);
  auto t0 = clk::now(); memcpy(p, src.data(), N);
  printf("warm 1T: %.3f ms\n", std::chrono::duration<double, std::milli>(clk::now() - t0).count());
  FILE* f = fopen("/sys/kernel/mm/transparent_hugepage/enabled", "r"); char b[256] = {}; if (f) { if (fread(b, 1, 255, f)) {}; printf("thp: %s", b); }
}
