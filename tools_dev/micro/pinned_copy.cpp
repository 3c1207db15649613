// Host memcpy rate into pinned (hipHostMalloc, several flag sets) vs pageable
// memory, on 1/4/8/16 threads, and the H2D rate out of each: what bounds the
// staging copy of bwagpu_chain2aln_submit (~20 MB per C2 record).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double copy_rate(char* dst, const char* src, size_t n, int nt, int reps) {
  auto part = [&](int t) {
    const size_t lo = n * t / nt, hi = n * (t + 1) / nt;
    memcpy(dst + lo, src + lo, hi - lo);
  };
  double best = 1e30;
  for (int r = 0; r < reps; ++r) {
    auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 1; t < nt; ++t) th.emplace_back(part, t);
    part(0);
    for (auto& x : th) x.join();
    double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (s < best) best = s;
  }
  return n / best / 1e9;
}

int main() {
  const size_t n = 20u << 20;
  char* src = (char*)malloc(n);
  memset(src, 1, n);
  char* dev = nullptr;
  if (hipMalloc(&dev, n) != hipSuccess) return 1;
  struct Kind {
    const char* name;
    unsigned flags;
    int pinned;
  } kinds[] = {{"pageable", 0, 0},
               {"hipHostMallocDefault", hipHostMallocDefault, 1},
               {"hipHostMallocNonCoherent", hipHostMallocNonCoherent, 1},
               {"hipHostMallocCoherent", hipHostMallocCoherent, 1},
               {"hipHostMallocWriteCombined", hipHostMallocWriteCombined, 1},
               {"hipHostRegister(malloc)", 0, 2}};
  hipStream_t st;
  (void)hipStreamCreate(&st);
  for (const Kind& k : kinds) {
    char* dst = nullptr;
    if (k.pinned == 1) {
      if (hipHostMalloc((void**)&dst, n, k.flags) != hipSuccess) { printf("%s: alloc failed\n", k.name); continue; }
    } else {
      dst = (char*)aligned_alloc(4096, n);
      memset(dst, 0, n);
      if (k.pinned == 2 && hipHostRegister(dst, n, hipHostRegisterDefault) != hipSuccess) { printf("register failed\n"); continue; }
    }
    printf("%-28s memcpy GB/s:", k.name);
    for (int nt : {1, 4, 8, 16}) printf(" %d thr %.1f", nt, copy_rate(dst, src, n, nt, 5));
    double best = 1e30;
    for (int r = 0; r < 5; ++r) {
      auto t0 = std::chrono::steady_clock::now();
      (void)hipMemcpyAsync(dev, dst, n, hipMemcpyHostToDevice, st);
      (void)hipStreamSynchronize(st);
      double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      if (s < best) best = s;
    }
    printf(" | H2D %.1f GB/s\n", n / best / 1e9);
    if (k.pinned == 1) (void)hipHostFree(dst);
    else {
      if (k.pinned == 2) (void)hipHostUnregister(dst);
      free(dst);
    }
  }
  return 0;
}
