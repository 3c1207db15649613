// Latency of one dependent FM-index step on gfx950 (seeding's bwt_extend
// chain): a lane walks LF steps k' = C[c] + occ_c(k) through a random
// 64-position-block occurrence table of seq_len positions (the device layout
// of seed.hip), so every step waits for the previous one's fetch.
//   mode 0: the fetch only (k' from the fetched words, no counting)
//   mode 1: block_counts64 for all four bases (seed.hip's occ4), pick c
//   mode 2: one base's count (eq-popcounts for c only)
//   mode 3: mode 1 with both ends of an interval (two fetches, occ4x2)
// usage: ext_chain <waves total> <steps> [seq_len]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                           \
  do {                                                                  \
    hipError_t e_ = (x);                                                \
    if (e_ != hipSuccess) {                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                          \
    }                                                                   \
  } while (0)

__device__ __forceinline__ void counts4(uint64_t k, uint4 hdr, uint4 w4, uint64_t cnt[4]) {
  const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
  const int nfull = (int)((k & 63) >> 4);
  const uint32_t tail = ~((1u << ((~(uint32_t)k & 15) << 1)) - 1);
  uint32_t c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = (i < nfull ? 0xffffffffu : i == nfull ? tail : 0u) & 0x55555555u;
    const uint32_t x1 = w[i] ^ 0x55555555u, x2 = w[i] ^ 0xaaaaaaaau, x3 = ~w[i];
    c1 += __popc(~(x1 | x1 >> 1) & m);
    c2 += __popc(~(x2 | x2 >> 1) & m);
    c3 += __popc(~(x3 | x3 >> 1) & m);
  }
  const uint32_t c0 = (uint32_t)(k & 63) + 1 - c1 - c2 - c3;
  cnt[0] = hdr.x + c0;
  cnt[1] = hdr.y + c1;
  cnt[2] = hdr.z + c2;
  cnt[3] = hdr.w + c3;
}

__device__ __forceinline__ uint32_t count1(uint64_t k, uint4 w4, int c) {
  const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
  const int nfull = (int)((k & 63) >> 4);
  const uint32_t tail = ~((1u << ((~(uint32_t)k & 15) << 1)) - 1);
  const uint32_t pat = (uint32_t)c * 0x55555555u;
  uint32_t n = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = (i < nfull ? 0xffffffffu : i == nfull ? tail : 0u) & 0x55555555u;
    const uint32_t x = w[i] ^ pat;
    n += __popc(~(x | x >> 1) & m);
  }
  return n;
}

template <int MODE>
__global__ void __launch_bounds__(256) walk(const uint4* __restrict__ occ, uint64_t n, int steps, uint64_t* out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t k = (t * 0x9E3779B97F4A7C15ull) % n, l = (k + 37) % n;
  uint64_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    const int c = (int)((k ^ (k >> 7) ^ s) & 3);
    const uint4* p = occ + 2 * (k >> 6);
    const uint4 h = p[0], w = p[1];
    uint64_t nk;
    if (MODE == 0) {
      nk = (uint64_t)(h.x ^ w.y) * 64 + (k & 63);
    } else if (MODE == 1) {
      uint64_t cnt[4];
      counts4(k, h, w, cnt);
      nk = c == 0 ? cnt[0] : c == 1 ? cnt[1] : c == 2 ? cnt[2] : cnt[3];
      nk = nk * 4 + c;
    } else if (MODE == 2) {
      const uint32_t hc = c == 0 ? h.x : c == 1 ? h.y : c == 2 ? h.z : h.w;
      nk = ((uint64_t)hc + count1(k, w, c)) * 4 + c;
    } else {
      const uint4* q = occ + 2 * (l >> 6);
      uint4 h2 = h, w2 = w;
      if ((k >> 6) != (l >> 6)) {
        h2 = q[0];
        w2 = q[1];
      }
      uint64_t ck[4], cl[4];
      counts4(k, h, w, ck);
      counts4(l, h2, w2, cl);
      const uint64_t a = c == 0 ? ck[0] : c == 1 ? ck[1] : c == 2 ? ck[2] : ck[3];
      const uint64_t b = c == 0 ? cl[0] : c == 1 ? cl[1] : c == 2 ? cl[2] : cl[3];
      nk = a * 4 + c;
      l = (nk + (b - a) + 1) % n;
    }
    acc += nk;
    k = nk % n;
  }
  out[t] = acc + k;
}

int main(int argc, char** argv) {
  const int waves = argc > 1 ? atoi(argv[1]) : 1;
  const int steps = argc > 2 ? atoi(argv[2]) : 1000;
  const uint64_t n = argc > 3 ? strtoull(argv[3], 0, 10) : 46709983ull;
  const uint64_t nb = (n + 63) / 64;
  std::vector<uint4> h(2 * nb);
  uint32_t cnt[4] = {0, 0, 0, 0};
  uint64_t st = 88172645463325252ull;
  for (uint64_t b = 0; b < nb; ++b) {
    h[2 * b] = make_uint4(cnt[0], cnt[1], cnt[2], cnt[3]);
    uint32_t w[4];
    for (int i = 0; i < 4; ++i) {
      st ^= st << 13, st ^= st >> 7, st ^= st << 17;
      w[i] = (uint32_t)st;
      for (int j = 0; j < 16; ++j) ++cnt[(w[i] >> (2 * j)) & 3];
    }
    h[2 * b + 1] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  uint4* d;
  uint64_t* o;
  CK(hipMalloc(&d, h.size() * sizeof(uint4)));
  CK(hipMalloc(&o, (size_t)waves * 64 * 8));
  CK(hipMemcpy(d, h.data(), h.size() * sizeof(uint4), hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int threads = waves >= 4 ? 256 : 64 * waves;
  const int blocks = (waves * 64 + threads - 1) / threads;
  for (int mode = 0; mode < 4; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (mode == 0) hipLaunchKernelGGL(walk<0>, dim3(blocks), dim3(threads), 0, 0, d, n, steps, o);
      if (mode == 1) hipLaunchKernelGGL(walk<1>, dim3(blocks), dim3(threads), 0, 0, d, n, steps, o);
      if (mode == 2) hipLaunchKernelGGL(walk<2>, dim3(blocks), dim3(threads), 0, 0, d, n, steps, o);
      if (mode == 3) hipLaunchKernelGGL(walk<3>, dim3(blocks), dim3(threads), 0, 0, d, n, steps, o);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep)
        printf("waves %6d mode %d: %.3f ms, %.1f ns per step, %.2f G lane-steps/s\n", waves, mode, ms,
               ms * 1e6 / steps, (double)waves * 64 * steps / ms / 1e6);
    }
  }
  return 0;
}
