// Cost of seed.hip's own extend1 in a dependent chain (a random occurrence
// table in the device layout, one superblock): the floor of a tier-1 step.
// usage: ext_real <waves total> <steps>
#include "../../bwa-flow_amd/csrc/seed.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

namespace bwagpu {
namespace {
__global__ void __launch_bounds__(256) chain(DevBwt b, int steps, uint64_t* out) {
  const uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  uint64_t st = t * 0x9E3779B97F4A7C15ull + 1;
  Ivl ik = set_intv(b, (int)(st & 3));
  uint64_t acc = 0;
  for (int s = 0; s < steps; ++s) {
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    const int c = (int)(st & 3);
    Ivl o = extend1(b, ik, c, 1);
    if (o.x[2] == 0) o = set_intv(b, c);
    acc += o.x[2];
    ik = o;
  }
  out[t] = acc + ik.x[0];
}
}  // namespace
}  // namespace bwagpu

int main(int argc, char** argv) {
  using namespace bwagpu;
  const int waves = argc > 1 ? atoi(argv[1]) : 1;
  const int steps = argc > 2 ? atoi(argv[2]) : 1000;
  const uint64_t n = 46709983ull;
  const uint64_t nb = (n + 63) / 64 + 1;
  std::vector<uint4> h(2 * nb);
  uint64_t cnt[4] = {0, 0, 0, 0};
  uint64_t s = 88172645463325252ull;
  for (uint64_t b = 0; b < nb; ++b) {
    h[2 * b] = make_uint4((uint32_t)cnt[0], (uint32_t)cnt[1], (uint32_t)cnt[2], (uint32_t)cnt[3]);
    uint32_t w[4];
    for (int i = 0; i < 4; ++i) {
      s ^= s << 13, s ^= s >> 7, s ^= s << 17;
      w[i] = (uint32_t)s;
      for (int j = 0; j < 16; ++j) ++cnt[(w[i] >> (2 * j)) & 3];
    }
    h[2 * b + 1] = make_uint4(w[0], w[1], w[2], w[3]);
  }
  DevBwt b{};
  b.seq_len = n;
  b.primary = n / 3;
  b.L2[0] = 0;
  for (int c = 0; c < 4; ++c) b.L2[c + 1] = b.L2[c] + n / 4;
  uint4* d;
  uint64_t *sup, *o;
  hipMalloc(&d, h.size() * sizeof(uint4));
  hipMalloc(&sup, 64);
  hipMemset(sup, 0, 64);
  hipMalloc(&o, (size_t)waves * 64 * 8);
  hipMemcpy(d, h.data(), h.size() * sizeof(uint4), hipMemcpyHostToDevice);
  b.occ = d;
  b.sup = sup;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int threads = waves >= 4 ? 256 : 64 * waves;
  const int blocks = (waves * 64 + threads - 1) / threads;
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(chain, dim3(blocks), dim3(threads), 0, 0, b, steps, o);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    if (rep) printf("waves %6d extend1 chain: %.3f ms, %.1f ns per step\n", waves, ms, ms * 1e6 / steps);
  }
  return 0;
}
