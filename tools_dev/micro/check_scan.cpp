// How fast the host-side batch check of bwagpu_chain2aln_submit can run: the
// C2 batch's arrays (dumped by tools_dev/micro/check_scan.py into $1) walked
// read -> chain -> seed as check_batch_seeds does, on 1/2/4/8 threads, and the
// seeds alone as one flat pass.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

struct Seed {
  int64_t rbeg;
  int32_t qbeg, len, score, pad_;
};
template <class T>
std::vector<T> load(const std::string& f) {
  FILE* fp = fopen(f.c_str(), "rb");
  if (!fp) return {};
  fseek(fp, 0, SEEK_END);
  long n = ftell(fp);
  fseek(fp, 0, SEEK_SET);
  std::vector<T> v(n / sizeof(T));
  if (fread(v.data(), 1, n, fp) != (size_t)n) v.clear();
  fclose(fp);
  return v;
}
static double us_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
}
int main(int argc, char** argv) {
  const std::string d = argc > 1 ? argv[1] : "/tmp/ck";
  auto so = load<int64_t>(d + "/seq_off.bin");
  auto rco = load<int32_t>(d + "/read_chain_off.bin");
  auto cso = load<int32_t>(d + "/chain_seed_off.bin");
  auto sd = load<Seed>(d + "/seeds.bin");
  if (so.empty() || sd.empty()) return 1;
  const int nr = (int)so.size() - 1, nc = (int)cso.size() - 1, ns = (int)sd.size();
  const int64_t two = 2 * 46709983LL;
  const int64_t* S = so.data();
  const int32_t* R = rco.data();
  const int32_t* CS = cso.data();
  const Seed* SD = sd.data();
  auto check_range = [=](int r0, int r1) -> int {
    bool bad = false;
    for (int r = r0; r < r1; ++r) {
      const int64_t l = S[r + 1] - S[r];
      const int c0 = R[r], c1 = R[r + 1];
      if (l < 0 || c0 < 0 || c1 < c0 || c1 > nc) return 3;
      for (int c = c0; c < c1; ++c) {
        const int k0 = CS[c], k1 = CS[c + 1];
        if (k0 < 0 || k1 < k0 || k1 > ns) return 4;
        for (int k = k0; k < k1; ++k) {
          const Seed& s = SD[k];
          bad |= (s.qbeg < 0) | (s.len <= 0) | ((int64_t)s.qbeg + s.len > l) | (s.rbeg < 0) | (s.rbeg + s.len > two);
        }
      }
    }
    return bad ? 5 : 0;
  };
  for (int nt : {1, 2, 4, 8}) {
    double best = 1e30;
    for (int rep = 0; rep < 5; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      std::vector<int> code(nt);
      std::vector<std::thread> th;
      for (int t = 1; t < nt; ++t) th.emplace_back([&, t] { code[t] = check_range((int64_t)nr * t / nt, (int64_t)nr * (t + 1) / nt); });
      code[0] = check_range(0, nr / nt);
      for (auto& x : th) x.join();
      best = std::min(best, us_since(t0));
    }
    printf("read-chain-seed walk, %d threads: %.0f us\n", nt, best);
  }
  double best = 1e30;
  for (int rep = 0; rep < 5; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    bool bad = false;
    for (int k = 0; k < ns; ++k) bad |= (SD[k].qbeg < 0) | (SD[k].len <= 0) | (SD[k].rbeg < 0) | (SD[k].rbeg + SD[k].len > two);
    best = std::min(best, us_since(t0));
    if (bad) printf("bad\n");
  }
  printf("flat seed pass, 1 thread: %.0f us (%d reads %d chains %d seeds)\n", best, nr, nc, ns);
  return 0;
}
