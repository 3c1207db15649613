/*
 * sim.h — TEST INFRASTRUCTURE ONLY: the synthetic genome and read simulator
 * shared by the golden-vector generator (gen_golden.c) and the SAM-parity
 * harness (sam_harness.c).  Our own code (no reference source): splitmix64,
 * a genome of iid ACGT with diverged interspersed repeats, tandem repeats and
 * N runs (restated for the bench by bwa-flow_amd/tools/synth.cpp
 * golden_genome), and reads with substitutions, 1-3 bp indels and Ns.
 */
#ifndef BWAGPU_ORACLE_SIM_H
#define BWAGPU_ORACLE_SIM_H
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* ---------------- RNG (splitmix64) ---------------- */
static uint64_t rng_s;
static uint64_t rnd(void)
{
  uint64_t z = (rng_s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}
static double urand(void) { return (rnd() >> 11) * (1.0 / 9007199254740992.0); }
static int irand(int n) { return (int)(urand() * n); }
static double nrand(void)
{
  double u = urand() + 1e-300, v = urand();
  return sqrt(-2 * log(u)) * cos(2 * M_PI * v);
}

/* ---------------- reference genome ---------------- */
static const char ACGT[] = "ACGT";

/* per Mb: 10 repeat families (4 copies each), 30 tandem repeats, 12 N runs
   (the counts of the 1 Mb golden genome; bwa-flow_amd/tools/synth.cpp
   golden_genome() restates this generator for the bench) */
static int per_mb(int k, int64_t L) { return (int)(k * (double)L / 1e6 + 0.5); }

static char *make_genome(int n_ctg, const int *ctg_len, int64_t *total)
{
  int64_t L = 0;
  for (int i = 0; i < n_ctg; ++i) L += ctg_len[i];
  char *g = (char *)malloc(L + 1);
  for (int64_t i = 0; i < L; ++i) g[i] = ACGT[rnd() & 3];
  const int n_fam = per_mb(10, L), n_tan = per_mb(30, L), n_nrun = per_mb(12, L);
  /* interspersed repeats: 4 copies per family, 1% diverged */
  for (int fam = 0; fam < n_fam; ++fam) {
    int len = 300 + irand(2700);
    int64_t src = (int64_t)(urand() * (L - len));
    for (int c = 0; c < 4; ++c) {
      int64_t dst = (int64_t)(urand() * (L - len));
      for (int k = 0; k < len; ++k) g[dst + k] = urand() < 0.01 ? ACGT[rnd() & 3] : g[src + k];
    }
  }
  /* tandem repeats */
  for (int t = 0; t < n_tan; ++t) {
    int per = 2 + irand(49), len = 200 + irand(800);
    int64_t dst = (int64_t)(urand() * (L - len));
    for (int k = per; k < len; ++k) g[dst + k] = urand() < 0.005 ? ACGT[rnd() & 3] : g[dst + k - per];
  }
  /* N runs (bwa turns them into random bases + holes, bntseq.c:261) */
  for (int t = 0; t < n_nrun; ++t) {
    int len = 10 + irand(300);
    int64_t dst = (int64_t)(urand() * (L - len));
    memset(g + dst, 'N', len);
  }
  g[L] = 0;
  *total = L;
  return g;
}

static int nt4(char c)
{
  switch (c) {
    case 'A': return 0; case 'C': return 1; case 'G': return 2; case 'T': return 3;
    default: return 4;
  }
}
static char comp(char c)
{
  switch (c) {
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
    default: return 'N';
  }
}

/* copy `len` bases of g starting at p (forward) with errors into out; returns length */
static int mutate(const char *src, int n, char *out, int cap)
{
  int o = 0;
  for (int i = 0; i < n && o < cap; ++i) {
    double u = urand();
    if (u < 0.0005) out[o++] = 'N';
    else if (u < 0.0005 + 0.008) { char c; do c = ACGT[rnd() & 3]; while (c == src[i]); out[o++] = c; }
    else if (u < 0.0005 + 0.008 + 0.0005) { /* deletion of 1-3 */
      i += irand(3);
    } else if (u < 0.0005 + 0.008 + 0.001) { /* insertion of 1-3 then the base */
      int k = 1 + irand(3);
      while (k-- && o < cap) out[o++] = ACGT[rnd() & 3];
      if (o < cap) out[o++] = src[i];
    } else out[o++] = src[i];
  }
  return o;
}

#endif
