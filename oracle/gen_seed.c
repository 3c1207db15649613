/*
 * gen_seed.c — TEST INFRASTRUCTURE ONLY: golden vectors for seeding's
 * interval collection (mem_collect_intv, bwa/bwamem.c:120-167).
 *
 * Linked (oracle/Makefile -> _ref/gen_seed) against the REFERENCE's bwa
 * objects compiled from /root/reference/bwa.  It builds a bwa index of the
 * golden genome (sim.h, the generator and seed gen_golden.c uses), simulates
 * reads, and for every read collects its SMEM intervals the way
 * mem_collect_intv does — the control flow of bwamem.c:120-167 around the
 * reference's own bwt_smem1 (bwt.c:353), bwt_seed_strategy1 (bwt.c:358) and
 * ks_introsort_mem_intv (the KSORT_INIT of bwamem.c:90-91).  mem_collect_intv
 * itself is static in bwamem.c, so its ~40 lines of control flow are the only
 * part restated here.  Output (raw little-endian files in <outdir>):
 *   bwt_hdr   int64 [primary, L2[0..4], seq_len, bwt_size]
 *   bwt       uint32 [bwt_size]  (bwt.h:46-57: 128-base blocks of 4 uint64
 *             counts + 8 words of 2-bit bases)
 *   seq_off   int64 [n+1], seq uint8 (0..4)
 *   intv_n    int32 [n], intv uint64 [sum intv_n][4] = bwtintv_t {x0, x1, x2, info}
 *   opt       int32 [min_seed_len, split_width, max_mem_intv], float split_factor
 *   sa_hdr    int64 [sa_intv, n_sa], sa uint64 [n_sa]  (the sampled suffix array)
 *   sa_q/sa_v uint64: BWT positions and the reference bwt_sa of each
 *
 * usage: gen_seed <outdir> <seed> <n_reads> <len:150|100|250|mix> [genome_len] [n_frac]
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bwa.h"
#include "bwamem.h"
#include "bwt.h"
#include "kvec.h"
#include "sim.h"

int bwa_idx_build(const char *fa, const char *prefix, int algo_type, int block_size);
void ks_introsort_mem_intv(size_t n, bwtintv_t a[]); /* bwamem.c:90-91 */

static void wr(const char *dir, const char *name, const void *p, size_t sz)
{
  char fn[4096];
  snprintf(fn, sizeof fn, "%s/%s.bin", dir, name);
  FILE *f = fopen(fn, "wb");
  if (!f) { perror(fn); exit(1); }
  if (sz && fwrite(p, 1, sz, f) != sz) { perror(fn); exit(1); }
  fclose(f);
}

/* bwamem.c:120-167 around the reference's own bwt_smem1 / bwt_seed_strategy1 / sort */
static void collect(const mem_opt_t *opt, const bwt_t *bwt, int len, const uint8_t *seq, bwtintv_v *mem,
                    bwtintv_v *mem1, bwtintv_v *tmpv[2])
{
  int i, k, x = 0, old_n;
  const int split_len = (int)(opt->min_seed_len * opt->split_factor + .499);
  mem->n = 0;
  while (x < len) {
    if (seq[x] < 4) {
      x = bwt_smem1(bwt, len, seq, x, 1, mem1, tmpv);
      for (i = 0; i < (int)mem1->n; ++i) {
        bwtintv_t *p = &mem1->a[i];
        if ((int)((uint32_t)p->info - (p->info >> 32)) >= opt->min_seed_len) kv_push(bwtintv_t, *mem, *p);
      }
    } else ++x;
  }
  old_n = (int)mem->n;
  for (k = 0; k < old_n; ++k) {
    bwtintv_t *p = &mem->a[k];
    int start = p->info >> 32, end = (int32_t)p->info;
    if (end - start < split_len || p->x[2] > (uint64_t)opt->split_width) continue;
    bwt_smem1(bwt, len, seq, (start + end) >> 1, p->x[2] + 1, mem1, tmpv);
    for (i = 0; i < (int)mem1->n; ++i)
      if ((uint32_t)mem1->a[i].info - (mem1->a[i].info >> 32) >= (uint32_t)opt->min_seed_len)
        kv_push(bwtintv_t, *mem, mem1->a[i]);
  }
  if (opt->max_mem_intv > 0) {
    x = 0;
    while (x < len) {
      if (seq[x] < 4) {
        bwtintv_t m;
        x = bwt_seed_strategy1(bwt, len, seq, x, opt->min_seed_len, opt->max_mem_intv, &m);
        if (m.x[2] > 0) kv_push(bwtintv_t, *mem, m);
      } else ++x;
    }
  }
  ks_introsort_mem_intv(mem->n, mem->a);
}

int main(int argc, char *argv[])
{
  if (argc < 5) {
    fprintf(stderr, "usage: gen_seed <outdir> <seed> <n_reads> <150|100|250|mix> [genome_len] [n_frac]\n");
    return 1;
  }
  const char *dir = argv[1];
  const uint64_t read_seed = strtoull(argv[2], 0, 10);
  const int n_reads = atoi(argv[3]);
  const char *lm = argv[4];
  const int64_t GL = argc > 5 ? strtoll(argv[5], 0, 10) : 1000000;
  const double n_frac = argc > 6 ? atof(argv[6]) : 0.0;
  int ctg_len[3] = {(int)(GL / 2), (int)(GL * 3 / 10), 0};
  ctg_len[2] = (int)(GL - ctg_len[0] - ctg_len[1]);
  int64_t G;
  bwa_verbose = 1;
  rng_s = 1234; /* the golden genome */
  char *g = make_genome(3, ctg_len, &G);
  char fa[4096];
  snprintf(fa, sizeof fa, "%s/ref.fa", dir);
  FILE *f = fopen(fa, "w");
  if (!f) { perror(fa); return 1; }
  for (int c = 0, off = 0; c < 3; off += ctg_len[c], ++c) {
    fprintf(f, ">chr%d\n", c + 1);
    for (int64_t i = 0; i < ctg_len[c]; i += 60) {
      const int64_t k = ctg_len[c] - i < 60 ? ctg_len[c] - i : 60;
      fwrite(g + off + i, 1, k, f);
      fputc('\n', f);
    }
  }
  fclose(f);
  bwa_idx_build(fa, fa, BWTALGO_AUTO, 10000000);
  bwaidx_t *idx = bwa_idx_load(fa, BWA_IDX_BWT); /* bwa_idx_load_bwt also restores the SA (bwa.c:244-260) */
  if (!idx) { fprintf(stderr, "index load failed\n"); return 1; }
  const bwt_t *bwt = idx->bwt;
  int64_t hdr[8] = {(int64_t)bwt->primary, (int64_t)bwt->L2[0], (int64_t)bwt->L2[1], (int64_t)bwt->L2[2],
                    (int64_t)bwt->L2[3],   (int64_t)bwt->L2[4], (int64_t)bwt->seq_len, (int64_t)bwt->bwt_size};
  wr(dir, "bwt_hdr", hdr, sizeof hdr);
  wr(dir, "bwt", bwt->bwt, 4 * (size_t)bwt->bwt_size);
  /* the sampled suffix array and bwt_sa (bwt.c:86-96) on a spread of BWT
     positions: every sa_intv-th one, its neighbours, primary, the ends */
  int64_t sah[2] = {bwt->sa_intv, (int64_t)bwt->n_sa};
  wr(dir, "sa_hdr", sah, sizeof sah);
  wr(dir, "sa", bwt->sa, 8 * (size_t)bwt->n_sa);
  {
    kvec_t(uint64_t) qk, qv;
    kv_init(qk); kv_init(qv);
    const uint64_t n = bwt->seq_len + 1;
    uint64_t s = 0x9e3779b97f4a7c15ULL;
    for (int i = 0; i < 20000; ++i) {
      s = s * 6364136223846793005ULL + 1442695040888963407ULL;
      kv_push(uint64_t, qk, (s >> 11) % n);
    }
    const uint64_t fixed[] = {0, 1, 31, 32, 33, bwt->primary - 1, bwt->primary, bwt->primary + 1, n - 2, n - 1};
    for (size_t i = 0; i < sizeof fixed / sizeof fixed[0]; ++i)
      if (fixed[i] < n) kv_push(uint64_t, qk, fixed[i]);
    for (size_t i = 0; i < qk.n; ++i) kv_push(uint64_t, qv, bwt_sa(bwt, qk.a[i]));
    wr(dir, "sa_q", qk.a, 8 * qk.n);
    wr(dir, "sa_v", qv.a, 8 * qv.n);
    free(qk.a); free(qv.a);
  }

  mem_opt_t *opt = mem_opt_init();
  int32_t ov[3] = {opt->min_seed_len, opt->split_width, opt->max_mem_intv};
  wr(dir, "opt", ov, sizeof ov);
  wr(dir, "split_factor", &opt->split_factor, sizeof(float));

  rng_s = read_seed;
  kvec_t(int64_t) seq_off;
  kvec_t(uint8_t) seq;
  kvec_t(int32_t) intv_n;
  bwtintv_v all, mem, mem1, t0, t1, *tmpv[2] = {&t0, &t1};
  kv_init(seq_off); kv_init(seq); kv_init(intv_n); kv_init(all); kv_init(mem); kv_init(mem1);
  kv_init(t0); kv_init(t1);
  kv_push(int64_t, seq_off, 0);
  char buf[4096], tmp[4096];
  for (int r = 0; r < n_reads; ++r) {
    const int L = !strcmp(lm, "mix") ? (int[]){100, 150, 250, 40, 19, 12}[r % 6] : atoi(lm);
    int n;
    const double kind = urand();
    if (kind < 0.01) { /* junk */
      n = L;
      for (int i = 0; i < n; ++i) buf[i] = ACGT[rnd() & 3];
    } else {
      int64_t pos = (int64_t)(urand() * (G - L));
      if (rnd() & 1) memcpy(tmp, g + pos, L);
      else for (int i = 0; i < L; ++i) tmp[i] = comp(g[pos + L - 1 - i]);
      n = mutate(tmp, L, buf, L + 16);
      if (n > L) n = L;
    }
    uint8_t q[4096];
    for (int i = 0; i < n; ++i) q[i] = (uint8_t)nt4(buf[i]);
    for (int i = 0; n_frac > 0 && i < n; ++i) /* ambiguous bases: N runs and singletons */
      if (urand() < n_frac) q[i] = 4;
    for (int i = 0; i < n; ++i) kv_push(uint8_t, seq, q[i]);
    kv_push(int64_t, seq_off, (int64_t)seq.n);
    collect(opt, bwt, n, q, &mem, &mem1, tmpv);
    kv_push(int32_t, intv_n, (int32_t)mem.n);
    for (size_t k = 0; k < mem.n; ++k) kv_push(bwtintv_t, all, mem.a[k]);
  }
  wr(dir, "seq_off", seq_off.a, 8 * seq_off.n);
  wr(dir, "seq", seq.a, seq.n);
  wr(dir, "intv_n", intv_n.a, 4 * intv_n.n);
  wr(dir, "intv", all.a, sizeof(bwtintv_t) * all.n);
  fprintf(stderr, "[gen_seed] reads=%d intervals=%ld bwt_words=%ld\n", n_reads, (long)all.n, (long)bwt->bwt_size);
  free(g);
  bwa_idx_destroy(idx);
  return 0;
}
