/*
 * gen_chain.c — TEST INFRASTRUCTURE ONLY: golden vectors for seeding's
 * chaining (bwa-flow's SeqsToChains after the interval search:
 * src/bwa_wrapper.cpp:105-115 = mem_chain -> mem_chain_flt ->
 * mem_flt_chained_seeds).
 *
 * Linked (oracle/Makefile -> _ref/gen_chain) against the REFERENCE's bwa
 * objects compiled from /root/reference/bwa.  It builds the bwa index of the
 * golden genome (sim.h, the same genome and index gen_seed.c writes to
 * tests/golden/seed_bwt.npz), simulates reads and runs, per read, the
 * reference's own
 *   mem_chain             (bwa/bwamem.c:260-330: mem_collect_intv, bwt_sa,
 *                          bns_intv2rid, the kbtree of chains, test_and_merge)
 *   mem_chain_flt         (bwamem.c:336-396)
 *   mem_flt_chained_seeds (bwamem.c:607-624, mem_seed_sw -> ksw_align2)
 * and dumps both the raw chains (mem_chain's kbtree traversal order) and the
 * filtered ones with every mem_chain_t field.  Nothing of the chaining is
 * restated here; only the read simulation and the dump are ours.
 *
 * usage: gen_chain <outdir> <read_seed> <n_reads> <lens> <opt_mode> [alt_rid] [min_raw_chains]
 *   lens            comma-separated read lengths, cycled
 *   opt_mode        0 defaults; 1 non-default chaining options (w, max_occ,
 *                   max_chain_gap, min_chain_weight, max_chain_extend,
 *                   mask_level, drop_ratio) and scoring (a=2)
 *   alt_rid         contig index marked ALT in the bns (-1: none)
 *   min_raw_chains  keep only reads whose raw chain count reaches this
 *                   (repeat-rich sets: many chains, equal chain positions)
 * Output (raw little-endian files in <outdir>):
 *   opt      int32 [w, max_chain_gap, max_occ, min_chain_weight, max_chain_extend,
 *                   min_seed_len, a, b, o_del, e_del, o_ins, e_ins, split_width,
 *                   max_mem_intv], float [mask_level, drop_ratio, split_factor]
 *   seq_off  int64 [n+1], seq uint8 (0..4)
 *   raw_n    int32 [n]: mem_chain's chains per read
 *   raw_chn  int64 [.][4]: pos, rid, n_seeds, is_alt
 *   raw_seed int64 [.][3]: rbeg, qbeg, len
 *   chn_n    int32 [n]: chains after mem_chain_flt
 *   chn      int64 [.][7]: pos, rid, n_seeds (after mem_flt_chained_seeds),
 *                          w, kept, first, is_alt;  chn_frac float32 [.]
 *   seed     int64 [.][4]: rbeg, qbeg, len, score
 *   stats    int64 [reads with equal raw chain positions, reads where
 *                   mem_flt_chained_seeds ran]
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bntseq.h"
#include "bwa.h"
#include "bwamem.h"
#include "bwt.h"
#include "kvec.h"
#include "sim.h"

int bwa_idx_build(const char *fa, const char *prefix, int algo_type, int block_size);

typedef struct {
  int64_t rbeg;
  int32_t qbeg, len;
  int score;
} seed_t;
typedef struct {
  int n, m, first, rid;
  uint32_t w : 29, kept : 2, is_alt : 1;
  float frac_rep;
  int64_t pos;
  seed_t *seeds;
} chain_t; /* == mem_chain_t, bwamem.c:180-186 */
typedef struct { size_t n, m; chain_t *a; } chain_v;

chain_v mem_chain(const mem_opt_t *opt, const bwt_t *bwt, const bntseq_t *bns, int len, const uint8_t *seq,
                  void *buf);
int mem_chain_flt(const mem_opt_t *opt, int n_chn, chain_t *a);
void mem_flt_chained_seeds(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                           const uint8_t *query, int n_chn, chain_t *a);

static void wr(const char *dir, const char *name, const void *p, size_t sz)
{
  char fn[4096];
  snprintf(fn, sizeof fn, "%s/%s.bin", dir, name);
  FILE *f = fopen(fn, "wb");
  if (!f) { perror(fn); exit(1); }
  if (sz && fwrite(p, 1, sz, f) != sz) { perror(fn); exit(1); }
  fclose(f);
}

int main(int argc, char *argv[])
{
  if (argc < 6) {
    fprintf(stderr, "usage: gen_chain <outdir> <read_seed> <n_reads> <lens> <opt_mode> [alt_rid] [min_raw_chains]\n");
    return 1;
  }
  const char *dir = argv[1];
  const uint64_t read_seed = strtoull(argv[2], 0, 10);
  const int n_reads = atoi(argv[3]);
  int lens[16], n_lens = 0;
  for (char *p = argv[4]; *p && n_lens < 16;) {
    lens[n_lens++] = (int)strtol(p, &p, 10);
    if (*p == ',') ++p;
  }
  const int opt_mode = atoi(argv[5]);
  const int alt_rid = argc > 6 ? atoi(argv[6]) : -1;
  const int min_raw = argc > 7 ? atoi(argv[7]) : 0;

  /* the golden genome and its index, exactly as gen_seed.c builds them */
  const int64_t GL = 1000000;
  int ctg_len[3] = {(int)(GL / 2), (int)(GL * 3 / 10), 0};
  ctg_len[2] = (int)(GL - ctg_len[0] - ctg_len[1]);
  int64_t G;
  bwa_verbose = 1;
  rng_s = 1234;
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
  bwaidx_t *idx = bwa_idx_load(fa, BWA_IDX_ALL);
  if (!idx) { fprintf(stderr, "index load failed\n"); return 1; }
  if (alt_rid >= 0 && alt_rid < idx->bns->n_seqs) idx->bns->anns[alt_rid].is_alt = 1;

  mem_opt_t *opt = mem_opt_init();
  if (opt_mode == 1) {
    opt->w = 20;
    opt->max_chain_gap = 300;
    opt->max_occ = 40;
    opt->min_chain_weight = 25;
    opt->max_chain_extend = 3;
    opt->mask_level = 0.7f;
    opt->drop_ratio = 0.3f;
    opt->a = 2;
    opt->b = 5;
    bwa_fill_scmat(opt->a, opt->b, opt->mat);
  }
  int32_t ov[14] = {opt->w, opt->max_chain_gap, opt->max_occ, opt->min_chain_weight, opt->max_chain_extend,
                    opt->min_seed_len, opt->a, opt->b, opt->o_del, opt->e_del, opt->o_ins, opt->e_ins,
                    opt->split_width, (int32_t)opt->max_mem_intv};
  float fv[3] = {opt->mask_level, opt->drop_ratio, opt->split_factor};
  wr(dir, "opt", ov, sizeof ov);
  wr(dir, "optf", fv, sizeof fv);

  rng_s = read_seed;
  kvec_t(int64_t) seq_off, raw_chn, raw_seed, chn, seed;
  kvec_t(uint8_t) seq;
  kvec_t(int32_t) raw_n, chn_n;
  kvec_t(float) chn_frac;
  kv_init(seq_off); kv_init(raw_chn); kv_init(raw_seed); kv_init(chn); kv_init(seed);
  kv_init(seq); kv_init(raw_n); kv_init(chn_n); kv_init(chn_frac);
  kv_push(int64_t, seq_off, 0);
  int64_t stats[2] = {0, 0};
  char buf[4096], tmp[4096];
  int kept_reads = 0;
  for (long tries = 0; kept_reads < n_reads && tries < 400L * n_reads; ++tries) {
    const int L = lens[tries % n_lens];
    int n;
    const double kind = urand();
    if (kind < 0.01) { /* junk */
      n = L;
      for (int i = 0; i < n; ++i) buf[i] = ACGT[rnd() & 3];
    } else {
      int64_t pos;
      if (kind < 0.03) { /* straddle a contig junction */
        const int c = irand(2);
        int64_t j = 0;
        for (int k = 0; k <= c; ++k) j += ctg_len[k];
        pos = j - 1 - irand(L);
      } else pos = (int64_t)(urand() * (G - L));
      if (pos < 0) pos = 0;
      if (pos + L > G) pos = G - L;
      if (rnd() & 1) memcpy(tmp, g + pos, L);
      else for (int i = 0; i < L; ++i) tmp[i] = comp(g[pos + L - 1 - i]);
      n = mutate(tmp, L, buf, L + 16);
      if (n > L) n = L;
    }
    uint8_t q[4096];
    for (int i = 0; i < n; ++i) q[i] = (uint8_t)nt4(buf[i]);

    chain_v c = mem_chain(opt, idx->bwt, idx->bns, n, q, 0);
    if ((int)c.n < min_raw) {
      for (size_t k = 0; k < c.n; ++k) free(c.a[k].seeds);
      free(c.a);
      continue;
    }
    ++kept_reads;
    for (int i = 0; i < n; ++i) kv_push(uint8_t, seq, q[i]);
    kv_push(int64_t, seq_off, (int64_t)seq.n);
    kv_push(int32_t, raw_n, (int32_t)c.n);
    int dup = 0;
    for (size_t k = 0; k < c.n; ++k) {
      const chain_t *p = &c.a[k];
      if (k && p->pos == c.a[k - 1].pos) dup = 1;
      kv_push(int64_t, raw_chn, p->pos);
      kv_push(int64_t, raw_chn, p->rid);
      kv_push(int64_t, raw_chn, p->n);
      kv_push(int64_t, raw_chn, p->is_alt);
      for (int s = 0; s < p->n; ++s) {
        kv_push(int64_t, raw_seed, p->seeds[s].rbeg);
        kv_push(int64_t, raw_seed, p->seeds[s].qbeg);
        kv_push(int64_t, raw_seed, p->seeds[s].len);
      }
    }
    stats[0] += dup;
    c.n = mem_chain_flt(opt, (int)c.n, c.a);
    {
      /* mem_flt_chained_seeds' own early return (bwamem.c:609-611) */
      const double min_l = opt->min_chain_weight ? 1.1f * opt->min_chain_weight : 5.5f * log(n);
      if (!(min_l > 0.05f * n) && c.n) stats[1] += 1;
    }
    mem_flt_chained_seeds(opt, idx->bns, idx->pac, n, q, (int)c.n, c.a);
    kv_push(int32_t, chn_n, (int32_t)c.n);
    for (size_t k = 0; k < c.n; ++k) {
      const chain_t *p = &c.a[k];
      kv_push(int64_t, chn, p->pos);
      kv_push(int64_t, chn, p->rid);
      kv_push(int64_t, chn, p->n);
      kv_push(int64_t, chn, p->w);
      kv_push(int64_t, chn, p->kept);
      kv_push(int64_t, chn, p->first);
      kv_push(int64_t, chn, p->is_alt);
      kv_push(float, chn_frac, p->frac_rep);
      for (int s = 0; s < p->n; ++s) {
        kv_push(int64_t, seed, p->seeds[s].rbeg);
        kv_push(int64_t, seed, p->seeds[s].qbeg);
        kv_push(int64_t, seed, p->seeds[s].len);
        kv_push(int64_t, seed, p->seeds[s].score);
      }
      free(p->seeds);
    }
    free(c.a);
  }
  wr(dir, "seq_off", seq_off.a, 8 * seq_off.n);
  wr(dir, "seq", seq.a, seq.n);
  wr(dir, "raw_n", raw_n.a, 4 * raw_n.n);
  wr(dir, "raw_chn", raw_chn.a, 8 * raw_chn.n);
  wr(dir, "raw_seed", raw_seed.a, 8 * raw_seed.n);
  wr(dir, "chn_n", chn_n.a, 4 * chn_n.n);
  wr(dir, "chn", chn.a, 8 * chn.n);
  wr(dir, "chn_frac", chn_frac.a, 4 * chn_frac.n);
  wr(dir, "seed", seed.a, 8 * seed.n);
  wr(dir, "stats", stats, sizeof stats);
  /* what the fixture's consumers must already hold (checked by gen_chain.py
     against tests/golden/ref.npz and seed_bwt.npz, not stored again) */
  wr(dir, "pac", idx->pac, (size_t)(idx->bns->l_pac / 4 + 1));
  wr(dir, "bwt", idx->bwt->bwt, 4 * (size_t)idx->bwt->bwt_size);
  fprintf(stderr, "[gen_chain] reads=%d raw_chains=%zu chains=%zu seeds=%zu dup_pos_reads=%ld flt_seed_reads=%ld\n",
          kept_reads, raw_chn.n / 4, chn.n / 7, seed.n / 4, (long)stats[0], (long)stats[1]);
  free(g);
  free(opt);
  bwa_idx_destroy(idx);
  return 0;
}
