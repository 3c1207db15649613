/*
 * gen_golden.c — TEST INFRASTRUCTURE ONLY: golden-vector generator.
 *
 * Linked (Makefile -> _ref/gen_golden) against the REFERENCE's bwa objects
 * compiled from /root/reference/bwa.  It
 *   1. writes a synthetic multi-contig reference (iid ACGT + diverged
 *      interspersed repeats + tandem repeats + N runs) and indexes it with the
 *      reference's own bwa_idx_build (bwa/bwtindex.c:256),
 *   2. simulates reads (pairs, ~N(400,40) fragments, 0.8% subs, 0.1% indels,
 *      some Ns, chimeras, junk and contig-straddling fragments),
 *   3. seeds + chains each read with the reference's own code exactly as
 *      bwa-flow's SeqsToChains does (src/bwa_wrapper.cpp:110-113:
 *      mem_chain -> mem_chain_flt -> mem_flt_chained_seeds),
 *   4. runs the reference mem_chain2aln (bwa/bwamem.c:641-795) per chain the
 *      way ChainsToRegions::compute does (src/Pipeline.cpp:514-529), recording
 *      every ksw_extend2 call through -Wl,--wrap, and
 *   5. dumps everything as raw little-endian arrays into <outdir>/ for
 *      gen_golden.py to pack into tests/golden/*.npz.
 *
 * usage: gen_golden <outdir> <seed> <n_pairs> <len_mode:150|100|250|mix> <opt_mode:0|1|2>
 *                   [genome_len [record]]
 *   genome_len  default 1,000,000 (contigs 500k/300k/200k); any other length
 *               keeps the 50/30/20 % contig split and scales the repeat
 *               families, tandem repeats and N runs per Mb (the bench's
 *               chr21-sized C2 genome: oracle/gen_c2_fixture.py)
 *   record      1 (default) records every ksw_extend2 / bwa_gen_cigar2 call
 *               and runs mem_reg2aln on every region; 0 skips both
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

chain_v mem_chain(const mem_opt_t *opt, const bwt_t *bwt, const bntseq_t *bns, int len,
                  const uint8_t *seq, void *buf);
int mem_chain_flt(const mem_opt_t *opt, int n_chn, chain_t *a);
void mem_flt_chained_seeds(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                           const uint8_t *query, int n_chn, chain_t *a);
void mem_chain2aln(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                   const uint8_t *query, const chain_t *c, mem_alnreg_v *av);
int bwa_idx_build(const char *fa, const char *prefix, int algo_type, int block_size);

/* ---------------- ksw_extend2 recorder ---------------- */
typedef struct { int32_t qlen, tlen, w, end_bonus, zdrop, h0; int64_t qoff, toff; } rtask_t;
typedef struct { int32_t score, qle, tle, gtle, gscore, max_off; } rres_t;
static kvec_t(rtask_t) g_tasks;
static kvec_t(rres_t) g_res;
static kvec_t(uint8_t) g_qpool, g_tpool;
static int g_rec = 1;

int __real_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                       const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore,
                       int *max_off);
int __wrap_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                       const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle, int *gscore,
                       int *max_off)
{
  int r = __real_ksw_extend2(qlen, query, tlen, target, m, mat, o_del, e_del, o_ins, e_ins, w,
                             end_bonus, zdrop, h0, qle, tle, gtle, gscore, max_off);
  if (g_rec) {
    rtask_t t = {qlen, tlen, w, end_bonus, zdrop, h0, (int64_t)g_qpool.n, (int64_t)g_tpool.n};
    rres_t o = {r, *qle, *tle, *gtle, *gscore, *max_off};
    for (int i = 0; i < qlen; ++i) kv_push(uint8_t, g_qpool, query[i]);
    for (int i = 0; i < tlen; ++i) kv_push(uint8_t, g_tpool, target[i]);
    kv_push(rtask_t, g_tasks, t);
    kv_push(rres_t, g_res, o);
  }
  return r;
}

/* ---------------- mem_reg2aln / bwa_gen_cigar2 recorder ---------------- */
typedef struct { int64_t rb, re, qoff; int32_t l_seq, qb, qe, truesc, w, read; } ctask_t;
typedef struct { int64_t pos; int32_t rid, is_rev, n_cigar, NM, cig_off, md_off, md_len, pad; } cres_t;
typedef struct { int32_t task, w, l_query, score, n_cigar, NM, cig_off, md_off; int64_t rb, re; } ccall_t;
static kvec_t(ctask_t) g_ctasks;
static kvec_t(cres_t) g_cres;
static kvec_t(ccall_t) g_ccalls;
static kvec_t(uint32_t) g_cig;
static kvec_t(char) g_md;
uint32_t *__real_bwa_gen_cigar2(const int8_t mat[25], int o_del, int e_del, int o_ins, int e_ins, int w_,
                                int64_t l_pac, const uint8_t *pac, int l_query, uint8_t *query, int64_t rb,
                                int64_t re, int *score, int *n_cigar, int *NM);
uint32_t *__wrap_bwa_gen_cigar2(const int8_t mat[25], int o_del, int e_del, int o_ins, int e_ins, int w_,
                                int64_t l_pac, const uint8_t *pac, int l_query, uint8_t *query, int64_t rb,
                                int64_t re, int *score, int *n_cigar, int *NM)
{
  uint32_t *c = __real_bwa_gen_cigar2(mat, o_del, e_del, o_ins, e_ins, w_, l_pac, pac, l_query, query, rb, re,
                                      score, n_cigar, NM);
  ccall_t k = {(int32_t)g_ctasks.n - 1, w_, l_query, *score, *n_cigar, *NM, (int32_t)g_cig.n, (int32_t)g_md.n, rb,
               re};
  if (c) {
    for (int i = 0; i < *n_cigar; ++i) kv_push(uint32_t, g_cig, c[i]);
    const char *md = (const char *)(c + *n_cigar);
    for (size_t i = 0; i <= strlen(md); ++i) kv_push(char, g_md, md[i]);
  }
  kv_push(ccall_t, g_ccalls, k);
  return c;
}

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
    fprintf(stderr, "usage: gen_golden <outdir> <seed> <n_pairs> <150|100|250|mix> <opt_mode>\n");
    return 1;
  }
  const char *dir = argv[1];
  rng_s = strtoull(argv[2], 0, 10);
  int n_pairs = atoi(argv[3]);
  const char *lm = argv[4];
  int opt_mode = atoi(argv[5]);
  char fa[4096];
  int ctg_len[3] = {500000, 300000, 200000};
  int64_t G;
  if (argc > 6) {
    const int64_t gl = strtoll(argv[6], 0, 10);
    ctg_len[0] = (int)(gl / 2);
    ctg_len[1] = (int)(gl * 3 / 10);
    ctg_len[2] = (int)(gl - ctg_len[0] - ctg_len[1]);
  }
  const int record = argc > 7 ? atoi(argv[7]) : 1;

  bwa_verbose = 1;
  uint64_t read_seed = rng_s;
  rng_s = 1234; /* the genome is the same for every fixture */
  char *g = make_genome(3, ctg_len, &G);
  rng_s = read_seed;
  snprintf(fa, sizeof fa, "%s/ref.fa", dir);
  FILE *f = fopen(fa, "w");
  int64_t off = 0;
  for (int c = 0; c < 3; ++c) {
    fprintf(f, ">chr%d\n", c + 1);
    for (int64_t i = 0; i < ctg_len[c]; i += 60) {
      int64_t n = ctg_len[c] - i < 60 ? ctg_len[c] - i : 60;
      fwrite(g + off + i, 1, n, f);
      fputc('\n', f);
    }
    off += ctg_len[c];
  }
  fclose(f);
  bwa_idx_build(fa, fa, BWTALGO_AUTO, 10000000);
  bwaidx_t *idx = bwa_idx_load(fa, BWA_IDX_ALL);
  if (!idx) { fprintf(stderr, "index load failed\n"); return 1; }

  mem_opt_t *opt = mem_opt_init();
  if (opt_mode == 1) { /* non-default scoring exercises every opt field */
    opt->a = 2; opt->b = 5; opt->o_del = 7; opt->e_del = 2; opt->o_ins = 5; opt->e_ins = 3;
    opt->w = 30; opt->zdrop = 40; opt->pen_clip5 = 3; opt->pen_clip3 = 9;
    bwa_fill_scmat(opt->a, opt->b, opt->mat);
  } else if (opt_mode == 2) { /* small band + aggressive z-drop: retries and breaks */
    opt->w = 8; opt->zdrop = 15; opt->pen_clip5 = opt->pen_clip3 = 1;
  }

  kvec_t(int64_t) seq_off;
  kvec_t(uint8_t) seq;
  kvec_t(int32_t) rco, cso, crid, nreg;
  kvec_t(float) cfr;
  kvec_t(seed_t) seeds;
  kvec_t(mem_alnreg_t) regs;
  kv_init(seq_off); kv_init(seq); kv_init(rco); kv_init(cso); kv_init(crid); kv_init(cfr);
  kv_init(seeds); kv_init(regs); kv_init(nreg);
  kv_push(int64_t, seq_off, 0);
  kv_push(int32_t, rco, 0);
  kv_push(int32_t, cso, 0);

  char *buf = (char *)malloc(4096), *frag = (char *)malloc(8192);
  for (int p = 0; p < n_pairs; ++p) {
    int L;
    if (!strcmp(lm, "mix")) L = (int[]){100, 150, 250}[p % 3];
    else L = atoi(lm);
    int fl = (int)(400 + 40 * nrand());
    if (fl < L + 10) fl = L + 10;
    if (fl > 4000) fl = 4000;
    int64_t pos;
    if (urand() < 0.02) { /* straddle / hug a contig junction */
      int c = irand(2);
      int64_t j = 0;
      for (int k = 0; k <= c; ++k) j += ctg_len[k];
      pos = j - irand(fl);
    } else pos = (int64_t)(urand() * (G - fl));
    if (pos < 0) pos = 0;
    if (pos + fl > G) pos = G - fl;
    memcpy(frag, g + pos, fl);
    int strand = rnd() & 1;
    for (int e = 0; e < 2; ++e) {
      int n;
      double kind = urand();
      if (kind < 0.005) { /* junk read: no chains */
        n = L;
        for (int i = 0; i < n; ++i) buf[i] = ACGT[rnd() & 3];
      } else {
        char tmp[4096];
        int fwd = (e == 0) ^ strand;
        if (fwd) memcpy(tmp, frag, L);
        else for (int i = 0; i < L; ++i) tmp[i] = comp(frag[fl - 1 - i]);
        if (kind < 0.015) { /* chimera: second half from elsewhere */
          int64_t q = (int64_t)(urand() * (G - L));
          memcpy(tmp + L / 2, g + q, L - L / 2);
        }
        n = mutate(tmp, L, buf, L + 16);
        if (n > L) n = L;
      }
      uint8_t q[4096];
      for (int i = 0; i < n; ++i) q[i] = (uint8_t)nt4(buf[i]);
      for (int i = 0; i < n; ++i) kv_push(uint8_t, seq, q[i]);
      kv_push(int64_t, seq_off, (int64_t)seq.n);

      g_rec = 0;
      chain_v chn = mem_chain(opt, idx->bwt, idx->bns, n, q, 0);
      chn.n = mem_chain_flt(opt, (int)chn.n, chn.a);
      mem_flt_chained_seeds(opt, idx->bns, idx->pac, n, q, (int)chn.n, chn.a);
      g_rec = record;
      mem_alnreg_v av;
      kv_init(av);
      for (size_t c = 0; c < chn.n; ++c) {
        chain_t *ch = &chn.a[c];
        for (int s = 0; s < ch->n; ++s) kv_push(seed_t, seeds, ch->seeds[s]);
        kv_push(int32_t, cso, (int32_t)seeds.n);
        kv_push(int32_t, crid, ch->rid);
        kv_push(float, cfr, ch->frac_rep);
        mem_chain2aln(opt, idx->bns, idx->pac, n, q, ch, &av);
        free(ch->seeds);
      }
      free(chn.a);
      /* the SAM stage's CIGAR step on every region (bwa_wrapper.cpp:611) */
      for (size_t k = 0; record && k < av.n; ++k) {
        const mem_alnreg_t *ar = &av.a[k];
        ctask_t t = {ar->rb, ar->re, (int64_t)(seq.n - n), n, ar->qb, ar->qe, ar->truesc, ar->w,
                     (int32_t)(seq_off.n - 2)};
        kv_push(ctask_t, g_ctasks, t);
        mem_aln_t a = mem_reg2aln(opt, idx->bns, idx->pac, n, (const char *)q, ar);
        cres_t o = {a.pos, a.rid, a.is_rev, a.n_cigar, a.NM, (int32_t)g_cig.n, (int32_t)g_md.n, 0, 0};
        for (int i = 0; i < a.n_cigar; ++i) kv_push(uint32_t, g_cig, a.cigar[i]);
        const char *md = (const char *)(a.cigar + a.n_cigar);
        o.md_len = (int32_t)strlen(md);
        for (int i = 0; i <= o.md_len; ++i) kv_push(char, g_md, md[i]);
        kv_push(cres_t, g_cres, o);
        free(a.cigar);
      }
      kv_push(int32_t, rco, (int32_t)crid.n);
      kv_push(int32_t, nreg, (int32_t)av.n);
      for (size_t k = 0; k < av.n; ++k) kv_push(mem_alnreg_t, regs, av.a[k]);
      free(av.a);
    }
  }

  /* opt in bwagpu_opt_t order */
  int32_t ov[10] = {opt->a, opt->b, opt->o_del, opt->e_del, opt->o_ins, opt->e_ins,
                    opt->pen_clip5, opt->pen_clip3, opt->w, opt->zdrop};
  wr(dir, "opt_int", ov, sizeof ov);
  wr(dir, "opt_mat", opt->mat, 25);
  int64_t lp = idx->bns->l_pac;
  wr(dir, "l_pac", &lp, 8);
  int64_t *aoff = (int64_t *)malloc(8 * idx->bns->n_seqs);
  int32_t *alen = (int32_t *)malloc(4 * idx->bns->n_seqs);
  for (int i = 0; i < idx->bns->n_seqs; ++i) { aoff[i] = idx->bns->anns[i].offset; alen[i] = idx->bns->anns[i].len; }
  wr(dir, "ann_offset", aoff, 8 * idx->bns->n_seqs);
  wr(dir, "ann_len", alen, 4 * idx->bns->n_seqs);
  wr(dir, "pac", idx->pac, (size_t)(lp / 4 + 1));
  wr(dir, "seq_off", seq_off.a, 8 * seq_off.n);
  wr(dir, "seq", seq.a, seq.n);
  wr(dir, "read_chain_off", rco.a, 4 * rco.n);
  wr(dir, "chain_seed_off", cso.a, 4 * cso.n);
  wr(dir, "chain_rid", crid.a, 4 * crid.n);
  wr(dir, "chain_frac_rep", cfr.a, 4 * cfr.n);
  wr(dir, "seeds", seeds.a, sizeof(seed_t) * seeds.n);
  wr(dir, "reg_n", nreg.a, 4 * nreg.n);
  wr(dir, "regs", regs.a, sizeof(mem_alnreg_t) * regs.n);
  wr(dir, "tasks", g_tasks.a, sizeof(rtask_t) * g_tasks.n);
  wr(dir, "task_res", g_res.a, sizeof(rres_t) * g_res.n);
  wr(dir, "qpool", g_qpool.a, g_qpool.n);
  wr(dir, "tpool", g_tpool.a, g_tpool.n);
  wr(dir, "cig_tasks", g_ctasks.a, sizeof(ctask_t) * g_ctasks.n);
  wr(dir, "cig_res", g_cres.a, sizeof(cres_t) * g_cres.n);
  wr(dir, "cig_calls", g_ccalls.a, sizeof(ccall_t) * g_ccalls.n);
  wr(dir, "cig_ops", g_cig.a, 4 * g_cig.n);
  wr(dir, "cig_md", g_md.a, g_md.n);
  fprintf(stderr, "[gen_golden] cigar jobs=%zu gen_cigar2 calls=%zu\n", g_ctasks.n, g_ccalls.n);
  fprintf(stderr, "[gen_golden] reads=%zu chains=%zu seeds=%zu regions=%zu ksw_calls=%zu sizeof(alnreg)=%zu\n",
          seq_off.n - 1, crid.n, seeds.n, regs.n, g_tasks.n, sizeof(mem_alnreg_t));
  bwa_idx_destroy(idx);
  free(opt);
  free(g);
  return 0;
}
