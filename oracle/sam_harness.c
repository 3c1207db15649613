/*
 * sam_harness.c — TEST INFRASTRUCTURE ONLY: SAM-level parity of the GPU stage.
 *
 * Linked (oracle/Makefile -> _ref/sam_harness) against the REFERENCE's bwa
 * objects compiled from /root/reference/bwa.  It builds a bwa index of a
 * synthetic genome (sim.h), simulates read pairs, and aligns them batch by
 * batch (batches of >= K bases, as `bwa mem -K` and bwa-flow's getKseqBatch,
 * src/Pipeline.cpp:123,146) in one of three modes:
 *
 *   ref    the reference's own mem_process_seqs (bwa/bwamem.c:1220-1249):
 *          worker1 -> mem_pestat -> worker2, exactly what `bwa mem` runs;
 *   split  the same pipeline restated stage by stage the way bwa-flow splits
 *          it (SeqsToChains -> ChainsToRegions -> RegionsToSam,
 *          src/Pipeline.cpp:110-113, 503-544, 546-648): mem_chain ->
 *          mem_chain_flt -> mem_flt_chained_seeds per read, then the
 *          reference mem_chain2aln per chain, then mem_sort_dedup_patch +
 *          is_alt (bwamem.c:1088-1100), mem_pestat, mem_sam_pe — must print
 *          the same SAM as `ref` (checks the harness itself, no GPU);
 *   gpu    `split` with the mem_chain2aln loop replaced by ONE
 *          bwagpu_chain2aln call per batch (bwa-flow_amd/lib/libbwagpu.so,
 *          dlopen'ed) — the drop-in this repository builds;
 *   gpusam `gpu` plus the SAM stage's Smith-Waterman on the device: mate
 *          rescue (ksw_align2 in mem_matesw) and CIGAR generation
 *          (mem_reg2aln) answered from the call cache of
 *          bwa-flow_amd/lib/libgpusam.so through the interposers of
 *          bwa-flow_amd/host/sam_hooks.c, the mem_sam_pe loop run as
 *          collect -> flush -> replay passes (include/bwagpu_sam.h).
 *
 *   gpuchain SeqsToChains and ChainsToRegions fused on the device
 *          (bwagpu_seqs2regions: interval search, SA lookups, the kbtree
 *          chaining, mem_chain_flt, mem_flt_chained_seeds and mem_chain2aln;
 *          no chain exists on the host), then the SAM stage as in `gpusam`.
 *   gpuseed `gpusam` with seeding's interval collection and SA lookups on the
 *          device too: bwagpu_collect_intv (mem_collect_intv) and
 *          bwagpu_bwt_sa (bwt_sa) per batch; the chaining around them
 *          (mem_chain's body, bwamem.c:262-318, and test_and_merge,
 *          bwamem.c:199-221, restated below with the reference's own
 *          kbtree.h) stays on the host, then the reference's mem_chain_flt /
 *          mem_flt_chained_seeds.
 *
 * The reference's objects are linked as a shared object (_ref/libbwaref.so,
 * -fPIC), so sam_hooks.c's ksw_align2 / mem_reg2aln interpose on every call
 * bwa makes; without a cache attached they forward to bwa's own.
 *
 * Every mode prints the SAM records (header: bwa_print_sam_hdr) to <out.sam>
 * and one JSON line of per-phase wall times to stderr.  The -m gpu test
 * (tests/test_gpu_sam.py) diffs `ref` against `gpu` byte for byte.
 *
 * usage: sam_harness <ref|split|gpu|gpusam|gpuseed|gpuchain> <workdir> <out.sam> <seed> <n_pairs> <len:150|100|250|mix>
 *                    [batch_bases=10000000] [threads=8] [genome_len=1000000]
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdio.h>
#include <unistd.h>
#include <stdlib.h>
#include <string.h>

#include "bntseq.h"
#include "bwa.h"
#include "bwamem.h"
#include "bwt.h"
#include "kvec.h"
#include "utils.h"
#include "sim.h"
#include "bwagpu.h"
#include "bwagpu_sam.h"

int bwagpu_sam_hooks_attach(bwagpu_samcache_t *c); /* bwa-flow_amd/host/sam_hooks.c */
int bwagpu_sam_hooks_errors(void);
void bwagpu_sam_hooks_quiet(int quiet);
int bwagpu_sam_hooks_take_misses(void);

typedef struct {
  int64_t rbeg;
  int32_t qbeg, len;
  int score;
} seed_t; /* == mem_seed_t, bwamem.c:174-178 */
typedef struct {
  int n, m, first, rid;
  uint32_t w : 29, kept : 2, is_alt : 1;
  float frac_rep;
  int64_t pos;
  seed_t *seeds;
} chain_t; /* == mem_chain_t, bwamem.c:180-186 */
typedef struct { size_t n, m; chain_t *a; } chain_v;

#include "kbtree.h"
#define chain_cmp(a, b) (((b).pos < (a).pos) - ((a).pos < (b).pos)) /* bwamem.c:192 */
KBTREE_INIT(chn, chain_t, chain_cmp)

chain_v mem_chain(const mem_opt_t *opt, const bwt_t *bwt, const bntseq_t *bns, int len, const uint8_t *seq,
                  void *buf);
int mem_chain_flt(const mem_opt_t *opt, int n_chn, chain_t *a);
void mem_flt_chained_seeds(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                           const uint8_t *query, int n_chn, chain_t *a);
void mem_chain2aln(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                   const uint8_t *query, const chain_t *c, mem_alnreg_v *av);
int mem_sort_dedup_patch(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, uint8_t *query, int n,
                         mem_alnreg_t *a);
int mem_sam_pe(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, const mem_pestat_t pes[4],
               uint64_t id, bseq1_t s[2], mem_alnreg_v a[2]);
void kt_for(int n_threads, void (*func)(void *, int, int), void *data, int n);
int bwa_idx_build(const char *fa, const char *prefix, int algo_type, int block_size);
extern unsigned char nst_nt4_table[256];

/* ---------------- the GPU library (dlopen: CPU modes run without it) ---------------- */
static struct {
  void *h;
  int (*create)(int, const bwagpu_opt_t *, const bwagpu_bns_t *, const uint8_t *, bwagpu_ctx_t **);
  int (*destroy)(bwagpu_ctx_t *);
  int (*chain2aln)(bwagpu_ctx_t *, const bwagpu_batch_t *, bwagpu_alnreg_t *, int32_t *);
  const char *(*last_error)(const bwagpu_ctx_t *);
  int (*set_bwt)(bwagpu_ctx_t *, const bwagpu_bwt_t *);
  int (*collect_intv)(bwagpu_ctx_t *, const bwagpu_seedopt_t *, int32_t, const int64_t *, const uint8_t *, int32_t,
                      bwagpu_intv_t *, int64_t, int32_t *);
  int (*bwt_sa)(bwagpu_ctx_t *, int64_t, const uint64_t *, uint64_t *);
  int (*set_alt)(bwagpu_ctx_t *, const uint8_t *);
  int (*seqs2regions)(bwagpu_ctx_t *, const bwagpu_seedopt_t *, const bwagpu_chainopt_t *, int32_t, const int64_t *,
                      const uint8_t *, int32_t *, const bwagpu_alnreg_t **, int64_t *);
  /* libgpusam.so (gpusam mode) */
  int (*sc_create)(bwagpu_ctx_t *, int32_t, int32_t, bwagpu_samcache_t **);
  int (*sc_destroy)(bwagpu_samcache_t *);
  int (*sc_clear)(bwagpu_samcache_t *);
  int64_t (*sc_flush)(bwagpu_samcache_t *);
  int (*sc_stats)(const bwagpu_samcache_t *, int64_t *);
} G;

static void gpusam_load(void)
{
  const char *p = getenv("BWAGPU_SAM_LIB");
  void *h = dlopen(p ? p : "bwa-flow_amd/lib/libgpusam.so", RTLD_NOW | RTLD_GLOBAL);
  if (!h) { fprintf(stderr, "dlopen: %s\n", dlerror()); exit(2); }
  G.sc_create = (int (*)(bwagpu_ctx_t *, int32_t, int32_t, bwagpu_samcache_t **))dlsym(h, "bwagpu_samcache_create");
  G.sc_destroy = (int (*)(bwagpu_samcache_t *))dlsym(h, "bwagpu_samcache_destroy");
  G.sc_clear = (int (*)(bwagpu_samcache_t *))dlsym(h, "bwagpu_samcache_clear");
  G.sc_flush = (int64_t (*)(bwagpu_samcache_t *))dlsym(h, "bwagpu_samcache_flush");
  G.sc_stats = (int (*)(const bwagpu_samcache_t *, int64_t *))dlsym(h, "bwagpu_samcache_stats");
  if (!G.sc_create || !G.sc_destroy || !G.sc_clear || !G.sc_flush || !G.sc_stats) {
    fprintf(stderr, "libgpusam: missing symbol\n");
    exit(2);
  }
}

static void gpu_load(void)
{
  const char *p = getenv("BWAGPU_LIB");
  G.h = dlopen(p ? p : "bwa-flow_amd/lib/libbwagpu.so", RTLD_NOW);
  if (!G.h) { fprintf(stderr, "dlopen: %s\n", dlerror()); exit(2); }
  G.create = (int (*)(int, const bwagpu_opt_t *, const bwagpu_bns_t *, const uint8_t *, bwagpu_ctx_t **))dlsym(G.h, "bwagpu_create");
  G.destroy = (int (*)(bwagpu_ctx_t *))dlsym(G.h, "bwagpu_destroy");
  G.chain2aln = (int (*)(bwagpu_ctx_t *, const bwagpu_batch_t *, bwagpu_alnreg_t *, int32_t *))dlsym(G.h, "bwagpu_chain2aln");
  G.last_error = (const char *(*)(const bwagpu_ctx_t *))dlsym(G.h, "bwagpu_last_error");
  G.set_bwt = (int (*)(bwagpu_ctx_t *, const bwagpu_bwt_t *))dlsym(G.h, "bwagpu_set_bwt");
  G.collect_intv = (int (*)(bwagpu_ctx_t *, const bwagpu_seedopt_t *, int32_t, const int64_t *, const uint8_t *,
                            int32_t, bwagpu_intv_t *, int64_t, int32_t *))dlsym(G.h, "bwagpu_collect_intv");
  G.bwt_sa = (int (*)(bwagpu_ctx_t *, int64_t, const uint64_t *, uint64_t *))dlsym(G.h, "bwagpu_bwt_sa");
  G.set_alt = (int (*)(bwagpu_ctx_t *, const uint8_t *))dlsym(G.h, "bwagpu_set_alt");
  G.seqs2regions = (int (*)(bwagpu_ctx_t *, const bwagpu_seedopt_t *, const bwagpu_chainopt_t *, int32_t,
                            const int64_t *, const uint8_t *, int32_t *, const bwagpu_alnreg_t **,
                            int64_t *))dlsym(G.h, "bwagpu_seqs2regions");
  if (!G.create || !G.destroy || !G.chain2aln || !G.last_error) { fprintf(stderr, "libbwagpu: missing symbol\n"); exit(2); }
}

/* ---------------- reads ---------------- */
static bseq1_t *simulate(const char *g, int64_t G_len, const int *ctg_len, int n_pairs, const char *lm, int *n_out)
{
  bseq1_t *s = (bseq1_t *)calloc(2 * (size_t)n_pairs, sizeof(bseq1_t));
  char frag[8192], buf[4096], tmp[4096], name[64];
  for (int p = 0; p < n_pairs; ++p) {
    const int L = !strcmp(lm, "mix") ? (int[]){100, 150, 250}[p % 3] : atoi(lm);
    int fl = (int)(400 + 40 * nrand());
    if (fl < L + 10) fl = L + 10;
    if (fl > 4000) fl = 4000;
    int64_t pos;
    if (urand() < 0.02) { /* straddle a contig junction */
      const int c = irand(2);
      int64_t j = 0;
      for (int k = 0; k <= c; ++k) j += ctg_len[k];
      pos = j - irand(fl);
    } else pos = (int64_t)(urand() * (G_len - fl));
    if (pos < 0) pos = 0;
    if (pos + fl > G_len) pos = G_len - fl;
    memcpy(frag, g + pos, fl);
    const int strand = rnd() & 1;
    snprintf(name, sizeof name, "r%d", p);
    for (int e = 0; e < 2; ++e) {
      int n;
      const double kind = urand();
      if (kind < 0.005) { /* junk */
        n = L;
        for (int i = 0; i < n; ++i) buf[i] = ACGT[rnd() & 3];
      } else {
        const int fwd = (e == 0) ^ strand;
        if (fwd) memcpy(tmp, frag, L);
        else for (int i = 0; i < L; ++i) tmp[i] = comp(frag[fl - 1 - i]);
        if (kind < 0.015) memcpy(tmp + L / 2, g + (int64_t)(urand() * (G_len - L)), L - L / 2); /* chimera */
        n = mutate(tmp, L, buf, L + 16);
        if (n > L) n = L;
      }
      bseq1_t *q = &s[2 * p + e];
      q->name = strdup(name);
      q->l_seq = n;
      q->seq = (char *)malloc(n + 1);
      q->qual = (char *)malloc(n + 1);
      memcpy(q->seq, buf, n);
      memset(q->qual, 'I', n);
      q->seq[n] = q->qual[n] = 0;
    }
  }
  *n_out = 2 * n_pairs;
  return s;
}

/* ---------------- the split pipeline ---------------- */
typedef struct {
  const mem_opt_t *opt;
  const bwaidx_t *idx;
  bseq1_t *seqs;
  chain_v *chn;
  mem_alnreg_v *regs;
  const mem_pestat_t *pes;
  int64_t n_processed;
} hw_t;

static void w_seed(void *data, int i, int tid) /* SeqsToChains (bwa_wrapper.cpp:110-113, bwamem.c:1072-1077) */
{
  hw_t *w = (hw_t *)data;
  bseq1_t *s = &w->seqs[i];
  for (int k = 0; k < s->l_seq; ++k) s->seq[k] = s->seq[k] < 4 ? s->seq[k] : nst_nt4_table[(int)s->seq[k]];
  chain_v c = mem_chain(w->opt, w->idx->bwt, w->idx->bns, s->l_seq, (uint8_t *)s->seq, 0);
  c.n = mem_chain_flt(w->opt, (int)c.n, c.a);
  mem_flt_chained_seeds(w->opt, w->idx->bns, w->idx->pac, s->l_seq, (uint8_t *)s->seq, (int)c.n, c.a);
  w->chn[i] = c;
}
static void w_ext_cpu(void *data, int i, int tid) /* ChainsToRegions::compute (Pipeline.cpp:514-529) */
{
  hw_t *w = (hw_t *)data;
  kv_init(w->regs[i]);
  for (size_t c = 0; c < w->chn[i].n; ++c)
    mem_chain2aln(w->opt, w->idx->bns, w->idx->pac, w->seqs[i].l_seq, (uint8_t *)w->seqs[i].seq, &w->chn[i].a[c],
                  &w->regs[i]);
}
static void w_free_chains(void *data, int i, int tid)
{
  hw_t *w = (hw_t *)data;
  for (size_t c = 0; c < w->chn[i].n; ++c) free(w->chn[i].a[c].seeds);
  free(w->chn[i].a);
}
static void w_post(void *data, int i, int tid) /* mem_align1_core's tail (bwamem.c:1088-1100) */
{
  hw_t *w = (hw_t *)data;
  mem_alnreg_v *r = &w->regs[i];
  r->n = mem_sort_dedup_patch(w->opt, w->idx->bns, w->idx->pac, (uint8_t *)w->seqs[i].seq, (int)r->n, r->a);
  for (size_t k = 0; k < r->n; ++k)
    if (r->a[k].rid >= 0 && w->idx->bns->anns[r->a[k].rid].is_alt) r->a[k].is_alt = 1;
}
static void w_sam(void *data, int i, int tid) /* worker2 (bwamem.c:1214-1216) */
{
  hw_t *w = (hw_t *)data;
  mem_sam_pe(w->opt, w->idx->bns, w->idx->pac, w->pes, (w->n_processed >> 1) + i, &w->seqs[i << 1], &w->regs[i << 1]);
  free(w->regs[i << 1 | 0].a);
  free(w->regs[i << 1 | 1].a);
}

/* one SAM pass over a list of pairs (gpusam modes): each pair's regions are a
   fresh copy of the stage's (mem_sam_pe consumes them); miss[k] = 1 when the
   pair's calls missed the cache, i.e. its text must be redone */
typedef struct {
  hw_t *w;
  const mem_alnreg_v *keep;
  const int *pairs;
  char *miss;
} pass_t;
static void w_sam_pass(void *data, int k, int tid)
{
  pass_t *p = (pass_t *)data;
  hw_t *w = p->w;
  const int i = p->pairs[k];
  mem_alnreg_v r[2];
  for (int e = 0; e < 2; ++e) {
    const mem_alnreg_v *s = &p->keep[i << 1 | e];
    r[e] = *s;
    r[e].a = (mem_alnreg_t *)malloc(sizeof(mem_alnreg_t) * (s->m ? s->m : 1));
    memcpy(r[e].a, s->a, sizeof(mem_alnreg_t) * s->n);
  }
  free(w->seqs[i << 1].sam); free(w->seqs[i << 1 | 1].sam);
  w->seqs[i << 1].sam = w->seqs[i << 1 | 1].sam = 0;
  (void)bwagpu_sam_hooks_take_misses();
  mem_sam_pe(w->opt, w->idx->bns, w->idx->pac, w->pes, (w->n_processed >> 1) + i, &w->seqs[i << 1], r);
  p->miss[k] = bwagpu_sam_hooks_take_misses() > 0;
  free(r[0].a);
  free(r[1].a);
}

/* ---------------- seeding on the device (gpuseed mode) ---------------- */
/* test_and_merge, bwamem.c:199-221 (static in the reference build) */
static int merge_seed(const mem_opt_t *opt, int64_t l_pac, chain_t *c, const seed_t *p, int seed_rid)
{
  const seed_t *last = &c->seeds[c->n - 1];
  const int64_t qend = last->qbeg + last->len, rend = last->rbeg + last->len;
  if (seed_rid != c->rid) return 0;
  if (p->qbeg >= c->seeds[0].qbeg && p->qbeg + p->len <= qend && p->rbeg >= c->seeds[0].rbeg && p->rbeg + p->len <= rend)
    return 1;
  if ((last->rbeg < l_pac || c->seeds[0].rbeg < l_pac) && p->rbeg >= l_pac) return 0;
  const int64_t x = p->qbeg - last->qbeg, y = p->rbeg - last->rbeg;
  if (y >= 0 && x - y <= opt->w && y - x <= opt->w && x - last->len < opt->max_chain_gap &&
      y - last->len < opt->max_chain_gap) {
    if (c->n == c->m) {
      c->m <<= 1;
      c->seeds = (seed_t *)realloc(c->seeds, c->m * sizeof(seed_t));
    }
    c->seeds[c->n++] = *p;
    return 1;
  }
  return 0;
}

typedef struct {
  const mem_opt_t *opt;
  const bntseq_t *bns;
  bseq1_t *seqs;
  chain_v *chn;
  const int32_t *intv_n;
  const int64_t *intv_off; /* first interval of each read */
  const bwagpu_intv_t *intv;
  const int64_t *sa_off;   /* first SA value of each read */
  const uint64_t *sa;
} sw_t;

/* mem_chain's body after mem_collect_intv (bwamem.c:273-318) with the
   device's intervals and bwt_sa values, in the same order */
static void w_chain(void *data, int i, int tid)
{
  sw_t *w = (sw_t *)data;
  const mem_opt_t *opt = w->opt;
  const int len = w->seqs[i].l_seq;
  chain_v chain = {0, 0, 0};
  if (len < opt->min_seed_len) { w->chn[i] = chain; return; }
  kbtree_t(chn) *tree = kb_init(chn, KB_DEFAULT_SIZE);
  const bwagpu_intv_t *iv = w->intv + w->intv_off[i];
  const int n_iv = w->intv_n[i];
  int b = 0, e = 0, l_rep = 0;
  for (int k = 0; k < n_iv; ++k) { /* frac_rep, bwamem.c:274-281 */
    const int sb = (int)(iv[k].info >> 32), se = (int)(uint32_t)iv[k].info;
    if (iv[k].x[2] <= (uint64_t)opt->max_occ) continue;
    if (sb > e) l_rep += e - b, b = sb, e = se;
    else e = e > se ? e : se;
  }
  l_rep += e - b;
  const uint64_t *sa = w->sa + w->sa_off[i];
  int64_t si = 0;
  for (int k = 0; k < n_iv; ++k) { /* bwamem.c:282-309 */
    const bwagpu_intv_t *p = &iv[k];
    const int slen = (int)((uint32_t)p->info - (p->info >> 32));
    const int64_t step = p->x[2] > (uint64_t)opt->max_occ ? (int64_t)(p->x[2] / opt->max_occ) : 1;
    int count = 0;
    for (int64_t kk = 0; kk < (int64_t)p->x[2] && count < opt->max_occ; kk += step, ++count) {
      chain_t tmp, *lower, *upper;
      seed_t sd;
      int to_add = 0;
      sd.rbeg = tmp.pos = (int64_t)sa[si++];
      sd.qbeg = (int32_t)(p->info >> 32);
      sd.score = sd.len = slen;
      const int rid = bns_intv2rid(w->bns, sd.rbeg, sd.rbeg + sd.len);
      if (rid < 0) continue;
      if (kb_size(tree)) {
        kb_intervalp(chn, tree, &tmp, &lower, &upper);
        if (!lower || !merge_seed(opt, w->bns->l_pac, lower, &sd, rid)) to_add = 1;
      } else to_add = 1;
      if (to_add) {
        tmp.n = 1; tmp.m = 4;
        tmp.seeds = (seed_t *)calloc(tmp.m, sizeof(seed_t));
        tmp.seeds[0] = sd;
        tmp.rid = rid;
        tmp.is_alt = !!w->bns->anns[rid].is_alt;
        kb_putp(chn, tree, &tmp);
      }
    }
  }
  kv_resize(chain_t, chain, kb_size(tree));
#define traverse_func(p_) (chain.a[chain.n++] = *(p_))
  __kb_traverse(chain_t, tree, traverse_func);
#undef traverse_func
  for (size_t k = 0; k < chain.n; ++k) chain.a[k].frac_rep = (float)l_rep / len;
  kb_destroy(chn, tree);
  chain.n = mem_chain_flt(opt, (int)chain.n, chain.a); /* SeqsToChains' filters (bwamem.c:1076-1077) */
  w->chn[i] = chain;
}
static void w_flt(void *data, int i, int tid)
{
  hw_t *w = (hw_t *)data;
  mem_flt_chained_seeds(w->opt, w->idx->bns, w->idx->pac, w->seqs[i].l_seq, (uint8_t *)w->seqs[i].seq,
                        (int)w->chn[i].n, w->chn[i].a);
}
static void w_nt4(void *data, int i, int tid)
{
  hw_t *w = (hw_t *)data;
  bseq1_t *s = &w->seqs[i];
  for (int k = 0; k < s->l_seq; ++k) s->seq[k] = s->seq[k] < 4 ? s->seq[k] : nst_nt4_table[(int)s->seq[k]];
}

/* SeqsToChains with the intervals and SA lookups on the device */
static void seed_gpu(bwagpu_ctx_t *ctx, hw_t *w, int n, int T, double *t_dev)
{
  const mem_opt_t *opt = w->opt;
  kt_for(T, w_nt4, w, n);
  int64_t *seq_off = (int64_t *)malloc(8 * (n + 1)), nb = 0;
  seq_off[0] = 0;
  for (int i = 0; i < n; ++i) seq_off[i + 1] = (nb += w->seqs[i].l_seq);
  uint8_t *seq = (uint8_t *)malloc(nb + 1);
  for (int i = 0; i < n; ++i) memcpy(seq + seq_off[i], w->seqs[i].seq, w->seqs[i].l_seq);
  bwagpu_seedopt_t so = {opt->min_seed_len, opt->split_width, opt->max_mem_intv, opt->split_factor};
  int32_t *cnt = (int32_t *)malloc(4 * (n + 1));
  int64_t cap = 64 * (int64_t)n;
  bwagpu_intv_t *iv = (bwagpu_intv_t *)malloc(sizeof(bwagpu_intv_t) * cap);
  double t0 = realtime();
  int rc = G.collect_intv(ctx, &so, n, seq_off, seq, 4096, iv, cap, cnt);
  if (rc == BWAGPU_E_UNSUPPORTED) { /* a batch with more intervals: size from the counts and again */
    cap = 0;
    for (int i = 0; i < n; ++i) cap += cnt[i] < 0 ? -cnt[i] : cnt[i];
    iv = (bwagpu_intv_t *)realloc(iv, sizeof(bwagpu_intv_t) * (cap + 1));
    rc = G.collect_intv(ctx, &so, n, seq_off, seq, 1 << 16, iv, cap, cnt);
  }
  if (rc) { fprintf(stderr, "bwagpu_collect_intv: rc=%d %s\n", rc, G.last_error(ctx)); exit(3); }
  /* the SA positions mem_chain visits (bwamem.c:282-288), in order */
  int64_t *ioff = (int64_t *)malloc(8 * (n + 1)), *soff = (int64_t *)malloc(8 * (n + 1)), ns = 0, ni = 0;
  for (int i = 0; i < n; ++i) {
    ioff[i] = ni;
    soff[i] = ns;
    if (w->seqs[i].l_seq >= opt->min_seed_len)
      for (int k = 0; k < cnt[i]; ++k) {
        const uint64_t x2 = iv[ni + k].x[2];
        const uint64_t step = x2 > (uint64_t)opt->max_occ ? x2 / opt->max_occ : 1;
        ns += (int64_t)((x2 + step - 1) / step < (uint64_t)opt->max_occ ? (x2 + step - 1) / step : (uint64_t)opt->max_occ);
      }
    ni += cnt[i];
  }
  ioff[n] = ni;
  soff[n] = ns;
  uint64_t *ks = (uint64_t *)malloc(8 * (ns + 1)), *sa = (uint64_t *)malloc(8 * (ns + 1));
  for (int i = 0, q = 0; i < n; ++i) {
    if (w->seqs[i].l_seq < opt->min_seed_len) continue;
    for (int k = 0; k < cnt[i]; ++k) {
      const bwagpu_intv_t *p = &iv[ioff[i] + k];
      const int64_t step = p->x[2] > (uint64_t)opt->max_occ ? (int64_t)(p->x[2] / opt->max_occ) : 1;
      int count = 0;
      for (int64_t kk = 0; kk < (int64_t)p->x[2] && count < opt->max_occ; kk += step, ++count) ks[q++] = p->x[0] + kk;
    }
  }
  rc = G.bwt_sa(ctx, ns, ks, sa);
  if (rc) { fprintf(stderr, "bwagpu_bwt_sa: rc=%d %s\n", rc, G.last_error(ctx)); exit(3); }
  *t_dev += realtime() - t0;
  sw_t sw = {opt, w->idx->bns, w->seqs, w->chn, cnt, ioff, iv, soff, sa};
  kt_for(T, w_chain, &sw, n);
  kt_for(T, w_flt, w, n);
  free(seq_off); free(seq); free(cnt); free(iv); free(ioff); free(soff); free(ks); free(sa);
}

/* SeqsToChains + ChainsToRegions in one device call (gpuchain mode): the
   reads go in, each read's mem_alnreg_v comes back (malloc'd per read, the
   ownership rule of ChainsToRegions); no chain is built on the host */
typedef struct {
  hw_t *w;
  const int32_t *cnt;
  const int64_t *off;
  const bwagpu_alnreg_t *regs;
} regs_t;
static void w_regs(void *data, int i, int tid)
{
  regs_t *f = (regs_t *)data;
  mem_alnreg_v *r = &f->w->regs[i];
  r->n = r->m = f->cnt[i];
  r->a = (mem_alnreg_t *)malloc(sizeof(mem_alnreg_t) * (f->cnt[i] ? f->cnt[i] : 1));
  memcpy(r->a, f->regs + f->off[i], sizeof(mem_alnreg_t) * f->cnt[i]);
}
static void seqs2regions_gpu(bwagpu_ctx_t *ctx, hw_t *w, int n, int T, double *t_dev)
{
  const mem_opt_t *opt = w->opt;
  kt_for(T, w_nt4, w, n);
  static int64_t *seq_off, *off, k_n;
  static int32_t *cnt;
  static uint8_t *seq;
  static int64_t k_nb;
  if (n + 1 > k_n) {
    free(seq_off); free(off); free(cnt);
    k_n = 2 * (int64_t)(n + 1);
    seq_off = (int64_t *)malloc(8 * k_n);
    off = (int64_t *)malloc(8 * k_n);
    cnt = (int32_t *)malloc(4 * k_n);
  }
  int64_t nb = 0;
  seq_off[0] = 0;
  for (int i = 0; i < n; ++i) seq_off[i + 1] = (nb += w->seqs[i].l_seq);
  if (nb + 1 > k_nb) { free(seq); k_nb = 2 * (nb + 1); seq = (uint8_t *)malloc(k_nb); }
  for (int i = 0; i < n; ++i) memcpy(seq + seq_off[i], w->seqs[i].seq, w->seqs[i].l_seq);
  bwagpu_seedopt_t so = {opt->min_seed_len, opt->split_width, (int32_t)opt->max_mem_intv, opt->split_factor};
  bwagpu_chainopt_t co = {opt->max_occ, opt->max_chain_gap, opt->min_chain_weight, opt->max_chain_extend,
                          opt->mask_level, opt->drop_ratio};
  const bwagpu_alnreg_t *regs = 0;
  int64_t nreg = 0;
  const double t0 = realtime();
  const int rc = G.seqs2regions(ctx, &so, &co, n, seq_off, seq, cnt, &regs, &nreg);
  if (rc) { fprintf(stderr, "bwagpu_seqs2regions: rc=%d %s\n", rc, G.last_error(ctx)); exit(3); }
  *t_dev += realtime() - t0;
  off[0] = 0;
  for (int i = 0; i < n; ++i) off[i + 1] = off[i] + cnt[i];
  regs_t f = {w, cnt, off, regs};
  kt_for(T, w_regs, &f, n);
}

/* one bwagpu_chain2aln call for the whole batch: flatten, run, unflatten into
   malloc'd mem_alnreg_v (the ownership rule of ChainsToRegions, bwa_wrapper.cpp:824-830);
   the per-read copies run on the stage's threads (offsets from one serial pass) */
typedef struct {
  hw_t *w;
  int64_t *seq_off;
  uint8_t *seq;
  int32_t *rco, *cso, *rid;
  float *fr;
  bwagpu_seed_t *sd;
  bwagpu_alnreg_t *out;
  int32_t *on;
} flat_t;
static void w_flat(void *data, int i, int tid)
{
  flat_t *f = (flat_t *)data;
  hw_t *w = f->w;
  memcpy(f->seq + f->seq_off[i], w->seqs[i].seq, w->seqs[i].l_seq);
  int32_t c0 = f->rco[i], s0 = f->cso[c0];
  for (size_t c = 0; c < w->chn[i].n; ++c) {
    const chain_t *ch = &w->chn[i].a[c];
    for (int k = 0; k < ch->n; ++k) {
      bwagpu_seed_t t = {ch->seeds[k].rbeg, ch->seeds[k].qbeg, ch->seeds[k].len, ch->seeds[k].score, 0};
      f->sd[s0++] = t;
    }
    f->rid[c0] = ch->rid;
    f->fr[c0] = ch->frac_rep;
    f->cso[++c0] = s0;
  }
}
static void w_unflat(void *data, int i, int tid)
{
  flat_t *f = (flat_t *)data;
  mem_alnreg_v *r = &f->w->regs[i];
  r->n = r->m = f->on[i];
  r->a = (mem_alnreg_t *)malloc(sizeof(mem_alnreg_t) * (f->on[i] ? f->on[i] : 1));
  memcpy(r->a, f->out + f->cso[f->rco[i]], sizeof(mem_alnreg_t) * f->on[i]);
}
static double g_t_flat, g_t_call, g_t_unflat, g_t_pass[3], g_t_clear, g_t_pestat;
static void ext_gpu(bwagpu_ctx_t *ctx, hw_t *w, int n, int T)
{
  const double t_a = realtime();
  int64_t *seq_off = (int64_t *)malloc(8 * (n + 1));
  int32_t *rco = (int32_t *)malloc(4 * (n + 1));
  seq_off[0] = 0;
  rco[0] = 0;
  int64_t ns = 0;
  for (int i = 0; i < n; ++i) {
    seq_off[i + 1] = seq_off[i] + w->seqs[i].l_seq;
    rco[i + 1] = rco[i] + (int32_t)w->chn[i].n;
    for (size_t c = 0; c < w->chn[i].n; ++c) ns += w->chn[i].a[c].n;
  }
  const int64_t nc = rco[n], nb = seq_off[n];
  int32_t *cso = (int32_t *)malloc(4 * (nc + 1)), *rid = (int32_t *)malloc(4 * (nc + 1));
  /* chain seed offsets: one more serial pass over the chains (cheap) */
  cso[0] = 0;
  for (int i = 0, c0 = 0; i < n; ++i)
    for (size_t c = 0; c < w->chn[i].n; ++c, ++c0) cso[c0 + 1] = cso[c0] + w->chn[i].a[c].n;
  /* the big per-batch buffers are kept from batch to batch (grow only): fresh
     ones would page-fault on every byte of every batch */
  static uint8_t *k_seq;
  static bwagpu_seed_t *k_sd;
  static bwagpu_alnreg_t *k_out;
  static int64_t k_nb, k_ns;
  if (nb + 1 > k_nb) { free(k_seq); k_nb = 2 * (nb + 1); k_seq = (uint8_t *)malloc(k_nb); }
  if (ns + 1 > k_ns) {
    free(k_sd); free(k_out);
    k_ns = 2 * (ns + 1);
    k_sd = (bwagpu_seed_t *)malloc(sizeof(bwagpu_seed_t) * k_ns);
    k_out = (bwagpu_alnreg_t *)malloc(sizeof(bwagpu_alnreg_t) * k_ns);
  }
  flat_t f = {w, seq_off, k_seq, rco, cso, rid, (float *)malloc(4 * (nc + 1)), k_sd, k_out,
              (int32_t *)malloc(4 * (n + 1))};
  kt_for(T, w_flat, &f, n);
  const double t_b = realtime();
  bwagpu_batch_t b = {n, (int32_t)nc, (int32_t)ns, 0, nb, seq_off, f.seq, rco, cso, rid, f.fr, f.sd};
  const int rc = G.chain2aln(ctx, &b, f.out, f.on);
  if (rc) { fprintf(stderr, "bwagpu_chain2aln: rc=%d %s\n", rc, G.last_error(ctx)); exit(3); }
  const double t_c = realtime();
  kt_for(T, w_unflat, &f, n);
  g_t_flat += t_b - t_a;
  g_t_call += t_c - t_b;
  g_t_unflat += realtime() - t_c;
  free(seq_off); free(rco); free(cso); free(rid); free(f.fr); free(f.on);
}

/* the SAM stage with its Smith-Waterman on the device (include/bwagpu_sam.h):
   mem_sam_pe over copies of the regions with the cache attached.  Pass 0
   (every pair, no SAM text) queues the mate rescues and the CIGARs of the
   pairs that need no rescue; a flush runs them.  Pass 1 (every pair, with
   text) is final for every pair without a miss; the pairs that missed (their
   rescue found a hit, so they print a region pass 0 could not know) are
   flushed and redone alone until none misses. */

/* The cache clear and the regions' free after a batch's SAM passes run on a
   thread of their own while the next batch (on the other cache) aligns; a
   cache is reused two batches later, after its clearer is joined. */
typedef struct {
  bwagpu_samcache_t *cache;
  mem_alnreg_v *regs;
  int n, live;
  double t;
  pthread_t th;
} clearer_t;
static void *clearer_main(void *arg)
{
  clearer_t *c = (clearer_t *)arg;
  const double t0 = realtime();
  G.sc_clear(c->cache);
  for (int i = 0; i < c->n; ++i) free(c->regs[i].a);
  free(c->regs);
  c->t = realtime() - t0;
  return 0;
}
static void clearer_join(clearer_t *c)
{
  if (!c->live) return;
  pthread_join(c->th, 0);
  g_t_clear += c->t;
  c->live = 0;
}
static void clearer_start(clearer_t *c, bwagpu_samcache_t *cache, mem_alnreg_v *regs, int n)
{
  c->cache = cache;
  c->regs = regs;
  c->n = n;
  c->live = 1;
  pthread_create(&c->th, 0, clearer_main, c);
}

/* the passes; the caller clears `cache` and frees w->regs afterwards */
static void sam_passes(bwagpu_samcache_t *cache, hw_t *w, int n, int T, int64_t *n_passes, double *t_flush)
{
  const int np = n >> 1;
  int *pairs = (int *)malloc(sizeof(int) * (np + 1)), m = np;
  char *miss = (char *)calloc(np + 1, 1);
  for (int k = 0; k < np; ++k) pairs[k] = k;
  pass_t p = {w, w->regs, pairs, miss};
  bwagpu_sam_hooks_attach(cache);
  for (int pass = 0; m > 0; ++pass) {
    bwagpu_sam_hooks_quiet(pass == 0);
    const double tp = realtime();
    kt_for(T, w_sam_pass, &p, m);
    g_t_pass[pass < 2 ? pass : 2] += realtime() - tp;
    ++*n_passes;
    if (bwagpu_sam_hooks_errors()) { fprintf(stderr, "sam_hooks: the device flagged a CIGAR job\n"); exit(4); }
    int m2 = 0;
    for (int k = 0; k < m; ++k)
      if (pass == 0 || miss[k]) pairs[m2++] = pairs[k];  /* pass 0's text is never final */
    m = m2;
    if (m == 0) break;
    const double t0 = realtime();
    const int64_t rc = G.sc_flush(cache);
    *t_flush += realtime() - t0;
    if (rc < 0 || (rc == 0 && pass > 0)) { fprintf(stderr, "bwagpu_samcache_flush: %ld\n", (long)rc); exit(3); }
  }
  bwagpu_sam_hooks_quiet(0);
  bwagpu_sam_hooks_attach(0);
  free(pairs);
  free(miss);
}

/* SAM output on its own thread, one batch in flight (bwa's own main loop
   overlaps the same way: kt_pipeline's output step, bwa/fastmap.c): batch i is
   written and freed while batch i+1 is aligned; every mode uses it */
typedef struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  FILE *out;
  bseq1_t *seqs;
  int n, busy, stop;
} writer_t;
static void *writer_main(void *arg)
{
  writer_t *wr = (writer_t *)arg;
  pthread_mutex_lock(&wr->mu);
  for (;;) {
    while (!wr->busy && !wr->stop) pthread_cond_wait(&wr->cv, &wr->mu);
    if (!wr->busy) break;
    bseq1_t *seqs = wr->seqs;
    const int n = wr->n;
    pthread_mutex_unlock(&wr->mu);
    for (int i = 0; i < n; ++i) {
      fputs(seqs[i].sam, wr->out);
      free(seqs[i].sam);
      free(seqs[i].name); free(seqs[i].seq); free(seqs[i].qual);
    }
    pthread_mutex_lock(&wr->mu);
    wr->busy = 0;
    pthread_cond_broadcast(&wr->cv);
  }
  pthread_mutex_unlock(&wr->mu);
  return 0;
}
static void writer_wait(writer_t *wr)
{
  pthread_mutex_lock(&wr->mu);
  while (wr->busy) pthread_cond_wait(&wr->cv, &wr->mu);
  pthread_mutex_unlock(&wr->mu);
}
static void writer_put(writer_t *wr, bseq1_t *seqs, int n)
{
  writer_wait(wr);
  pthread_mutex_lock(&wr->mu);
  wr->seqs = seqs;
  wr->n = n;
  wr->busy = 1;
  pthread_cond_broadcast(&wr->cv);
  pthread_mutex_unlock(&wr->mu);
}

/* gpuchain: the device stage runs one record ahead (bwa-flow's kflow
   pipeline: SeqsToChains -> ChainsToRegions of record i+1 proceed while the SAM
   stage works on record i, src/main.cpp:262-371, kflow/include/kflow/Pipeline.h:98-144).
   A feeder thread owns its own device context and calls bwagpu_seqs2regions per
   record, in order, at most FEED_DEPTH records ahead of the main thread, which
   does the host post-processing, mem_pestat and the SAM passes (the SAM cache
   on a second context) and hands the record to the writer; record order and
   every per-record computation are those of the serial loop, so the SAM is the
   same bytes. */
enum { FEED_DEPTH = 2 };
typedef struct {
  int r0, n;
  hw_t *w;
} feed_job_t;
typedef struct {
  pthread_mutex_t mu;
  pthread_cond_t cv;
  feed_job_t *jobs;
  int n_jobs, produced, consumed;
  bwagpu_ctx_t *ctx;
  const mem_opt_t *opt;
  const bwaidx_t *idx;
  bseq1_t *all;
  int T;
  double t_busy, t_dev;
} feeder_t;
static void *feeder_main(void *arg)
{
  feeder_t *f = (feeder_t *)arg;
  for (int b = 0; b < f->n_jobs; ++b) {
    pthread_mutex_lock(&f->mu);
    while (f->produced - f->consumed >= FEED_DEPTH) pthread_cond_wait(&f->cv, &f->mu);
    pthread_mutex_unlock(&f->mu);
    feed_job_t *j = &f->jobs[b];
    hw_t *w = (hw_t *)calloc(1, sizeof(hw_t));
    w->opt = f->opt;
    w->idx = f->idx;
    w->seqs = f->all + j->r0;
    w->chn = (chain_v *)calloc(j->n, sizeof(chain_v));
    w->regs = (mem_alnreg_v *)calloc(j->n, sizeof(mem_alnreg_v));
    w->n_processed = j->r0;
    const double t0 = realtime();
    seqs2regions_gpu(f->ctx, w, j->n, f->T, &f->t_dev);
    f->t_busy += realtime() - t0;
    pthread_mutex_lock(&f->mu);
    j->w = w;
    ++f->produced;
    pthread_cond_broadcast(&f->cv);
    pthread_mutex_unlock(&f->mu);
  }
  return 0;
}
static hw_t *feeder_take(feeder_t *f, int b)
{
  pthread_mutex_lock(&f->mu);
  while (f->produced <= b) pthread_cond_wait(&f->cv, &f->mu);
  hw_t *w = f->jobs[b].w;
  pthread_mutex_unlock(&f->mu);
  return w;
}
static void feeder_done(feeder_t *f)
{
  pthread_mutex_lock(&f->mu);
  ++f->consumed;
  pthread_cond_broadcast(&f->cv);
  pthread_mutex_unlock(&f->mu);
}

int main(int argc, char *argv[])
{
  if (argc < 7) {
    fprintf(stderr, "usage: sam_harness <ref|split|gpu|index> <workdir> <out.sam> <seed> <n_pairs> <150|100|250|mix> "
                    "[batch_bases] [threads] [genome_len]\n");
    return 1;
  }
  const char *mode = argv[1], *dir = argv[2], *outp = argv[3];
  const uint64_t seed = strtoull(argv[4], 0, 10);
  const int n_pairs = atoi(argv[5]);
  const char *lm = argv[6];
  const int64_t K = argc > 7 ? strtoll(argv[7], 0, 10) : 10000000;
  const int T = argc > 8 ? atoi(argv[8]) : 8;
  const int64_t GL = argc > 9 ? strtoll(argv[9], 0, 10) : 1000000;
  const int is_chain = !strcmp(mode, "gpuchain");
  const int is_seed = is_chain || !strcmp(mode, "gpuseed");
  const int is_sam = is_seed || !strcmp(mode, "gpusam"), is_gpu = is_sam || !strcmp(mode, "gpu"),
            is_ref = !strcmp(mode, "ref");
  /* index: build (or find, by its stamp) the genome's bwa index in <workdir> and stop */
  const int is_index = !strcmp(mode, "index");
  if (!is_gpu && !is_ref && !is_index && strcmp(mode, "split")) { fprintf(stderr, "unknown mode %s\n", mode); return 1; }
  if (is_gpu) gpu_load();
  if (is_sam) gpusam_load();

  /* genome (the golden genome's generator and seed) + bwa index */
  int ctg_len[3] = {500000, 300000, 200000};
  if (GL != 1000000) {
    ctg_len[0] = (int)(GL / 2);
    ctg_len[1] = (int)(GL * 3 / 10);
    ctg_len[2] = (int)(GL - ctg_len[0] - ctg_len[1]);
  }
  int64_t G_len;
  bwa_verbose = 1;
  rng_s = 1234;
  char *g = make_genome(3, ctg_len, &G_len);
  char fa[4096], stamp[4200], want[64];
  snprintf(fa, sizeof fa, "%s/ref.fa", dir);
  snprintf(stamp, sizeof stamp, "%s/ref.fa.stamp", dir);
  snprintf(want, sizeof want, "golden 1234 %ld\n", (long)GL);
  /* an index built earlier for the same genome (the stamp file) is reused:
     bwa_idx_build takes ~50 s at chr21 size */
  char have[64] = {0};
  FILE *sf = fopen(stamp, "r");
  if (sf) { if (!fgets(have, sizeof have, sf)) have[0] = 0; fclose(sf); }
  if (strcmp(have, want) != 0) {
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
    remove(fa); /* the index files are all bwa_idx_load reads */
    sf = fopen(stamp, "w");
    if (sf) { fputs(want, sf); fclose(sf); }
  }
  if (is_index) { free(g); return 0; }
  bwaidx_t *idx = bwa_idx_load(fa, BWA_IDX_ALL);
  if (!idx) { fprintf(stderr, "index load failed\n"); return 1; }
  { /* every mode starts with the index's pages resident (outside the timed part) */
    volatile uint64_t sink = 0;
    const uint8_t *parts[3] = {(const uint8_t *)idx->bwt->bwt, (const uint8_t *)idx->bwt->sa, idx->pac};
    const size_t lens[3] = {idx->bwt->bwt_size * 4, (size_t)idx->bwt->n_sa * 8, (size_t)(idx->bns->l_pac / 4 + 1)};
    for (int k = 0; k < 3; ++k)
      for (size_t o = 0; o < lens[k]; o += 4096) sink += parts[k][o];
    (void)sink;
  }

  rng_s = seed;
  int n_all;
  bseq1_t *all = simulate(g, G_len, ctg_len, n_pairs, lm, &n_all);
  free(g);

  mem_opt_t *opt = mem_opt_init();
  opt->flag |= MEM_F_PE;
  opt->n_threads = T;

  bwagpu_ctx_t *ctx = 0;
  if (is_gpu) {
    bwagpu_opt_t go;
    memset(&go, 0, sizeof go);
    go.a = opt->a; go.b = opt->b; go.o_del = opt->o_del; go.e_del = opt->e_del; go.o_ins = opt->o_ins;
    go.e_ins = opt->e_ins; go.pen_clip5 = opt->pen_clip5; go.pen_clip3 = opt->pen_clip3; go.w = opt->w;
    go.zdrop = opt->zdrop;
    memcpy(go.mat, opt->mat, 25);
    const bntseq_t *bns = idx->bns;
    int64_t *ao = (int64_t *)malloc(8 * bns->n_seqs);
    int32_t *al = (int32_t *)malloc(4 * bns->n_seqs);
    for (int i = 0; i < bns->n_seqs; ++i) { ao[i] = bns->anns[i].offset; al[i] = bns->anns[i].len; }
    bwagpu_bns_t gb = {bns->l_pac, bns->n_seqs, 0, ao, al};
    const int rc = G.create(0, &go, &gb, idx->pac, &ctx);
    if (rc) { fprintf(stderr, "bwagpu_create: rc=%d\n", rc); return 3; }
  }
  if (is_seed) {
    const bwt_t *bt = idx->bwt;
    bwagpu_bwt_t gb = {bt->primary, {bt->L2[0], bt->L2[1], bt->L2[2], bt->L2[3], bt->L2[4]}, bt->seq_len,
                       bt->bwt_size, bt->bwt, bt->sa_intv, 0, bt->n_sa, bt->sa};
    if (G.set_bwt(ctx, &gb)) { fprintf(stderr, "bwagpu_set_bwt: %s\n", G.last_error(ctx)); return 3; }
    if (is_chain) {
      uint8_t *alt = (uint8_t *)calloc(idx->bns->n_seqs, 1);
      int any = 0;
      for (int i = 0; i < idx->bns->n_seqs; ++i) any |= alt[i] = (uint8_t)!!idx->bns->anns[i].is_alt;
      if (G.set_alt(ctx, any ? alt : 0)) { fprintf(stderr, "bwagpu_set_alt: %s\n", G.last_error(ctx)); return 3; }
      free(alt);
    }
  }
  bwagpu_samcache_t *caches[2] = {0, 0};
  clearer_t clr[2];
  memset(clr, 0, sizeof clr);
  /* gpuchain: the SAM cache on a context of its own (the feeder thread's
     records run on ctx meanwhile) */
  bwagpu_ctx_t *ctx_sam = ctx;
  if (is_chain) {
    bwagpu_opt_t go;
    memset(&go, 0, sizeof go);
    go.a = opt->a; go.b = opt->b; go.o_del = opt->o_del; go.e_del = opt->e_del; go.o_ins = opt->o_ins;
    go.e_ins = opt->e_ins; go.pen_clip5 = opt->pen_clip5; go.pen_clip3 = opt->pen_clip3; go.w = opt->w;
    go.zdrop = opt->zdrop;
    memcpy(go.mat, opt->mat, 25);
    const bntseq_t *bns = idx->bns;
    int64_t *ao = (int64_t *)malloc(8 * bns->n_seqs);
    int32_t *al = (int32_t *)malloc(4 * bns->n_seqs);
    for (int i = 0; i < bns->n_seqs; ++i) { ao[i] = bns->anns[i].offset; al[i] = bns->anns[i].len; }
    bwagpu_bns_t gb = {bns->l_pac, bns->n_seqs, 0, ao, al};
    if (G.create(0, &go, &gb, idx->pac, &ctx_sam)) { fprintf(stderr, "bwagpu_create (SAM context) failed\n"); return 3; }
  }
  /* first-launch capacities sized for short reads (2x150: a handful of CIGAR
     ops, MD well under 128 bytes); the rare longer ones are re-run with room */
  for (int k = 0; k < 2 && is_sam; ++k)
    if (G.sc_create(ctx_sam, 16, 128, &caches[k])) { fprintf(stderr, "bwagpu_samcache_create failed\n"); return 3; }
  int64_t n_passes = 0;

  FILE *out = fopen(outp, "w");
  if (!out) { perror(outp); return 1; }
  {
    int fd_save = dup(fileno(stdout));
    fflush(stdout);
    dup2(fileno(out), fileno(stdout));
    bwa_print_sam_hdr(idx->bns, 0);
    fflush(stdout);
    dup2(fd_save, fileno(stdout));
    close(fd_save);
  }
  double t_seed = 0, t_seed_dev = 0, t_ext = 0, t_sam = 0, t_flush = 0, t_post = 0, t_out = 0, t0, t_all = realtime();
  int64_t n_processed = 0;
  writer_t wr = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, out, 0, 0, 0, 0};
  pthread_t wth;
  pthread_create(&wth, 0, writer_main, &wr);
  /* the batches: reads until >= K bases, an even count (getKseqBatch / bseq_read) */
  int n_jobs = 0;
  feed_job_t *jobs = (feed_job_t *)calloc(n_all + 1, sizeof(feed_job_t));
  for (int r0 = 0; r0 < n_all;) {
    int r1 = r0;
    int64_t bases = 0;
    while (r1 < n_all && bases < K) bases += all[r1++].l_seq;
    if ((r1 - r0) & 1) ++r1;
    jobs[n_jobs].r0 = r0;
    jobs[n_jobs++].n = r1 - r0;
    r0 = r1;
  }
  feeder_t fd = {PTHREAD_MUTEX_INITIALIZER, PTHREAD_COND_INITIALIZER, jobs, n_jobs, 0, 0, ctx, opt, idx, all,
                 T / 4 > 2 ? T / 4 : 2, 0, 0};
  pthread_t fth;
  if (is_chain) pthread_create(&fth, 0, feeder_main, &fd);
  for (int b = 0; b < n_jobs; ++b) {
    const int r0 = jobs[b].r0, n = jobs[b].n;
    bseq1_t *seqs = all + r0;
    if (is_chain) {
      /* the feeder ran SeqsToChains + ChainsToRegions of this record */
      t0 = realtime();
      hw_t *wp = feeder_take(&fd, b);
      t_seed += realtime() - t0; /* the main thread's wait for the device stage */
      hw_t w = *wp;
      free(wp);
      t0 = realtime();
      kt_for(T, w_free_chains, &w, n);
      kt_for(T, w_post, &w, n);
      t_post += realtime() - t0;
      mem_pestat_t pes[4];
      const double tq = realtime();
      mem_pestat(opt, idx->bns->l_pac, n, w.regs, pes);
      g_t_pestat += realtime() - tq;
      w.pes = pes;
      clearer_join(&clr[b & 1]);
      sam_passes(caches[b & 1], &w, n, T, &n_passes, &t_flush);
      clearer_start(&clr[b & 1], caches[b & 1], w.regs, n);
      t_sam += realtime() - t0;
      free(w.chn);
      feeder_done(&fd);
    } else if (is_ref) {
      t0 = realtime();
      mem_process_seqs(opt, idx->bwt, idx->bns, idx->pac, n_processed, n, seqs, 0);
      t_ext += realtime() - t0;
    } else {
      hw_t w = {opt, idx, seqs, (chain_v *)calloc(n, sizeof(chain_v)), (mem_alnreg_v *)calloc(n, sizeof(mem_alnreg_v)),
                0, n_processed};
      t0 = realtime();
      if (is_seed) seed_gpu(ctx, &w, n, T, &t_seed_dev);
      else kt_for(T, w_seed, &w, n);
      t_seed += realtime() - t0;
      t0 = realtime();
      if (is_gpu) ext_gpu(ctx, &w, n, T);
      else kt_for(T, w_ext_cpu, &w, n);
      t_ext += realtime() - t0;
      t0 = realtime();
      kt_for(T, w_free_chains, &w, n);
      kt_for(T, w_post, &w, n);
      t_post += realtime() - t0;
      mem_pestat_t pes[4];
      const double tq = realtime();
      mem_pestat(opt, idx->bns->l_pac, n, w.regs, pes);
      g_t_pestat += realtime() - tq;
      w.pes = pes;
      if (is_sam) {
        clearer_join(&clr[b & 1]);
        sam_passes(caches[b & 1], &w, n, T, &n_passes, &t_flush);
        clearer_start(&clr[b & 1], caches[b & 1], w.regs, n);
      } else {
        kt_for(T, w_sam, &w, n >> 1);
        free(w.regs);
      }
      t_sam += realtime() - t0;
      free(w.chn);
    }
    const double t_o = realtime();
    writer_put(&wr, seqs, n); /* waits for the previous batch's output */
    t_out += realtime() - t_o;
    n_processed += n;
  }
  if (is_chain) {
    pthread_join(fth, 0);
    t_seed_dev = fd.t_dev;
  }
  free(jobs);
  {
    const double t_o = realtime();
    writer_wait(&wr);
    pthread_mutex_lock(&wr.mu);
    wr.stop = 1;
    pthread_cond_broadcast(&wr.cv);
    pthread_mutex_unlock(&wr.mu);
    pthread_join(wth, 0);
    t_out += realtime() - t_o;
  }
  fclose(out);
  t_all = realtime() - t_all;
  int64_t st[8] = {0};
  clearer_join(&clr[0]);
  clearer_join(&clr[1]);
  for (int k = 0; k < 2; ++k)
    if (caches[k]) {
      int64_t s2[8];
      G.sc_stats(caches[k], s2);
      for (int i = 0; i < 8; ++i) st[i] += s2[i];
    }
  fprintf(stderr, "{\"mode\": \"%s\", \"reads\": %ld, \"threads\": %d, \"seed_s\": %.4f, \"ext_s\": %.4f, "
                  "\"sam_s\": %.4f, \"flush_s\": %.4f, \"sam_passes\": %ld, \"align2_calls\": %ld, "
                  "\"reg2aln_calls\": %ld, \"seed_device_s\": %.4f, \"post_s\": %.4f, \"out_s\": %.4f, \"ext_flat_s\": %.4f, "
                  "\"ext_call_s\": %.4f, \"ext_unflat_s\": %.4f, \"pass0_s\": %.4f, \"pass1_s\": %.4f, \"pass2_s\": %.4f, "
                  "\"clear_s\": %.4f, \"pestat_s\": %.4f, \"feeder_s\": %.4f, \"total_s\": %.4f}\n",
          mode, (long)n_processed, T, t_seed, t_ext, t_sam, t_flush, (long)n_passes, (long)st[4], (long)st[5],
          t_seed_dev, t_post, t_out, g_t_flat, g_t_call, g_t_unflat, g_t_pass[0], g_t_pass[1], g_t_pass[2], g_t_clear, g_t_pestat, fd.t_busy, t_all);
  for (int k = 0; k < 2; ++k)
    if (caches[k]) G.sc_destroy(caches[k]);
  if (ctx_sam && ctx_sam != ctx) G.destroy(ctx_sam);
  if (ctx) G.destroy(ctx);
  free(all);
  free(opt);
  bwa_idx_destroy(idx);
  return 0;
}
