/*
 * ref_shim.c — TEST INFRASTRUCTURE ONLY.
 *
 * Batch shim over the REFERENCE's own mem_chain2aln / ksw_extend2, compiled
 * from /root/reference/bwa (see Makefile: _ref/libbwaref.so).  It exposes the
 * same flattened-batch signature as oracle_chain2aln_batch so that tests can
 * check the restatement (liboracle.so) and the GPU path against the real
 * reference, and bench.py can time the reference on the host as the
 * cpu_baseline ("kind": "reference").
 *
 * Per read it does exactly what ChainsToRegions::compute does
 * (src/Pipeline.cpp:511-530): kv_init the read's mem_alnreg_v and call
 * mem_chain2aln for each of its chains in order.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bntseq.h"
#include "bwamem.h"
#include "ksw.h"
#include "kvec.h"
#include "bwagpu.h"

/* mem_chain_t / mem_chain_v are private to bwamem.c (bwamem.c:180-188);
   this is the same declaration bwa-flow makes in src/bwa_wrapper.h:68-80 */
typedef struct {
  int n, m, first, rid;
  uint32_t w : 29, kept : 2, is_alt : 1;
  float frac_rep;
  int64_t pos;
  bwagpu_seed_t *seeds; /* layout-identical to mem_seed_t */
} ref_chain_t;

void mem_chain2aln(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                   const uint8_t *query, const ref_chain_t *c, mem_alnreg_v *av);

int ref_abi_check(void) { return (int)(sizeof(mem_alnreg_t) * 1000 + sizeof(bwagpu_seed_t)); }

static void fill_opt(const bwagpu_opt_t *o, mem_opt_t *mo)
{
  mem_opt_t *d = mem_opt_init();
  *mo = *d;
  free(d);
  mo->a = o->a; mo->b = o->b;
  mo->o_del = o->o_del; mo->e_del = o->e_del;
  mo->o_ins = o->o_ins; mo->e_ins = o->e_ins;
  mo->pen_clip5 = o->pen_clip5; mo->pen_clip3 = o->pen_clip3;
  mo->w = o->w; mo->zdrop = o->zdrop;
  memcpy(mo->mat, o->mat, 25);
}

typedef struct {
  const mem_opt_t *opt;
  const bntseq_t *bns;
  const uint8_t *pac;
  const bwagpu_batch_t *b;
  bwagpu_alnreg_t *out;
  int32_t *out_n;
  int r0, r1;
} rjob_t;

static void *rjob(void *arg)
{
  rjob_t *J = (rjob_t *)arg;
  const bwagpu_batch_t *b = J->b;
  for (int r = J->r0; r < J->r1; ++r) {
    mem_alnreg_v av;
    int c0 = b->read_chain_off[r], c1 = b->read_chain_off[r + 1];
    int lq = (int)(b->seq_off[r + 1] - b->seq_off[r]);
    kv_init(av);
    for (int c = c0; c < c1; ++c) {
      ref_chain_t ch;
      memset(&ch, 0, sizeof(ch));
      ch.n = ch.m = b->chain_seed_off[c + 1] - b->chain_seed_off[c];
      ch.rid = b->chain_rid[c];
      ch.frac_rep = b->chain_frac_rep[c];
      ch.seeds = (bwagpu_seed_t *)(b->seeds + b->chain_seed_off[c]);
      mem_chain2aln(J->opt, J->bns, J->pac, lq, b->seq + b->seq_off[r], &ch, &av);
    }
    memcpy(J->out + b->chain_seed_off[c0], av.a, av.n * sizeof(mem_alnreg_t));
    J->out_n[r] = (int32_t)av.n;
    free(av.a);
  }
  return 0;
}

int ref_chain2aln_batch(const bwagpu_opt_t *o, const bwagpu_bns_t *gb, const uint8_t *pac,
                        const bwagpu_batch_t *batch, bwagpu_alnreg_t *out_regs, int32_t *out_n,
                        int n_threads)
{
  mem_opt_t opt;
  bntseq_t bns;
  bntann1_t *anns;
  int nt = n_threads < 1 ? 1 : n_threads;
  rjob_t *jobs;
  pthread_t *th;

  fill_opt(o, &opt);
  memset(&bns, 0, sizeof(bns));
  bns.l_pac = gb->l_pac;
  bns.n_seqs = gb->n_seqs;
  anns = (bntann1_t *)calloc((size_t)gb->n_seqs, sizeof(bntann1_t));
  for (int i = 0; i < gb->n_seqs; ++i) {
    anns[i].offset = gb->ann_offset[i];
    anns[i].len = gb->ann_len[i];
    anns[i].name = (char *)"ref";
  }
  bns.anns = anns;

  if (nt > batch->n_reads) nt = batch->n_reads > 0 ? batch->n_reads : 1;
  jobs = (rjob_t *)calloc((size_t)nt, sizeof(rjob_t));
  th = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
  for (int t = 0; t < nt; ++t) {
    jobs[t].opt = &opt; jobs[t].bns = &bns; jobs[t].pac = pac; jobs[t].b = batch;
    jobs[t].out = out_regs; jobs[t].out_n = out_n;
    jobs[t].r0 = (int)((int64_t)batch->n_reads * t / nt);
    jobs[t].r1 = (int)((int64_t)batch->n_reads * (t + 1) / nt);
  }
  if (nt == 1) rjob(&jobs[0]);
  else {
    for (int t = 0; t < nt; ++t) pthread_create(&th[t], 0, rjob, &jobs[t]);
    for (int t = 0; t < nt; ++t) pthread_join(th[t], 0);
  }
  free(jobs);
  free(th);
  free(anns);
  return 0;
}

int ref_extend_batch(const bwagpu_opt_t *o, int32_t n_tasks, const bwagpu_ext_task_t *tasks,
                     const uint8_t *qpool, const uint8_t *tpool, bwagpu_ext_result_t *results)
{
  for (int32_t k = 0; k < n_tasks; ++k) {
    const bwagpu_ext_task_t *t = &tasks[k];
    bwagpu_ext_result_t *r = &results[k];
    r->score = ksw_extend2(t->qlen, qpool + t->qoff, t->tlen, tpool + t->toff, 5, o->mat, o->o_del,
                           o->e_del, o->o_ins, o->e_ins, t->w, t->end_bonus, t->zdrop, t->h0,
                           &r->qle, &r->tle, &r->gtle, &r->gscore, &r->max_off);
  }
  return 0;
}

/* mate-rescue local SW: the reference ksw_align2 per task (m = 5, opt->mat,
   qry = 0 as mem_matesw passes, bwamem_pair.c:151).  ksw_align2 reverses the
   query/target prefixes in place for XSTART, so work on copies. */
int ref_align2_batch(const bwagpu_opt_t *o, int32_t n_tasks, const bwagpu_align2_task_t *tasks,
                     const uint8_t *qpool, const uint8_t *tpool, bwagpu_kswr_t *results)
{
  for (int32_t k = 0; k < n_tasks; ++k) {
    const bwagpu_align2_task_t *t = &tasks[k];
    uint8_t *q = (uint8_t *)malloc((size_t)t->qlen + 1), *r = (uint8_t *)malloc((size_t)t->tlen + 1);
    kswr_t a;
    memcpy(q, qpool + t->qoff, (size_t)t->qlen);
    memcpy(r, tpool + t->toff, (size_t)t->tlen);
    a = ksw_align2(t->qlen, q, t->tlen, r, 5, o->mat, o->o_del, o->e_del, o->o_ins, o->e_ins, t->xtra, 0);
    results[k].score = a.score; results[k].te = a.te; results[k].qe = a.qe;
    results[k].score2 = a.score2; results[k].te2 = a.te2; results[k].tb = a.tb; results[k].qb = a.qb;
    free(q);
    free(r);
  }
  return 0;
}

/* the reference mem_reg2aln per job (bwa/bwamem.c:1104-1174) — its CIGAR (with
   clips), MD, NM, strand, contig and position; ar->rid is set to the contig
   of the region's first base so that mem_reg2aln's assert(a.rid == ar->rid)
   holds for jobs inside one contig */
int ref_reg2aln_batch(const bwagpu_opt_t *o, const bwagpu_bns_t *gb, const uint8_t *pac, int32_t n,
                      const bwagpu_reg2aln_task_t *tasks, const uint8_t *qpool, int max_ops, int max_md,
                      bwagpu_aln_t *out, uint32_t *cigar, char *md)
{
  mem_opt_t opt;
  bntseq_t bns;
  fill_opt(o, &opt);
  memset(&bns, 0, sizeof(bns));
  bns.l_pac = gb->l_pac;
  bns.n_seqs = gb->n_seqs;
  bns.anns = (bntann1_t *)calloc((size_t)gb->n_seqs, sizeof(bntann1_t));
  for (int i = 0; i < gb->n_seqs; ++i) {
    bns.anns[i].offset = gb->ann_offset[i];
    bns.anns[i].len = gb->ann_len[i];
    bns.anns[i].name = (char *)"ref";
  }
  for (int32_t k = 0; k < n; ++k) {
    const bwagpu_reg2aln_task_t *t = &tasks[k];
    mem_alnreg_t ar;
    int is_rev;
    memset(&ar, 0, sizeof(ar));
    ar.rb = t->rb; ar.re = t->re; ar.qb = t->qb; ar.qe = t->qe;
    ar.truesc = ar.score = t->truesc; ar.w = t->w;
    ar.rid = t->rb >= 0 ? bns_pos2rid(&bns, bns_depos(&bns, t->rb < bns.l_pac ? t->rb : t->re - 1, &is_rev)) : -1;
    mem_aln_t a = mem_reg2aln(&opt, &bns, pac, t->l_seq, (const char *)(qpool + t->qoff), &ar);
    bwagpu_aln_t *r = &out[k];
    memset(r, 0, sizeof(*r));
    r->pos = a.pos; r->rid = a.rid; r->is_rev = a.is_rev; r->NM = a.NM;
    if (a.rid < 0) {
      r->status = BWAGPU_ALN_UNMAPPED;
      continue;
    }
    const char *m = (const char *)(a.cigar + a.n_cigar);
    const int ml = (int)strlen(m);
    if (a.n_cigar > max_ops || ml + 1 > max_md) {
      r->status = BWAGPU_ALN_OVERFLOW;
    } else {
      r->n_cigar = a.n_cigar;
      r->md_len = ml;
      memcpy(cigar + (size_t)k * max_ops, a.cigar, 4 * (size_t)a.n_cigar);
      memcpy(md + (size_t)k * max_md, m, (size_t)ml + 1);
    }
    free(a.cigar);
  }
  free(bns.anns);
  return 0;
}

/* ---- seeding on the host with the reference's own code (cpu baselines of
   bench.py's seeding_stage / chaining_stage legs) ----
   mode 0: the interval search alone — mem_collect_intv's control flow
   (bwamem.c:120-167, static in the reference build, so restated here as in
   oracle/gen_seed.c) around the reference's bwt_smem1 / bwt_seed_strategy1 /
   ks_introsort_mem_intv; mode 1: bwa-flow's SeqsToChains
   (src/bwa_wrapper.cpp:105-115): the reference's mem_chain -> mem_chain_flt ->
   mem_flt_chained_seeds.  Reads are handed out in chunks of 64 to n_threads
   pthreads; the index is loaded once per prefix (bwa_idx_load). */
#include <sys/time.h>
#include "bwa.h"
#include "bwt.h"

typedef struct { size_t n, m; ref_chain_t *a; } ref_chain_v;
ref_chain_v mem_chain(const mem_opt_t *opt, const bwt_t *bwt, const bntseq_t *bns, int len, const uint8_t *seq,
                      void *buf);
int mem_chain_flt(const mem_opt_t *opt, int n_chn, ref_chain_t *a);
void mem_flt_chained_seeds(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query,
                           const uint8_t *query, int n_chn, ref_chain_t *a);
void ks_introsort_mem_intv(size_t n, bwtintv_t a[]); /* bwamem.c:90-91 */

static char g_prefix[4096];
static bwaidx_t *g_idx;

static int collect_count(const mem_opt_t *opt, const bwt_t *bwt, int len, const uint8_t *seq, bwtintv_v *mem,
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
  return (int)mem->n;
}

typedef struct {
  const mem_opt_t *opt;
  int mode;
  int32_t n_reads;
  const int64_t *seq_off;
  const uint8_t *seq;
  volatile int next;
  pthread_mutex_t mu;
  int64_t count;
  ref_chain_v *keep; /* mode 2: every read's chains, kept for the caller */
} sjob_t;

static void *sworker(void *arg)
{
  sjob_t *j = (sjob_t *)arg;
  bwtintv_v mem = {0, 0, 0}, mem1 = {0, 0, 0}, t0 = {0, 0, 0}, t1 = {0, 0, 0}, *tmpv[2] = {&t0, &t1};
  int64_t cnt = 0;
  uint8_t *q = (uint8_t *)malloc(8192);
  for (;;) {
    pthread_mutex_lock(&j->mu);
    const int r0 = j->next;
    j->next = r0 + 64;
    pthread_mutex_unlock(&j->mu);
    if (r0 >= j->n_reads) break;
    const int r1 = r0 + 64 < j->n_reads ? r0 + 64 : j->n_reads;
    for (int r = r0; r < r1; ++r) {
      const int len = (int)(j->seq_off[r + 1] - j->seq_off[r]);
      memcpy(q, j->seq + j->seq_off[r], len); /* mem_chain takes a writable copy of the read in bwa-flow too */
      if (j->mode == 0) {
        cnt += collect_count(j->opt, g_idx->bwt, len, q, &mem, &mem1, tmpv);
      } else {
        ref_chain_v c = mem_chain(j->opt, g_idx->bwt, g_idx->bns, len, q, 0);
        c.n = mem_chain_flt(j->opt, (int)c.n, c.a);
        mem_flt_chained_seeds(j->opt, g_idx->bns, g_idx->pac, len, q, (int)c.n, c.a);
        cnt += (int64_t)c.n;
        if (j->mode == 2) {
          j->keep[r] = c;
          continue;
        }
        for (size_t k = 0; k < c.n; ++k) free(c.a[k].seeds);
        free(c.a);
      }
    }
  }
  free(q);
  free(mem.a); free(mem1.a); free(t0.a); free(t1.a);
  pthread_mutex_lock(&j->mu);
  j->count += cnt;
  pthread_mutex_unlock(&j->mu);
  return 0;
}

static int load_index(const char *prefix)
{
  if (!g_idx || strcmp(prefix, g_prefix) != 0) {
    if (g_idx) bwa_idx_destroy(g_idx);
    bwa_verbose = 1;
    g_idx = bwa_idx_load(prefix, BWA_IDX_ALL);
    if (!g_idx) return -1;
    snprintf(g_prefix, sizeof g_prefix, "%s", prefix);
  }
  return 0;
}

double ref_seeding_bench(const char *prefix, int mode, int32_t n_reads, const int64_t *seq_off, const uint8_t *seq,
                         int n_threads, int reps, int64_t *out_count)
{
  if (load_index(prefix) < 0) return -1.0;
  mem_opt_t *opt = mem_opt_init();
  struct timeval a, b;
  gettimeofday(&a, 0);
  int64_t count = 0;
  for (int rep = 0; rep < reps; ++rep) {
    sjob_t j = {opt, mode == 2 ? 1 : mode, n_reads, seq_off, seq, 0, PTHREAD_MUTEX_INITIALIZER, 0, 0};
    pthread_t th[256];
    const int nt = n_threads < 1 ? 1 : n_threads > 256 ? 256 : n_threads;
    for (int t = 0; t < nt; ++t) pthread_create(&th[t], 0, sworker, &j);
    for (int t = 0; t < nt; ++t) pthread_join(th[t], 0);
    count = j.count;
  }
  gettimeofday(&b, 0);
  free(opt);
  if (out_count) *out_count = count;
  return (b.tv_sec - a.tv_sec) + 1e-6 * (b.tv_usec - a.tv_usec);
}

/* The reference's SeqsToChains (mem_chain -> mem_chain_flt ->
   mem_flt_chained_seeds, src/bwa_wrapper.cpp:105-115, default mem_opt_t) over
   a batch of reads on n_threads, its chains flattened in read order into the
   bwagpu_batch_t layout (chain_rid / chain_frac_rep / chain_seed_off / seeds).
   The checker of bench.py's C2 stream, whose chains the device makes
   (bwagpu_seqs2chains).  Returns 0; -1 when the index does not load; -2 when
   cap_chains / cap_seeds are too small (*n_chains / *n_seeds: what is needed). */
int ref_seqs2chains_batch(const char *prefix, int32_t n_reads, const int64_t *seq_off, const uint8_t *seq,
                          int n_threads, int32_t *read_chain_off, int64_t cap_chains, int32_t *chain_rid,
                          float *chain_frac_rep, int32_t *chain_seed_off, int64_t cap_seeds, bwagpu_seed_t *seeds,
                          int64_t *n_chains, int64_t *n_seeds)
{
  if (load_index(prefix) < 0) return -1;
  mem_opt_t *opt = mem_opt_init();
  ref_chain_v *keep = (ref_chain_v *)calloc(n_reads > 0 ? n_reads : 1, sizeof(ref_chain_v));
  sjob_t j = {opt, 2, n_reads, seq_off, seq, 0, PTHREAD_MUTEX_INITIALIZER, 0, keep};
  pthread_t th[256];
  const int nt = n_threads < 1 ? 1 : n_threads > 256 ? 256 : n_threads;
  for (int t = 0; t < nt; ++t) pthread_create(&th[t], 0, sworker, &j);
  for (int t = 0; t < nt; ++t) pthread_join(th[t], 0);
  int64_t nc = 0, ns = 0;
  for (int32_t r = 0; r < n_reads; ++r) {
    nc += (int64_t)keep[r].n;
    for (size_t k = 0; k < keep[r].n; ++k) ns += keep[r].a[k].n;
  }
  int rc = 0;
  if (nc > cap_chains || ns > cap_seeds) {
    rc = -2;
  } else {
    int64_t c = 0, s = 0;
    read_chain_off[0] = 0;
    chain_seed_off[0] = 0;
    for (int32_t r = 0; r < n_reads; ++r) {
      for (size_t k = 0; k < keep[r].n; ++k, ++c) {
        const ref_chain_t *ch = &keep[r].a[k];
        chain_rid[c] = ch->rid;
        chain_frac_rep[c] = ch->frac_rep;
        memcpy(seeds + s, ch->seeds, sizeof(bwagpu_seed_t) * (size_t)ch->n);
        for (int i = 0; i < ch->n; ++i) seeds[s + i].pad_ = 0;
        s += ch->n;
        chain_seed_off[c + 1] = (int32_t)s;
      }
      read_chain_off[r + 1] = (int32_t)c;
    }
  }
  for (int32_t r = 0; r < n_reads; ++r) {
    for (size_t k = 0; k < keep[r].n; ++k) free(keep[r].a[k].seeds);
    free(keep[r].a);
  }
  free(keep);
  free(opt);
  *n_chains = nc;
  *n_seeds = ns;
  return rc;
}
