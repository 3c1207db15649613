/*
 * chain2aln.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Clean-room restatement of the per-read work of the ChainsToRegions stage
 * (src/Pipeline.cpp:503-544): every chain of a read goes through
 * mem_chain2aln (bwa/bwamem.c:641-795), appending regions to that read's
 * region vector.  Also restates the reference-window fetch
 * bns_fetch_seq/bns_get_seq (bwa/bntseq.c:398-446) on bwa's forward-strand
 * 2-bit pac (bntseq.c:225, MSB-first within a byte).
 */
#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define BAND_TRIES 2 /* MAX_BAND_TRY, bwamem.c:639 */

static inline int64_t lmin(int64_t a, int64_t b) { return a < b ? a : b; }
static inline int64_t lmax(int64_t a, int64_t b) { return a > b ? a : b; }

/* cal_max_gap, bwamem.c:630-637 */
static int max_gap_len(const bwagpu_opt_t *o, int qlen)
{
  int ld = (int)((double)(qlen * o->a - o->o_del) / o->e_del + 1.);
  int li = (int)((double)(qlen * o->a - o->o_ins) / o->e_ins + 1.);
  int l = ld > li ? ld : li;
  if (l < 1) l = 1;
  return l < (o->w << 1) ? l : (o->w << 1);
}

int oracle_max_gap_len(const bwagpu_opt_t *o, int qlen) { return max_gap_len(o, qlen); }

static inline int pac_base(const uint8_t *pac, int64_t k) { return pac[k >> 2] >> ((~k & 3) << 1) & 3; }

/* materialise [beg,end) of the 2-strand coordinate space (bns_get_seq) */
static void get_window(int64_t l_pac, const uint8_t *pac, int64_t beg, int64_t end, uint8_t *out)
{
  if (beg >= l_pac) { /* reverse strand: complement of the reversed forward */
    for (int64_t k = beg; k < end; ++k) out[k - beg] = 3 - pac_base(pac, (l_pac << 1) - 1 - k);
  } else {
    for (int64_t k = beg; k < end; ++k) out[k - beg] = pac_base(pac, k);
  }
}

void oracle_get_window(int64_t l_pac, const uint8_t *pac, int64_t beg, int64_t end, uint8_t *out)
{
  get_window(l_pac, pac, beg, end, out);
}

static int cmp_u64(const void *a, const void *b)
{
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return x < y ? -1 : x > y;
}

typedef struct {
  int64_t cells[2];
  int64_t calls;
} tally_t;
#define tl_cells(t) ((t)->cells)

/* One seed's extension, bwamem.c:717-792: the left ksw_extend2 over the
   reversed query prefix and reversed window prefix with the MAX_BAND_TRY
   retry, the right one from the left score, the local vs to-end choice of each
   side.  win = the window [lo, hi); qrev/trev = scratch of lq / hi - lo bytes.
   Fills w, score, truesc, qb, qe, rb, re of *a (nothing else). */
void oracle_seed_extend(const bwagpu_opt_t *opt, int lq, const uint8_t *q, const bwagpu_seed_t *s, int64_t lo,
                        int64_t hi, const uint8_t *win, uint8_t *qrev, uint8_t *trev, bwagpu_alnreg_t *a,
                        int64_t *cells, int64_t *calls)
{
  int aw0 = opt->w, aw1 = opt->w, mo, i;
  a->w = opt->w;
  a->score = a->truesc = -1;

  if (s->qbeg) { /* leftwards: reversed query prefix against reversed window prefix */
    int qle = 0, tle = 0, gtle = 0, gsc = 0;
    int64_t ltl = s->rbeg - lo;
    for (i = 0; i < s->qbeg; ++i) qrev[i] = q[s->qbeg - 1 - i];
    for (i = 0; i < ltl; ++i) trev[i] = win[ltl - 1 - i];
    for (i = 0; i < BAND_TRIES; ++i) {
      int before = a->score;
      aw0 = opt->w << i;
      a->score = oracle_ksw_extend2(s->qbeg, qrev, (int)ltl, trev, 5, opt->mat, opt->o_del, opt->e_del,
                                    opt->o_ins, opt->e_ins, aw0, opt->pen_clip5, opt->zdrop,
                                    s->len * opt->a, &qle, &tle, &gtle, &gsc, &mo, cells);
      ++*calls;
      if (a->score == before || mo < (aw0 >> 1) + (aw0 >> 2)) break;
    }
    if (gsc <= 0 || gsc <= a->score - opt->pen_clip5) {
      a->qb = s->qbeg - qle;
      a->rb = s->rbeg - tle;
      a->truesc = a->score;
    } else {
      a->qb = 0;
      a->rb = s->rbeg - gtle;
      a->truesc = gsc;
    }
  } else {
    a->score = a->truesc = s->len * opt->a;
    a->qb = 0;
    a->rb = s->rbeg;
  }

  if (s->qbeg + s->len != lq) { /* rightwards from the seed end */
    int qle = 0, tle = 0, gtle = 0, gsc = 0, sc0 = a->score;
    int qe = s->qbeg + s->len;
    int64_t re = s->rbeg + s->len - lo;
    for (i = 0; i < BAND_TRIES; ++i) {
      int before = a->score;
      aw1 = opt->w << i;
      a->score = oracle_ksw_extend2(lq - qe, q + qe, (int)(hi - lo - re), win + re, 5, opt->mat,
                                    opt->o_del, opt->e_del, opt->o_ins, opt->e_ins, aw1,
                                    opt->pen_clip3, opt->zdrop, sc0, &qle, &tle, &gtle, &gsc, &mo,
                                    cells);
      ++*calls;
      if (a->score == before || mo < (aw1 >> 1) + (aw1 >> 2)) break;
    }
    if (gsc <= 0 || gsc <= a->score - opt->pen_clip3) {
      a->qe = qe + qle;
      a->re = lo + re + tle;
      a->truesc += a->score - sc0;
    } else {
      a->qe = lq;
      a->re = lo + re + gtle;
      a->truesc += gsc - sc0;
    }
  } else {
    a->qe = lq;
    a->re = s->rbeg + s->len;
  }
  a->w = aw0 > aw1 ? aw0 : aw1;
}

/* one chain; regs/nreg is the read's region vector (capacity = read's seeds) */
static int one_chain(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const uint8_t *pac, int lq,
                     const uint8_t *q, const bwagpu_seed_t *sd, int ns, int rid, float frac_rep,
                     bwagpu_alnreg_t *regs, int *nreg, tally_t *tl)
{
  const int64_t l_pac = bns->l_pac, two = l_pac << 1;
  int64_t lo = two, hi = 0;
  uint8_t *win, *qrev, *trev;
  uint64_t *key;
  int i, k;

  if (ns == 0) return 0;
  for (i = 0; i < ns; ++i) {
    const bwagpu_seed_t *t = &sd[i];
    int tail = lq - t->qbeg - t->len;
    lo = lmin(lo, t->rbeg - (t->qbeg + max_gap_len(opt, t->qbeg)));
    hi = lmax(hi, t->rbeg + t->len + (tail + max_gap_len(opt, tail)));
  }
  lo = lmax(lo, 0);
  hi = lmin(hi, two);
  if (lo < l_pac && l_pac < hi) { /* never straddle the strand boundary */
    if (sd[0].rbeg < l_pac) hi = l_pac;
    else lo = l_pac;
  }
  { /* clip to the contig holding the first seed (bns_fetch_seq) */
    int64_t mid = sd[0].rbeg, fpos = mid >= l_pac ? two - 1 - mid : mid, cb, ce;
    if (rid < 0 || rid >= bns->n_seqs) return -2;
    cb = bns->ann_offset[rid];
    ce = cb + bns->ann_len[rid];
    if (fpos < cb || fpos >= ce) return -2; /* reference: assert(c->rid == rid) */
    if (mid >= l_pac) { int64_t t0 = cb; cb = two - ce; ce = two - t0; }
    lo = lmax(lo, cb);
    hi = lmin(hi, ce);
  }
  win = (uint8_t *)malloc((size_t)(hi - lo) + 1);
  get_window(l_pac, pac, lo, hi, win);

  key = (uint64_t *)malloc((size_t)ns * sizeof(uint64_t));
  for (i = 0; i < ns; ++i) key[i] = (uint64_t)sd[i].score << 32 | (uint32_t)i;
  qsort(key, (size_t)ns, sizeof(uint64_t), cmp_u64);
  qrev = (uint8_t *)malloc((size_t)lq + 1);
  trev = (uint8_t *)malloc((size_t)(hi - lo) + 1);

  for (k = ns - 1; k >= 0; --k) {
    const bwagpu_seed_t *s = &sd[(uint32_t)key[k]];
    bwagpu_alnreg_t *a;

    /* is the seed (almost) inside a region already found for this read? */
    for (i = 0; i < *nreg; ++i) {
      const bwagpu_alnreg_t *p = &regs[i];
      int64_t rd;
      int qd, g, bw;
      if (s->rbeg < p->rb || s->rbeg + s->len > p->re || s->qbeg < p->qb || s->qbeg + s->len > p->qe)
        continue;
      if (s->len - p->seedlen0 > .1 * lq) continue;
      qd = s->qbeg - p->qb;
      rd = s->rbeg - p->rb;
      g = max_gap_len(opt, qd < rd ? qd : (int)rd);
      bw = g < p->w ? g : p->w;
      if (qd - rd < bw && rd - qd < bw) break;
      qd = p->qe - (s->qbeg + s->len);
      rd = p->re - (s->rbeg + s->len);
      g = max_gap_len(opt, qd < rd ? qd : (int)rd);
      bw = g < p->w ? g : p->w;
      if (qd - rd < bw && rd - qd < bw) break;
    }
    if (i < *nreg) { /* contained: extend only if a long overlapping seed disagrees */
      for (i = k + 1; i < ns; ++i) {
        const bwagpu_seed_t *t;
        if (key[i] == 0) continue;
        t = &sd[(uint32_t)key[i]];
        if (t->len < s->len * .95) continue;
        if (s->qbeg <= t->qbeg && s->qbeg + s->len - t->qbeg >= s->len >> 2 &&
            t->qbeg - s->qbeg != t->rbeg - s->rbeg)
          break;
        if (t->qbeg <= s->qbeg && t->qbeg + t->len - s->qbeg >= s->len >> 2 &&
            s->qbeg - t->qbeg != s->rbeg - t->rbeg)
          break;
      }
      if (i == ns) { key[k] = 0; continue; }
    }

    a = &regs[(*nreg)++];
    memset(a, 0, sizeof(*a));
    a->rid = rid;
    oracle_seed_extend(opt, lq, q, s, lo, hi, win, qrev, trev, a, tl->cells, &tl->calls);
    a->seedcov = 0;
    for (i = 0; i < ns; ++i) {
      const bwagpu_seed_t *t = &sd[i];
      if (t->qbeg >= a->qb && t->qbeg + t->len <= a->qe && t->rbeg >= a->rb && t->rbeg + t->len <= a->re)
        a->seedcov += t->len;
    }
    a->seedlen0 = s->len;
    a->frac_rep = frac_rep;
  }
  free(key);
  free(win);
  free(qrev);
  free(trev);
  return 0;
}

typedef struct {
  const bwagpu_opt_t *opt;
  const bwagpu_bns_t *bns;
  const uint8_t *pac;
  const bwagpu_batch_t *b;
  bwagpu_alnreg_t *out;
  int32_t *out_n;
  int r0, r1, err;
  tally_t tl;
} job_t;

static void *run_job(void *arg)
{
  job_t *J = (job_t *)arg;
  const bwagpu_batch_t *b = J->b;
  for (int r = J->r0; r < J->r1 && !J->err; ++r) {
    int c0 = b->read_chain_off[r], c1 = b->read_chain_off[r + 1];
    int lq = (int)(b->seq_off[r + 1] - b->seq_off[r]);
    int nreg = 0;
    bwagpu_alnreg_t *regs = J->out + b->chain_seed_off[c0];
    for (int c = c0; c < c1; ++c) {
      int s0 = b->chain_seed_off[c], s1 = b->chain_seed_off[c + 1];
      int rc = one_chain(J->opt, J->bns, J->pac, lq, b->seq + b->seq_off[r], b->seeds + s0, s1 - s0,
                         b->chain_rid[c], b->chain_frac_rep[c], regs, &nreg, &J->tl);
      if (rc) { J->err = rc; break; }
    }
    J->out_n[r] = nreg;
  }
  return 0;
}

int oracle_chain2aln_batch(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const uint8_t *pac,
                           const bwagpu_batch_t *batch, bwagpu_alnreg_t *out_regs, int32_t *out_n,
                           int n_threads, int64_t *stats)
{
  int nt = n_threads < 1 ? 1 : n_threads, err = 0;
  job_t *jobs;
  pthread_t *th;
  if (nt > batch->n_reads) nt = batch->n_reads > 0 ? batch->n_reads : 1;
  jobs = (job_t *)calloc((size_t)nt, sizeof(job_t));
  th = (pthread_t *)calloc((size_t)nt, sizeof(pthread_t));
  for (int t = 0; t < nt; ++t) {
    jobs[t].opt = opt; jobs[t].bns = bns; jobs[t].pac = pac; jobs[t].b = batch;
    jobs[t].out = out_regs; jobs[t].out_n = out_n;
    jobs[t].r0 = (int)((int64_t)batch->n_reads * t / nt);
    jobs[t].r1 = (int)((int64_t)batch->n_reads * (t + 1) / nt);
  }
  if (nt == 1) run_job(&jobs[0]);
  else {
    for (int t = 0; t < nt; ++t) pthread_create(&th[t], 0, run_job, &jobs[t]);
    for (int t = 0; t < nt; ++t) pthread_join(th[t], 0);
  }
  if (stats) stats[0] = stats[1] = stats[2] = 0;
  for (int t = 0; t < nt; ++t) {
    if (jobs[t].err && !err) err = jobs[t].err;
    if (stats) { stats[0] += jobs[t].tl.cells[0]; stats[1] += jobs[t].tl.cells[1]; stats[2] += jobs[t].tl.calls; }
  }
  free(jobs);
  free(th);
  return err;
}
