/*
 * ksw_global.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Clean-room restatement of the CIGAR step of bwa-flow's SAM stage
 * (SURVEY.md §8f rank 2): mem_reg2aln (bwa/bwamem.c:1104-1174) minus the
 * mapq/flag fields, i.e.
 *   infer_bw            bwamem.c:801-808 (band from the local score)
 *   the band loop       bwamem.c:1123-1134 (up to 3 tries, band doubling)
 *   bwa_gen_cigar2      bwa/bwa.c:121-207 (window fetch, strand flip, band
 *                       rule, ungapped shortcut, NM and the MD string)
 *   ksw_global2         bwa/ksw.c:504-606 (banded global DP + backtrack)
 *   the squeeze/clip    bwamem.c:1137-1166 and bns_depos / bns_pos2rid
 *                       (bntseq.h:87-90, bntseq.c:349-363)
 * called from src/bwa_wrapper.cpp:611/728/736/774 (mem_reg2aln per output
 * region).
 *
 * The DP keeps the reference's integer arithmetic exactly, including the
 * -0x40000000 "minus infinity" values outside the band and the per-cell
 * direction byte (h source in bits 0-1, E-extension flag in bit 2, F-extension
 * flag as the value 2 in bits 4-5), because the backtrack reads those bits
 * with a state-dependent shift.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define NEG_INF (-0x40000000)

typedef struct { uint32_t *a; int n, m; } ops_t;

static void ops_push(ops_t *c, int op, int len)
{
  if (c->n > 0 && (int)(c->a[c->n - 1] & 0xf) == op) {
    c->a[c->n - 1] += (uint32_t)len << 4;
    return;
  }
  if (c->n == c->m) {
    c->m = c->m ? c->m * 2 : 16;
    c->a = (uint32_t *)realloc(c->a, sizeof(uint32_t) * c->m);
  }
  c->a[c->n++] = (uint32_t)len << 4 | (uint32_t)op;
}

/* banded global alignment of q[0,ql) against t[0,tl) with band w; returns
   H at (tl-1, ql-1) as ksw_global2 does; the CIGAR (M=0, I=1, D=2) in *ops */
static int global2(int ql, const uint8_t *q, int tl, const uint8_t *t, const int8_t *mat, int o_del,
                   int e_del, int o_ins, int e_ins, int w, ops_t *ops)
{
  const int ncol = ql < 2 * w + 1 ? ql : 2 * w + 1;
  int *H = (int *)malloc(sizeof(int) * (ql + 1)), *E = (int *)malloc(sizeof(int) * (ql + 1));
  uint8_t *dir = (uint8_t *)malloc((size_t)ncol * (tl > 0 ? tl : 1));
  /* H[j] holds H(i-1, j-1) when row i starts (row -1: the insertion border) */
  H[0] = 0;
  E[0] = NEG_INF;
  int j = 1;
  for (; j <= ql && j <= w; ++j) H[j] = -(o_ins + e_ins * j), E[j] = NEG_INF;
  for (; j <= ql; ++j) H[j] = E[j] = NEG_INF;
  for (int i = 0; i < tl; ++i) {
    const int lo = i > w ? i - w : 0, hi = i + w + 1 < ql ? i + w + 1 : ql;
    const int8_t *srow = mat + t[i] * 5;
    int f = NEG_INF;
    int left = lo == 0 ? -(o_del + e_del * (i + 1)) : NEG_INF; /* H(i, lo-1) */
    uint8_t *drow = dir + (size_t)i * ncol;
    for (j = lo; j < hi; ++j) {
      int m = H[j] + srow[q[j]];
      int e = E[j];
      uint8_t d = m >= e ? 0 : 1;
      int h = m >= e ? m : e;
      if (!(h >= f)) d = 2, h = f;
      H[j] = left;
      left = h;
      const int od = m - (o_del + e_del), oi = m - (o_ins + e_ins);
      e -= e_del;
      if (e > od) d |= 4; else e = od;
      E[j] = e;
      f -= e_ins;
      if (f > oi) d |= 32; else f = oi;
      drow[j - lo] = d;
    }
    H[hi] = left;
    E[hi] = NEG_INF;
  }
  const int score = H[ql];
  /* backtrack from the last cell of the last row */
  int i = tl - 1, k = (i + w + 1 < ql ? i + w + 1 : ql) - 1, st = 0;
  ops->n = 0;
  while (i >= 0 && k >= 0) {
    const int lo = i > w ? i - w : 0;
    st = dir[(size_t)i * ncol + (k - lo)] >> (st << 1) & 3;
    if (st == 0) ops_push(ops, 0, 1), --i, --k;
    else if (st == 1) ops_push(ops, 2, 1), --i;
    else ops_push(ops, 1, 1), --k;
  }
  if (i >= 0) ops_push(ops, 2, i + 1);
  if (k >= 0) ops_push(ops, 1, k + 1);
  for (int a = 0, b = ops->n - 1; a < b; ++a, --b) {
    uint32_t x = ops->a[a];
    ops->a[a] = ops->a[b];
    ops->a[b] = x;
  }
  free(H);
  free(E);
  free(dir);
  return score;
}

static int base2(const uint8_t *pac, int64_t x) { return pac[x >> 2] >> ((~x & 3) << 1) & 3; }

typedef struct { char *s; int l, m; } str_t;
static void s_putc(str_t *s, char c)
{
  if (s->l + 1 >= s->m) {
    s->m = s->m ? s->m * 2 : 64;
    s->s = (char *)realloc(s->s, s->m);
  }
  s->s[s->l++] = c;
}
static void s_putw(str_t *s, int v)
{
  char b[16];
  int n = 0;
  unsigned x = v < 0 ? (unsigned)-v : (unsigned)v;
  do b[n++] = (char)('0' + x % 10), x /= 10; while (x);
  if (v < 0) s_putc(s, '-');
  while (n) s_putc(s, b[--n]);
}

/* bwa_gen_cigar2: returns 1 with a CIGAR, 0 when the reference returns none */
static int gen_cigar2(const bwagpu_opt_t *o, const int8_t *mat, int w_, int64_t l_pac, const uint8_t *pac,
                      int ql, const uint8_t *query_in, int64_t rb, int64_t re, int *score, ops_t *ops, int *NM,
                      str_t *md)
{
  ops->n = 0;
  *NM = -1;
  md->l = 0;
  if (ql <= 0 || rb >= re || (rb < l_pac && re > l_pac)) return 0;
  /* bns_get_seq: clip to [0, 2 l_pac); a window must lie on one strand */
  int64_t beg = rb < 0 ? 0 : rb, end = re > (l_pac << 1) ? (l_pac << 1) : re;
  if (!(beg >= l_pac || end <= l_pac)) return 0;
  const int64_t rlen = end - beg;
  if (rlen != re - rb) return 0;
  uint8_t *r = (uint8_t *)malloc(rlen > 0 ? rlen : 1), *q = (uint8_t *)malloc(ql);
  for (int64_t x = 0; x < rlen; ++x) {
    const int64_t p = beg + x;
    r[x] = p >= l_pac ? (uint8_t)(3 - base2(pac, (l_pac << 1) - 1 - p)) : (uint8_t)base2(pac, p);
  }
  memcpy(q, query_in, ql);
  const int rev = rb >= l_pac;
  if (rev) { /* both sequences reversed: indels end up leftmost */
    for (int a = 0, b = ql - 1; a < b; ++a, --b) { uint8_t x = q[a]; q[a] = q[b]; q[b] = x; }
    for (int64_t a = 0, b = rlen - 1; a < b; ++a, --b) { uint8_t x = r[a]; r[a] = r[b]; r[b] = x; }
  }
  if (ql == re - rb && w_ == 0) {
    ops_push(ops, 0, ql);
    int s = 0;
    for (int x = 0; x < ql; ++x) s += mat[r[x] * 5 + q[x]];
    *score = s;
  } else {
    const int half = (ql + 1) >> 1;
    int mi = (int)((double)(half * mat[0] - o->o_ins) / o->e_ins + 1.);
    int md_ = (int)((double)(half * mat[0] - o->o_del) / o->e_del + 1.);
    int mg = mi > md_ ? mi : md_;
    mg = mg > 1 ? mg : 1;
    const int dl = abs((int)rlen - ql);
    int w = (mg + dl + 1) >> 1;
    w = w < w_ ? w : w_;
    w = w > dl + 3 ? w : dl + 3;
    *score = global2(ql, q, (int)rlen, r, mat, o->o_del, o->e_del, o->o_ins, o->e_ins, w, ops);
  }
  /* NM and MD (deletions at either end of the CIGAR are not reported) */
  const char *b2c = rb < l_pac ? "ACGTN" : "TGCAN";
  int x = 0, y = 0, u = 0, n_mm = 0, n_gap = 0;
  for (int k = 0; k < ops->n; ++k) {
    const int op = ops->a[k] & 0xf, len = ops->a[k] >> 4;
    if (op == 0) {
      for (int a = 0; a < len; ++a) {
        if (q[x + a] != r[y + a]) {
          s_putw(md, u);
          s_putc(md, b2c[r[y + a]]);
          ++n_mm;
          u = 0;
        } else ++u;
      }
      x += len;
      y += len;
    } else if (op == 2) {
      if (k > 0 && k < ops->n - 1) {
        s_putw(md, u);
        s_putc(md, '^');
        for (int a = 0; a < len; ++a) s_putc(md, b2c[r[y + a]]);
        u = 0;
        n_gap += len;
      }
      y += len;
    } else if (op == 1) {
      x += len;
      n_gap += len;
    }
  }
  s_putw(md, u);
  md->s[md->l] = 0;
  *NM = n_mm + n_gap;
  free(r);
  free(q);
  return 1;
}

static int infer_bw(int l1, int l2, int score, int a, int q, int r)
{
  if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
  int w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
  if (w < abs(l1 - l2)) w = abs(l1 - l2);
  return w;
}

int oracle_reg2aln(const bwagpu_opt_t *o, const bwagpu_bns_t *bns, const uint8_t *pac, const uint8_t *read,
                   const bwagpu_reg2aln_task_t *t, int max_ops, int max_md, bwagpu_aln_t *out, uint32_t *cigar,
                   char *md_out)
{
  int8_t mat[25];
  memset(out, 0, sizeof *out);
  if (t->rb < 0 || t->re < 0) { /* unmapped record */
    out->rid = -1;
    out->pos = -1;
    out->status = BWAGPU_ALN_UNMAPPED;
    return 0;
  }
  for (int i = 0; i < 4; ++i) {
    for (int j = 0; j < 4; ++j) mat[i * 5 + j] = i == j ? o->a : -o->b;
    mat[i * 5 + 4] = -1;
  }
  for (int j = 0; j < 5; ++j) mat[20 + j] = -1;
  const int lq = t->qe - t->qb;
  const int64_t rl = t->re - t->rb;
  int w2 = infer_bw(lq, (int)rl, t->truesc, o->a, o->o_del, o->e_del);
  const int wi = infer_bw(lq, (int)rl, t->truesc, o->a, o->o_ins, o->e_ins);
  w2 = wi > w2 ? wi : w2;
  if (w2 > o->w) w2 = w2 < t->w ? w2 : t->w;
  const int wmax = o->w << 2;
  ops_t ops = {0, 0, 0};
  str_t md = {0, 0, 0};
  s_putc(&md, 0);
  md.l = 0;
  int score = 0, NM = -1, last = -(1 << 30), ok = 0, tries = 0, wcall = 0;
  do {
    w2 = w2 < wmax ? w2 : wmax;
    wcall = w2;
    ok = gen_cigar2(o, mat, w2, bns->l_pac, pac, lq, read + t->qb, t->rb, t->re, &score, &ops, &NM, &md);
    if (!ok) break;
    if (score == last || w2 == wmax) break;
    last = score;
    w2 <<= 1;
  } while (++tries < 3 && score < t->truesc - o->a);
  out->score = score;
  out->w = wcall;
  if (!ok) {
    out->status = BWAGPU_ALN_NO_CIGAR;
    out->NM = -1;
    free(ops.a);
    free(md.s);
    return 0;
  }
  out->NM = NM;
  /* bns_depos */
  int64_t pos = t->rb < bns->l_pac ? t->rb : t->re - 1;
  const int is_rev = pos >= bns->l_pac;
  if (is_rev) pos = (bns->l_pac << 1) - 1 - pos;
  int n = ops.n, s0 = 0;
  if (n > 0) {
    if ((ops.a[0] & 0xf) == 2) {
      pos += ops.a[0] >> 4;
      s0 = 1;
      --n;
    } else if ((ops.a[n - 1] & 0xf) == 2) {
      --n;
    }
  }
  int clip5 = 0, clip3 = 0;
  if (t->qb != 0 || t->qe != t->l_seq) {
    clip5 = is_rev ? t->l_seq - t->qe : t->qb;
    clip3 = is_rev ? t->qb : t->l_seq - t->qe;
  }
  const int total = n + (clip5 != 0) + (clip3 != 0);
  if (total > max_ops || md.l + 1 > max_md) {
    out->status = BWAGPU_ALN_OVERFLOW;
    free(ops.a);
    free(md.s);
    return 0;
  }
  int c = 0;
  if (clip5) cigar[c++] = (uint32_t)clip5 << 4 | 3;
  for (int k = 0; k < n; ++k) cigar[c++] = ops.a[s0 + k];
  if (clip3) cigar[c++] = (uint32_t)clip3 << 4 | 3;
  memcpy(md_out, md.s, md.l + 1);
  out->n_cigar = c;
  out->md_len = md.l;
  out->is_rev = is_rev;
  /* bns_pos2rid */
  int left = 0, mid = 0, right = bns->n_seqs;
  if (pos >= bns->l_pac) mid = -1;
  else
    while (left < right) {
      mid = (left + right) >> 1;
      if (pos >= bns->ann_offset[mid]) {
        if (mid == bns->n_seqs - 1) break;
        if (pos < bns->ann_offset[mid + 1]) break;
        left = mid + 1;
      } else right = mid;
    }
  out->rid = mid;
  out->pos = mid >= 0 ? pos - bns->ann_offset[mid] : pos;
  free(ops.a);
  free(md.s);
  return 0;
}

int oracle_reg2aln_batch(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const uint8_t *pac, int32_t n,
                         const bwagpu_reg2aln_task_t *tasks, const uint8_t *qpool, int max_ops, int max_md,
                         bwagpu_aln_t *out, uint32_t *cigar, char *md)
{
  for (int32_t k = 0; k < n; ++k)
    oracle_reg2aln(opt, bns, pac, qpool + tasks[k].qoff, &tasks[k], max_ops, max_md, &out[k],
                   cigar + (size_t)k * max_ops, md + (size_t)k * max_md);
  return 0;
}
