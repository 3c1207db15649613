/*
 * ksw_align.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Clean-room restatement of the local Smith-Waterman used by bwa's mate
 * rescue: ksw_align2 (bwa/ksw.c:337-357) over
 * ksw_u8 (ksw.c:111-232) / ksw_i16 (ksw.c:234-328) with the query profile of
 * ksw_qinit (ksw.c:69-108), as called by mem_matesw (bwa/bwamem_pair.c:150).
 *
 * The reference computes the DP with Farrar's striped layout: p = 16 (u8)
 * or 8 (i16) lanes, slen = ceil(qlen/p), column c = k*slen + j sits in lane
 * k of vector j, so lane k covers the column SEGMENT [k*slen, (k+1)*slen);
 * columns qlen .. p*slen-1 are padding with score 0.  Its results depend on
 * that segmentation in one place, restated here row by row in plain order:
 *
 *   first pass (ksw.c:146-171):  within a segment F starts at 0,
 *     h_fp(c) = max(M(c), E(c), Fseg(c)),  M(c) = H(i-1, c-1) + S(t_i, q_c)
 *     E(i+1,c) = max(E(i,c) - e_del, h_fp(c) - oe_del, 0)   <- from h_fp
 *     row max = max over all p*slen columns of h_fp
 *   lazy F (ksw.c:173-184): F continued across segments, E NOT recomputed
 *     (comment at ksw.c:172).  Restated literally below: time steps
 *     k*slen + j visit column s*slen + j of every segment s at once, F only
 *     decays, and the loop stops at the first step where every lane has
 *     f - e_ins <= H - oe_ins.  For o_ins > 0 that stop never cuts off a
 *     live F, so H(i,c) = max(h_fp(c), Ffull(c)) with Ffull the unsegmented
 *     F from h_fp (the GPU kernel's form); for o_ins == 0 it can (equality
 *     case), which is why this oracle keeps the literal loop.
 *
 * In u8 the M path saturates: max(min(H + S + shift, 255) - shift, 0).
 * Everything else (row maxima list for the 2nd best score, qe ties to the
 * smallest column, XSTOP/XSUBO/XSTART, the reverse pass for the start) is
 * restated from ksw.c:191-231 and 343-356.
 */
#include <limits.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define KSW_XBYTE 0x10000
#define KSW_XSTOP 0x20000
#define KSW_XSUBO 0x40000
#define KSW_XSTART 0x80000

static inline int imax2(int a, int b) { return a > b ? a : b; }
static inline int imin2(int a, int b) { return a < b ? a : b; }
static inline int sat0(int a) { return a > 0 ? a : 0; }

/* one striped pass (ksw_u8 when size == 1, ksw_i16 when size == 2) */
static void sw_pass(int size, int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat,
                    int o_del, int e_del, int o_ins, int e_ins, int xtra, bwagpu_kswr_t *r, int64_t *cells)
{
  const int p = size == 1 ? 16 : 8;
  const int slen = (qlen + p - 1) / p, ncol = slen * p;
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  int minsc = (xtra & KSW_XSUBO) ? (xtra & 0xffff) : 0x10000;
  int endsc = (xtra & KSW_XSTOP) ? (xtra & 0xffff) : 0x10000;
  int shift, qmax = 0, gmax = 0, te = -1, i, c;
  int *H = (int *)calloc((size_t)ncol + 1, sizeof(int));    /* H(i-1, .) */
  int *Hn = (int *)calloc((size_t)ncol + 1, sizeof(int));
  int *E = (int *)calloc((size_t)ncol + 1, sizeof(int));
  int *hfp = (int *)calloc((size_t)ncol + 1, sizeof(int));
  int *Hmax = (int *)calloc((size_t)ncol + 1, sizeof(int));
  int fexit[16], fl[16];
  uint64_t *b = 0;
  int n_b = 0, m_b = 0;
  {
    /* ksw_qinit: shift = -min(mat) as a byte, max = max(mat, 0) (ksw.c:78-86) */
    int mn = 127;
    for (i = 0; i < 25; ++i) {
      mn = imin2(mn, mat[i]);
      qmax = imax2(qmax, mat[i]);
    }
    shift = (256 - (mn & 0xff)) & 0xff;
  }
  r->score = 0; r->te = -1; r->qe = -1; r->score2 = -1; r->te2 = -1; r->tb = -1; r->qb = -1;
  for (i = 0; i < tlen; ++i) {
    const int8_t *ma = mat + target[i] * 5;
    int fseg = 0, rowmax = 0, k, j, s;
    for (c = 0; c < ncol; ++c) {
      const int sc = c < qlen ? ma[query[c]] : 0;
      const int hd = c == 0 ? 0 : H[c - 1];
      int m, h;
      if (c % slen == 0) { /* a new segment: the first pass starts F at 0 */
        if (c) fexit[c / slen - 1] = fseg;
        fseg = 0;
      }
      /* u8: the profile byte is (uint8)(score + shift), ksw.c:93 */
      if (size == 1) m = sat0(imin2(hd + (uint8_t)(sc + shift), 255) - shift);
      else m = hd + sc;
      h = imax2(imax2(m, E[c]), fseg);
      hfp[c] = h;
      rowmax = imax2(rowmax, h);
      E[c] = imax2(sat0(E[c] - e_del), sat0(h - oe_del));
      fseg = imax2(sat0(fseg - e_ins), sat0(h - oe_ins));
    }
    fexit[p - 1] = fseg;
    memcpy(Hn, hfp, sizeof(int) * (size_t)ncol);
    /* lazy F (ksw.c:173-184 / 284-294): lane s holds f; a shift moves lane
       s-1's f into lane s and zero into lane 0 */
    for (s = p - 1; s > 0; --s) fl[s] = fexit[s - 1];
    fl[0] = 0;
    for (k = 0; k < 16; ++k) {
      if (k)
        for (s = p - 1; s >= 0; --s) fl[s] = s ? fl[s - 1] : 0;
      for (j = 0; j < slen; ++j) {
        int live = 0;
        for (s = 0; s < p; ++s) {
          const int cc = s * slen + j;
          const int h = imax2(Hn[cc], fl[s]);
          Hn[cc] = h;
          fl[s] = sat0(fl[s] - e_ins);
          if (fl[s] > sat0(h - oe_ins)) live = 1;
        }
        if (!live) goto lazy_done;
      }
    }
  lazy_done:
    if (cells) { cells[0] += qlen; cells[1] += 1; }
    if (rowmax >= minsc) { /* ksw.c:191-198 */
      if (n_b == 0 || (int32_t)b[n_b - 1] + 1 != i) {
        if (n_b == m_b) {
          m_b = m_b ? m_b << 1 : 8;
          b = (uint64_t *)realloc(b, 8 * (size_t)m_b);
        }
        b[n_b++] = (uint64_t)rowmax << 32 | (uint32_t)i;
      } else if ((int)(b[n_b - 1] >> 32) < rowmax) {
        b[n_b - 1] = (uint64_t)rowmax << 32 | (uint32_t)i;
      }
    }
    { int *t = H; H = Hn; Hn = t; }
    if (rowmax > gmax) { /* ksw.c:199-204 */
      gmax = rowmax;
      te = i;
      memcpy(Hmax, H, sizeof(int) * (size_t)ncol);
      if ((size == 1 && gmax + shift >= 255) || gmax >= endsc) break;
    }
  }
  r->score = (size == 1 && gmax + shift >= 255) ? 255 : gmax;
  r->te = te;
  if (!(size == 1 && r->score == 255)) { /* ksw.c:208-227 */
    int mx = -1;
    for (c = 0; c < ncol; ++c)
      if (Hmax[c] > mx) mx = Hmax[c], r->qe = c; /* ascending c: ties keep the smallest column */
    if (b) {
      const int k = (r->score + qmax - 1) / qmax;
      const int low = te - k, high = te + k;
      for (i = 0; i < n_b; ++i) {
        const int e = (int32_t)b[i];
        if ((e < low || e > high) && (int)(b[i] >> 32) > r->score2) r->score2 = (int)(b[i] >> 32), r->te2 = e;
      }
    }
  }
  free(H); free(Hn); free(E); free(hfp); free(Hmax); free(b);
}

void oracle_ksw_align2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, const int8_t *mat, int o_del,
                       int e_del, int o_ins, int e_ins, int xtra, bwagpu_kswr_t *r, int64_t *cells)
{
  const int size = (xtra & KSW_XBYTE) ? 1 : 2;
  bwagpu_kswr_t rr;
  uint8_t *q2, *t2;
  int k;
  sw_pass(size, qlen, query, tlen, target, mat, o_del, e_del, o_ins, e_ins, xtra, r, cells);
  if ((xtra & KSW_XSTART) == 0 || ((xtra & KSW_XSUBO) && r->score < (xtra & 0xffff))) return;
  /* the start: align the reversed query prefix [0, qe] against the target
     whose first te+1 bases are reversed, stopping at the score (ksw.c:345-355) */
  q2 = (uint8_t *)malloc((size_t)r->qe + 2);
  t2 = (uint8_t *)malloc((size_t)tlen + 1);
  for (k = 0; k <= r->qe; ++k) q2[k] = query[r->qe - k];
  memcpy(t2, target, (size_t)tlen);
  for (k = 0; k <= r->te; ++k) t2[k] = target[r->te - k];
  sw_pass(size, r->qe + 1, q2, tlen, t2, mat, o_del, e_del, o_ins, e_ins, KSW_XSTOP | r->score, &rr, cells);
  free(q2);
  free(t2);
  if (r->score == rr.score) r->tb = r->te - rr.te, r->qb = r->qe - rr.qe;
}

int oracle_align2_batch(const bwagpu_opt_t *opt, int32_t n_tasks, const bwagpu_align2_task_t *tasks,
                        const uint8_t *qpool, const uint8_t *tpool, bwagpu_kswr_t *results, int64_t *cells)
{
  for (int32_t k = 0; k < n_tasks; ++k) {
    const bwagpu_align2_task_t *t = &tasks[k];
    oracle_ksw_align2(t->qlen, qpool + t->qoff, t->tlen, tpool + t->toff, opt->mat, opt->o_del, opt->e_del,
                      opt->o_ins, opt->e_ins, t->xtra, &results[k], cells);
  }
  return 0;
}
