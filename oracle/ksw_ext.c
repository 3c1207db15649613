/*
 * ksw_ext.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Clean-room restatement of ksw_extend2 (bwa/ksw.c:380-479): banded,
 * affine-gap, semi-global extension of a seed hit whose upstream part scored
 * h0.  Written from the recurrences, in row-major order over the target, with
 * a persistent per-column state that mirrors the reference's eh[] array:
 *
 *   hdiag[j] (= eh[j].h): before row i, H(i-1, j-1); column -1 is the virtual
 *            "first column" whose value is h0 - o_del - e_del*(i+1)
 *   ecol[j]  (= eh[j].e): before row i, E(i, j)
 *
 * Per row i over the band [lo, hi):
 *   M      = hdiag[j] ? hdiag[j] + S(t_i, q_j) : 0        (ksw.c:433)
 *   H(i,j) = max(M, E(i,j), F(i,j))                       (ksw.c:434-435)
 *   E(i+1,j) = max(E(i,j) - e_del, max(M - oe_del, 0))    (ksw.c:440-443)
 *   F(i,j+1) = max(F(i,j) - e_ins, max(M - oe_ins, 0))    (ksw.c:444-447)
 * with the row max m / its LAST column mj (ksw.c:436-437), the end-of-row
 * bookkeeping (ksw.c:449-464) and the zero-trimmed band (ksw.c:466-469).
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

static inline int imax(int a, int b) { return a > b ? a : b; }
static inline int imin(int a, int b) { return a < b ? a : b; }

/* band clamp of ksw.c:399-407 — (int)(double(...)/e + 1.) then >= 1 */
static int gap_cap(int qlen, int best, int end_bonus, int o, int e)
{
  int l = (int)((double)(qlen * best + end_bonus - o) / e + 1.);
  return l > 1 ? l : 1;
}

static int ksw_extend2_core(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                            const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                            int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle,
                            int *gscore, int *max_off, int64_t *cells, int row_bound)
{
  const int oe_del = o_del + e_del, oe_ins = o_ins + e_ins;
  int32_t *hdiag, *ecol;
  int8_t *prof;
  int best_mat = 0, lo, hi, i, j;
  int best, best_i, best_j, end_i, end_sc, off;
  int64_t n_cells = 0, n_rows = 0;

  if (h0 <= 0) return -1; /* reference: assert(h0 > 0), ksw.c:385 */

  hdiag = (int32_t *)calloc((size_t)qlen + 1, sizeof(int32_t));
  ecol = (int32_t *)calloc((size_t)qlen + 1, sizeof(int32_t));
  prof = (int8_t *)malloc((size_t)(qlen > 0 ? qlen : 1) * (size_t)m);
  for (int b = 0; b < m; ++b)
    for (j = 0; j < qlen; ++j) prof[b * qlen + j] = mat[b * m + query[j]];

  /* row "-1": H(-1,-1)=h0, then one insertion gap opened and extended while
     positive (ksw.c:392-395); closed form of that loop */
  hdiag[0] = h0;
  for (j = 1; j <= qlen; ++j) {
    int v = h0 - oe_ins - (j - 1) * e_ins;
    if (v <= 0) break;
    hdiag[j] = v;
  }

  for (i = 0; i < m * m; ++i) best_mat = imax(best_mat, mat[i]);
  w = imin(w, gap_cap(qlen, best_mat, end_bonus, o_ins, e_ins));
  w = imin(w, gap_cap(qlen, best_mat, end_bonus, o_del, e_del));

  best = h0;
  best_i = best_j = -1;
  end_i = -1;
  end_sc = -1;
  off = 0;
  lo = 0;
  hi = qlen;
  for (i = 0; i < tlen; ++i) {
    const int8_t *srow = &prof[target[i] * qlen];
    int left, f = 0, rmax = 0, rarg = -1;
    lo = imax(lo, i - w);
    hi = imin(imin(hi, i + w + 1), qlen);
    /* value of the virtual column j = -1 in this row */
    left = lo == 0 ? imax(h0 - (o_del + e_del * (i + 1)), 0) : 0;
    for (j = lo; j < hi; ++j) {
      int mv = hdiag[j], ev = ecol[j], h;
      hdiag[j] = left;                /* becomes H(i, j-1) for row i+1 */
      mv = mv ? mv + srow[j] : 0;
      h = imax(imax(mv, ev), f);
      left = h;
      if (h >= rmax) { rmax = h; rarg = j; } /* ties -> last column */
      ecol[j] = imax(ev - e_del, imax(mv - oe_del, 0));
      f = imax(f - e_ins, imax(mv - oe_ins, 0));
    }
    n_rows++;
    if (hi > lo) n_cells += hi - lo;
    hdiag[hi] = left;
    ecol[hi] = 0;
    /* the loop variable ends at max(lo, hi) (ksw.c:424,450) */
    if (imax(lo, hi) == qlen) {
      if (!(end_sc > left)) end_i = i; /* ties -> last row */
      end_sc = imax(end_sc, left);
    }
    if (rmax == 0) break;
    if (rmax > best) {
      best = rmax;
      best_i = i;
      best_j = rarg;
      off = imax(off, abs(rarg - i));
    } else if (zdrop > 0) {
      int di = i - best_i, dj = rarg - best_j;
      int drop = di > dj ? best - rmax - (di - dj) * e_del : best - rmax - (dj - di) * e_ins;
      if (drop > zdrop) break;
    }
    /* NOT part of ksw_extend2: the row bound the GPU kernels apply
       (ksw_dev.h extend_quad), here only to test its
       claim on the golden calls — no later cell exceeds a stored positive
       diagonal value plus max(mat) per query column ahead of it, so once that
       bound is below gscore (<= best) no output can change */
    if (row_bound) {
      int bnd = 0;
      for (j = lo; j <= qlen; ++j)
        if (hdiag[j] > 0) bnd = imax(bnd, hdiag[j] + (qlen - j) * best_mat);
      if (lo == 0 && h0 - (o_del + e_del * (i + 2)) > 0) bnd = imax(bnd, h0 - (o_del + e_del * (i + 2)) + qlen * best_mat);
      if (bnd < end_sc) break;
    }
    /* trim the band to the columns whose state is not all-zero */
    for (j = lo; j < hi && hdiag[j] == 0 && ecol[j] == 0; ++j)
      ;
    lo = j;
    for (j = hi; j >= lo && hdiag[j] == 0 && ecol[j] == 0; --j)
      ;
    hi = imin(j + 2, qlen);
  }
  free(hdiag);
  free(ecol);
  free(prof);
  if (qle) *qle = best_j + 1;
  if (tle) *tle = best_i + 1;
  if (gtle) *gtle = end_i + 1;
  if (gscore) *gscore = end_sc;
  if (max_off) *max_off = off;
  if (cells) { cells[0] += n_cells; cells[1] += n_rows; }
  return best;
}

int oracle_ksw_extend2(int qlen, const uint8_t *query, int tlen, const uint8_t *target, int m,
                       const int8_t *mat, int o_del, int e_del, int o_ins, int e_ins, int w,
                       int end_bonus, int zdrop, int h0, int *qle, int *tle, int *gtle,
                       int *gscore, int *max_off, int64_t *cells)
{
  return ksw_extend2_core(qlen, query, tlen, target, m, mat, o_del, e_del, o_ins, e_ins, w, end_bonus, zdrop,
                          h0, qle, tle, gtle, gscore, max_off, cells, 0);
}

/* the same calls with the row bound (tests only: the bound's claim) */
int oracle_extend_batch_bounded(const bwagpu_opt_t *opt, int32_t n_tasks, const bwagpu_ext_task_t *tasks,
                                const uint8_t *qpool, const uint8_t *tpool, bwagpu_ext_result_t *results,
                                int64_t *cells)
{
  for (int32_t k = 0; k < n_tasks; ++k) {
    const bwagpu_ext_task_t *t = &tasks[k];
    bwagpu_ext_result_t *r = &results[k];
    r->score = ksw_extend2_core(t->qlen, qpool + t->qoff, t->tlen, tpool + t->toff, 5, opt->mat, opt->o_del,
                                opt->e_del, opt->o_ins, opt->e_ins, t->w, t->end_bonus, t->zdrop, t->h0, &r->qle,
                                &r->tle, &r->gtle, &r->gscore, &r->max_off, cells, 1);
  }
  return 0;
}

int oracle_extend_batch(const bwagpu_opt_t *opt, int32_t n_tasks, const bwagpu_ext_task_t *tasks,
                        const uint8_t *qpool, const uint8_t *tpool, bwagpu_ext_result_t *results,
                        int64_t *cells)
{
  for (int32_t k = 0; k < n_tasks; ++k) {
    const bwagpu_ext_task_t *t = &tasks[k];
    bwagpu_ext_result_t *r = &results[k];
    r->score = oracle_ksw_extend2(t->qlen, qpool + t->qoff, t->tlen, tpool + t->toff, 5, opt->mat,
                                  opt->o_del, opt->e_del, opt->o_ins, opt->e_ins, t->w,
                                  t->end_bonus, t->zdrop, t->h0, &r->qle, &r->tle, &r->gtle,
                                  &r->gscore, &r->max_off, cells);
  }
  return 0;
}
