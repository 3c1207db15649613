/*
 * sam_hooks.c — the bwa side of the SAM-stage GPU path (include/bwagpu_sam.h).
 *
 * Compiled together with bwa (it includes bwa's bwamem.h / ksw.h), this file
 * defines ksw_align2 and mem_reg2aln.  Linked into a program that loads bwa
 * as a shared object (built -fPIC, so bwa's own calls go through the PLT —
 * mem_reg2sam's call at bwamem.c:1037 included), these definitions take the
 * place of bwa's for every caller: mem_matesw (bwamem_pair.c:154),
 * mem_sam_pe (bwamem_pair.c:343/351/382), mem_reg2sam (bwamem.c:1037/1050),
 * mem_gen_alt (bwamem_extra.c:119).  With no cache attached they forward to
 * bwa's own functions (dlsym RTLD_NEXT), so the CPU path is unchanged.
 *
 * With a cache attached (bwagpu_sam_hooks_attach), ksw_align2 answers from the
 * cache and mem_reg2aln builds its mem_aln_t from the cached GPU job exactly as
 * bwamem.c:1104-1174 fills it: CIGAR/MD/NM/strand/contig/position from the
 * device (bwagpu_reg2aln_batch), mapq/flag/score/sub/is_alt/alt_sc from the
 * region (bwamem.c:1121-1122, 1170-1171).  Misses answer with placeholders and
 * are queued; the stage loop flushes and re-runs the pass until a pass has no
 * miss (see bwagpu_sam.h).
 *
 * Requirements: the ksw_align2 calls answered from the cache are mem_matesw's
 * (m = 5, the stage's opt->mat / gap penalties, qry = NULL); any other call
 * (qry != NULL, m != 5) goes to bwa's function.  The cache's bwagpu context
 * must have been created from the same mem_opt_t.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "bntseq.h"
#include "bwamem.h"
#include "kstring.h"
#include "ksw.h"
#include "bwagpu_sam.h"

extern unsigned char nst_nt4_table[256];
int mem_approx_mapq_se(const mem_opt_t *opt, const mem_alnreg_t *a); /* bwamem.c:967 */

typedef kswr_t (*align2_fn)(int, uint8_t *, int, uint8_t *, int, const int8_t *, int, int, int, int, int, kswq_t **);
typedef mem_aln_t (*reg2aln_fn)(const mem_opt_t *, const bntseq_t *, const uint8_t *, int, const char *,
                                const mem_alnreg_t *);
typedef int (*cache_a2_fn)(bwagpu_samcache_t *, int32_t, const uint8_t *, int32_t, const uint8_t *, int32_t,
                           bwagpu_kswr_t *);
typedef int (*cache_r2_fn)(bwagpu_samcache_t *, int32_t, const uint8_t *, int64_t, int64_t, int32_t, int32_t,
                           int32_t, int32_t, bwagpu_aln_t *, uint32_t **);

static bwagpu_samcache_t *g_cache;
static cache_a2_fn g_a2;
static cache_r2_fn g_r2;
static align2_fn real_align2;
static reg2aln_fn real_reg2aln;
static volatile int g_error; /* a cached job the device could not align */
static __thread int g_tls_miss; /* misses of the calling thread since the last take */

/* cache misses of the calling thread since the last call, reset to 0: a
   stage worker brackets one pair's mem_sam_pe with it to learn whether that
   pair's text must be redone after the next flush */
int bwagpu_sam_hooks_take_misses(void)
{
  const int m = g_tls_miss;
  g_tls_miss = 0;
  return m;
}

static void resolve_real(void)
{
  if (!real_align2) real_align2 = (align2_fn)dlsym(RTLD_NEXT, "ksw_align2");
  if (!real_reg2aln) real_reg2aln = (reg2aln_fn)dlsym(RTLD_NEXT, "mem_reg2aln");
  if (!real_align2 || !real_reg2aln) {
    fprintf(stderr, "sam_hooks: bwa's ksw_align2 / mem_reg2aln not found (bwa must be a shared object)\n");
    abort();
  }
}

/* attach a cache (NULL detaches).  The cache functions are looked up in the
   global scope (libgpusam.so linked, or dlopen'ed RTLD_GLOBAL).  Call with no
   stage thread running.  Returns 0, or -1 if libgpusam.so is not loaded. */
int bwagpu_sam_hooks_attach(bwagpu_samcache_t *c)
{
  resolve_real();
  if (c) {
    g_a2 = (cache_a2_fn)dlsym(RTLD_DEFAULT, "bwagpu_samcache_align2");
    g_r2 = (cache_r2_fn)dlsym(RTLD_DEFAULT, "bwagpu_samcache_reg2aln");
    if (!g_a2 || !g_r2) return -1;
  }
  g_cache = c;
  return 0;
}

/* quiet passes: mem_aln2sam (bwamem.c:837-930) writes no SAM text — the
   collect passes' text is discarded anyway, and formatting is most of a
   pass's CPU time.  The string is still allocated and terminated, since
   mem_sam_pe strdup's it (bwamem_pair.c:359). */
static volatile int g_quiet;
void bwagpu_sam_hooks_quiet(int quiet) { g_quiet = quiet; }

typedef void (*aln2sam_fn)(const mem_opt_t *, const bntseq_t *, kstring_t *, bseq1_t *, int, const mem_aln_t *, int,
                           const mem_aln_t *);
static aln2sam_fn real_aln2sam;

void mem_aln2sam(const mem_opt_t *opt, const bntseq_t *bns, kstring_t *str, bseq1_t *s, int n, const mem_aln_t *list,
                 int which, const mem_aln_t *m)
{
  if (g_quiet && g_cache) {
    if (!str->s) {
      str->m = 16;
      str->s = (char *)malloc(str->m);
    }
    str->s[str->l] = 0;
    return;
  }
  if (!real_aln2sam) real_aln2sam = (aln2sam_fn)dlsym(RTLD_NEXT, "mem_aln2sam");
  real_aln2sam(opt, bns, str, s, n, list, which, m);
}

/* jobs the device flagged since the last call (BWAGPU_ALN_NO_CIGAR: the
   reference itself would dereference NULL there), reset to 0 */
int bwagpu_sam_hooks_errors(void)
{
  const int e = g_error;
  g_error = 0;
  return e;
}

kswr_t ksw_align2(int qlen, uint8_t *query, int tlen, uint8_t *target, int m, const int8_t *mat, int o_del,
                  int e_del, int o_ins, int e_ins, int xtra, kswq_t **qry)
{
  if (!g_cache || qry || m != 5) {
    if (!real_align2) resolve_real();
    return real_align2(qlen, query, tlen, target, m, mat, o_del, e_del, o_ins, e_ins, xtra, qry);
  }
  bwagpu_kswr_t r;
  const int rc = g_a2(g_cache, qlen, query, tlen, target, xtra, &r);
  if (rc < 0) {
    fprintf(stderr, "sam_hooks: bwagpu_samcache_align2 failed\n");
    abort();
  }
  g_tls_miss += rc;
  kswr_t x;
  x.score = r.score; x.te = r.te; x.qe = r.qe; x.score2 = r.score2; x.te2 = r.te2; x.tb = r.tb; x.qb = r.qb;
  return x;
}

mem_aln_t mem_reg2aln(const mem_opt_t *opt, const bntseq_t *bns, const uint8_t *pac, int l_query, const char *query_,
                      const mem_alnreg_t *ar)
{
  if (!g_cache || ar == 0 || ar->rb < 0 || ar->re < 0) { /* no cache, or the unmapped record (no SW work) */
    if (!real_reg2aln) resolve_real();
    return real_reg2aln(opt, bns, pac, l_query, query_, ar);
  }
  uint8_t qs[1024], *q = l_query <= (int)sizeof qs ? qs : (uint8_t *)malloc(l_query);
  for (int i = 0; i < l_query; ++i) /* the nt4 conversion of bwamem.c:1119-1120 */
    q[i] = query_[i] < 5 ? query_[i] : nst_nt4_table[(int)query_[i]];
  bwagpu_aln_t g;
  uint32_t *cig = 0;
  const int rc = g_r2(g_cache, l_query, q, ar->rb, ar->re, ar->qb, ar->qe, ar->truesc, ar->w, &g, &cig);
  if (q != qs) free(q);
  if (rc < 0) {
    fprintf(stderr, "sam_hooks: bwagpu_samcache_reg2aln failed\n");
    abort();
  }
  g_tls_miss += rc;
  mem_aln_t a;
  memset(&a, 0, sizeof a);
  a.mapq = ar->secondary < 0 ? mem_approx_mapq_se(opt, ar) : 0;
  if (ar->secondary >= 0) a.flag |= 0x100;
  a.cigar = cig;
  if (rc == 0 && g.status == BWAGPU_ALN_OK) {
    a.n_cigar = g.n_cigar;
    a.NM = g.NM;
    a.is_rev = g.is_rev;
    a.rid = g.rid;
    a.pos = g.pos;
  } else { /* a miss (placeholder for this pass) or a job the device flagged */
    if (rc == 0) g_error = 1;
    a.rid = ar->rid;
    a.pos = 0;
  }
  a.score = ar->score;
  a.sub = ar->sub > ar->csub ? ar->sub : ar->csub;
  a.is_alt = ar->is_alt;
  a.alt_sc = ar->alt_sc;
  return a;
}
