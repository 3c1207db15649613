/*
 * seed.c — TEST INFRASTRUCTURE ONLY (part of liboracle.so): a clean-room C
 * restatement of seeding's interval collection, mem_collect_intv
 * (bwa/bwamem.c:120-167), with everything under it: the occurrence counts of
 * the interleaved BWT (bwt_occ4, bwt.c:169-187), the bidirectional extension
 * (bwt_extend, bwt.c:262-276), SMEM search (bwt_smem1a, bwt.c:289-351), the
 * LAST-like pass (bwt_seed_strategy1, bwt.c:358-378) and klib's introsort of
 * the intervals by info (ksort.h:176-226 instantiated at bwamem.c:90-91).
 *
 * It is the checker of bwagpu_collect_intv; it is pinned against
 * tests/golden/seed_*.npz, which oracle/_ref/gen_seed produces from the
 * reference's own bwt_smem1 / bwt_seed_strategy1 / ks_introsort_mem_intv.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

typedef struct {
  uint64_t x[3], info;
} ivl_t; /* == bwtintv_t (bwt.h:60-62) */

typedef struct {
  uint64_t primary, L2[5], seq_len;
  const uint32_t *bwt;
} obwt_t;

/* bwt.c:169-187: counts of A/C/G/T in bwt[0..k] ($ removed) */
static void occ4(const obwt_t *b, uint64_t k, uint64_t cnt[4])
{
  if (k == (uint64_t)-1) {
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
    return;
  }
  k -= (k >= b->primary);
  const uint32_t *p = b->bwt + (k >> 7 << 4); /* the 128-base block: 4 uint64 counts, 8 words of bases */
  memcpy(cnt, p, 4 * sizeof(uint64_t));
  const uint32_t *w = p + 8;
  const int nfull = (int)((k & 127) >> 4);
  uint32_t c[4] = {0, 0, 0, 0};
  for (int i = 0; i <= nfull; ++i) {
    /* bases are packed first-in-highest-bits: base j of a word at bits (15-j)*2 */
    const uint32_t m = i < nfull ? 0xffffffffu : ~((1u << ((~k & 15) << 1)) - 1);
    for (int v = 1; v < 4; ++v) {
      const uint32_t x = w[i] ^ (0x55555555u * (uint32_t)v);
      c[v] += (uint32_t)__builtin_popcount(~(x | x >> 1) & 0x55555555u & m);
    }
  }
  c[0] = (uint32_t)(k & 127) + 1 - c[1] - c[2] - c[3];
  for (int v = 0; v < 4; ++v) cnt[v] += c[v];
}

static uint64_t n_extend; /* bwt_extend calls (work statistics for the device kernel's tiers) */
uint64_t oracle_seed_extends(void) { return n_extend; }

/* bwt.c:262-276 */
static void extend(const obwt_t *b, const ivl_t *ik, ivl_t ok[4], int is_back)
{
  uint64_t tk[4], tl[4];
  ++n_extend;
  occ4(b, ik->x[!is_back] - 1, tk);
  occ4(b, ik->x[!is_back] - 1 + ik->x[2], tl);
  for (int i = 0; i < 4; ++i) {
    ok[i].x[!is_back] = b->L2[i] + 1 + tk[i];
    ok[i].x[2] = tl[i] - tk[i];
  }
  ok[3].x[is_back] = ik->x[is_back] + (ik->x[!is_back] <= b->primary && ik->x[!is_back] + ik->x[2] - 1 >= b->primary);
  ok[2].x[is_back] = ok[3].x[is_back] + ok[3].x[2];
  ok[1].x[is_back] = ok[2].x[is_back] + ok[2].x[2];
  ok[0].x[is_back] = ok[1].x[is_back] + ok[1].x[2];
}

static void set_intv(const obwt_t *b, int c, ivl_t *ik) /* bwt.h:80 */
{
  ik->x[0] = b->L2[c] + 1;
  ik->x[2] = b->L2[c + 1] - b->L2[c];
  ik->x[1] = b->L2[3 - c] + 1;
  ik->info = 0;
}

typedef struct {
  ivl_t *a;
  int n, m;
} ivec_t;

static void push(ivec_t *v, const ivl_t *x)
{
  if (v->n == v->m) {
    v->m = v->m ? v->m << 1 : 16;
    v->a = (ivl_t *)realloc(v->a, sizeof(ivl_t) * (size_t)v->m);
  }
  v->a[v->n++] = *x;
}

static void reverse(ivec_t *v)
{
  for (int j = 0; j < v->n >> 1; ++j) {
    ivl_t t = v->a[v->n - 1 - j];
    v->a[v->n - 1 - j] = v->a[j];
    v->a[j] = t;
  }
}

/* bwt.c:289-351 with max_intv = 0 (bwt_smem1, bwt.c:353-356) */
static int smem1(const obwt_t *b, int len, const uint8_t *q, int x, int min_intv, ivec_t *mem, ivec_t *prev,
                 ivec_t *curr)
{
  ivl_t ik, ok[4];
  int i, ret;
  mem->n = 0;
  if (q[x] > 3) return x + 1;
  if (min_intv < 1) min_intv = 1;
  set_intv(b, q[x], &ik);
  ik.info = (uint64_t)(x + 1);
  curr->n = 0;
  for (i = x + 1; i < len; ++i) { /* forward */
    if (q[i] < 4) {
      const int c = 3 - q[i];
      extend(b, &ik, ok, 0);
      if (ok[c].x[2] != ik.x[2]) {
        push(curr, &ik);
        if (ok[c].x[2] < (uint64_t)min_intv) break;
      }
      ik = ok[c];
      ik.info = (uint64_t)(i + 1);
    } else {
      push(curr, &ik);
      break;
    }
  }
  if (i == len) push(curr, &ik);
  reverse(curr); /* longest matches first */
  ret = (int)curr->a[0].info;
  ivec_t *t = curr; curr = prev; prev = t;
  for (i = x - 1; i >= -1; --i) { /* backward */
    const int c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
    curr->n = 0;
    for (int j = 0; j < prev->n; ++j) {
      const ivl_t *p = &prev->a[j];
      if (c >= 0) extend(b, p, ok, 1);
      if (c < 0 || ok[c].x[2] < (uint64_t)min_intv) {
        if (curr->n == 0 && (mem->n == 0 || (uint64_t)(i + 1) < mem->a[mem->n - 1].info >> 32)) {
          ik = *p;
          ik.info |= (uint64_t)(i + 1) << 32;
          push(mem, &ik);
        }
      } else if (curr->n == 0 || ok[c].x[2] != curr->a[curr->n - 1].x[2]) {
        ok[c].info = p->info;
        push(curr, &ok[c]);
      }
    }
    if (curr->n == 0) break;
    t = curr; curr = prev; prev = t;
  }
  reverse(mem); /* by start */
  return ret;
}

/* bwt.c:358-378 */
static int seed_strategy1(const obwt_t *b, int len, const uint8_t *q, int x, int min_len, int max_intv, ivl_t *mem)
{
  ivl_t ik, ok[4];
  memset(mem, 0, sizeof *mem);
  if (q[x] > 3) return x + 1;
  set_intv(b, q[x], &ik);
  for (int i = x + 1; i < len; ++i) {
    if (q[i] < 4) {
      const int c = 3 - q[i];
      extend(b, &ik, ok, 0);
      if (ok[c].x[2] < (uint64_t)max_intv && i - x >= min_len) {
        *mem = ok[c];
        mem->info = (uint64_t)x << 32 | (uint64_t)(i + 1);
        return i + 1;
      }
      ik = ok[c];
    } else return i + 1;
  }
  return len;
}

/* klib introsort (ksort.h:146-226) ordered by info: a partition scheme with a
   median of three, an explicit stack, comb sort past 2*ceil(log2 n) levels and
   one insertion sort at the end — reproduced step for step, since the order of
   intervals with equal info depends on it */
#define LT(a, b) ((a).info < (b).info)
static void insert_sort(ivl_t *s, ivl_t *t)
{
  for (ivl_t *i = s + 1; i < t; ++i)
    for (ivl_t *j = i; j > s && LT(*j, *(j - 1)); --j) {
      ivl_t x = *j; *j = *(j - 1); *(j - 1) = x;
    }
}
static void comb_sort(size_t n, ivl_t *a)
{
  const double shrink = 1.2473309501039786540366528676643;
  size_t gap = n;
  int swapped;
  do {
    if (gap > 2) {
      gap = (size_t)(gap / shrink);
      if (gap == 9 || gap == 10) gap = 11;
    }
    swapped = 0;
    for (ivl_t *i = a; i < a + n - gap; ++i) {
      ivl_t *j = i + gap;
      if (LT(*j, *i)) { ivl_t x = *i; *i = *j; *j = x; swapped = 1; }
    }
  } while (swapped || gap > 2);
  if (gap != 1) insert_sort(a, a + n);
}
static void intro_sort(size_t n, ivl_t *a)
{
  if (n < 1) return;
  if (n == 2) {
    if (LT(a[1], a[0])) { ivl_t x = a[0]; a[0] = a[1]; a[1] = x; }
    return;
  }
  int d;
  for (d = 2; 1ul << d < n; ++d);
  struct { ivl_t *l, *r; int d; } stack[2 * 64 + 2], *top = stack;
  ivl_t *s = a, *t = a + (n - 1), *i, *j, *k, rp, x;
  d <<= 1;
  for (;;) {
    if (s < t) {
      if (--d == 0) {
        comb_sort((size_t)(t - s + 1), s);
        t = s;
        continue;
      }
      i = s; j = t; k = i + ((j - i) >> 1) + 1;
      if (LT(*k, *i)) {
        if (LT(*k, *j)) k = j;
      } else k = LT(*j, *i) ? i : j;
      rp = *k;
      if (k != t) { x = *k; *k = *t; *t = x; }
      for (;;) {
        do ++i; while (LT(*i, rp));
        do --j; while (i <= j && LT(rp, *j));
        if (j <= i) break;
        x = *i; *i = *j; *j = x;
      }
      x = *i; *i = *t; *t = x;
      if (i - s > t - i) {
        if (i - s > 16) { top->l = s; top->r = i - 1; top->d = d; ++top; }
        s = t - i > 16 ? i + 1 : t;
      } else {
        if (t - i > 16) { top->l = i + 1; top->r = t; top->d = d; ++top; }
        t = i - s > 16 ? i - 1 : s;
      }
    } else {
      if (top == stack) {
        insert_sort(a, a + n);
        return;
      }
      --top; s = top->l; t = top->r; d = top->d;
    }
  }
}

/* bwamem.c:120-167.  hdr = {primary, L2[0..4], seq_len}; opt = {min_seed_len,
   split_width, max_mem_intv}.  Writes up to cap intervals (x0, x1, x2, info)
   to out; returns how many the read has (may exceed cap). */
int oracle_collect_intv(const int64_t *hdr, const uint32_t *bwt_words, const int32_t *opt, float split_factor,
                        int len, const uint8_t *seq, uint64_t *out, int cap)
{
  obwt_t b;
  b.primary = (uint64_t)hdr[0];
  for (int i = 0; i < 5; ++i) b.L2[i] = (uint64_t)hdr[1 + i];
  b.seq_len = (uint64_t)hdr[6];
  b.bwt = bwt_words;
  const int min_seed_len = opt[0], split_width = opt[1], max_mem_intv = opt[2];
  const int split_len = (int)(min_seed_len * split_factor + .499);
  ivec_t mem = {0, 0, 0}, mem1 = {0, 0, 0}, va = {0, 0, 0}, vb = {0, 0, 0};
  int x = 0;
  while (x < len) { /* SMEMs */
    if (seq[x] < 4) {
      x = smem1(&b, len, seq, x, 1, &mem1, &va, &vb);
      for (int i = 0; i < mem1.n; ++i)
        if ((int)((uint32_t)mem1.a[i].info - (mem1.a[i].info >> 32)) >= min_seed_len) push(&mem, &mem1.a[i]);
    } else ++x;
  }
  const int old_n = mem.n;
  for (int k = 0; k < old_n; ++k) { /* re-seeding inside long SMEMs */
    const ivl_t p = mem.a[k];
    const int start = (int)(p.info >> 32), end = (int32_t)p.info;
    if (end - start < split_len || p.x[2] > (uint64_t)split_width) continue;
    smem1(&b, len, seq, (start + end) >> 1, (int)(p.x[2] + 1), &mem1, &va, &vb);
    for (int i = 0; i < mem1.n; ++i)
      if ((uint32_t)mem1.a[i].info - (mem1.a[i].info >> 32) >= (uint32_t)min_seed_len) push(&mem, &mem1.a[i]);
  }
  if (max_mem_intv > 0) { /* LAST-like */
    x = 0;
    while (x < len) {
      if (seq[x] < 4) {
        ivl_t m;
        x = seed_strategy1(&b, len, seq, x, min_seed_len, max_mem_intv, &m);
        if (m.x[2] > 0) push(&mem, &m);
      } else ++x;
    }
  }
  intro_sort((size_t)mem.n, mem.a);
  for (int i = 0; i < mem.n && i < cap; ++i) memcpy(out + 4 * i, &mem.a[i], sizeof(ivl_t));
  const int n = mem.n;
  free(mem.a); free(mem1.a); free(va.a); free(vb.a);
  return n;
}

/* bwt_sa (bwt.c:86-96) with bwt_invPsi (bwt.c:53-59): walk the LF mapping
   until a sampled row, counting steps.  hdr as for oracle_collect_intv. */
uint64_t oracle_bwt_sa(const int64_t *hdr, const uint32_t *bwt_words, const uint64_t *sa, int sa_intv, uint64_t k)
{
  obwt_t b;
  b.primary = (uint64_t)hdr[0];
  for (int i = 0; i < 5; ++i) b.L2[i] = (uint64_t)hdr[1 + i];
  b.seq_len = (uint64_t)hdr[6];
  b.bwt = bwt_words;
  uint64_t steps = 0;
  const uint64_t mask = (uint64_t)sa_intv - 1;
  while (k & mask) {
    ++steps;
    if (k == b.primary) {
      k = 0;
      continue;
    }
    const uint64_t x = k - (k > b.primary);
    const int c = (int)(b.bwt[(x >> 7 << 4) + 8 + ((x & 127) >> 4)] >> ((~x & 15) << 1) & 3); /* bwt_B0 */
    uint64_t cnt[4];
    occ4(&b, k, cnt); /* bwt_occ(k, c), bwt.c:107-128; k == seq_len gives the column total */
    k = b.L2[c] + cnt[c];
  }
  return steps + sa[k / (uint64_t)sa_intv];
}
