/*
 * chain.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Clean-room restatement of seeding's chaining, the part of bwa-flow's
 * SeqsToChains after the interval search (src/bwa_wrapper.cpp:105-115:
 * mem_chain -> mem_chain_flt -> mem_flt_chained_seeds):
 *   mem_chain's body      bwa/bwamem.c:260-330 (frac_rep, the SA positions of
 *                         each interval stepped to max_occ, bns_intv2rid
 *                         bntseq.c:365-373, the kbtree of chains keyed by pos)
 *   kbtree                bwa/kbtree.h:54-313 for mem_chain_t at
 *                         KB_DEFAULT_SIZE (t = 5): lower-bound node search,
 *                         kb_intervalp, kb_putp with pre-emptive splits, the
 *                         in-order traversal — restated as a B-tree of chain
 *                         indices, because the order of chains with EQUAL pos
 *                         (and which of them kb_intervalp returns) follows the
 *                         tree's shape
 *   test_and_merge        bwamem.c:199-221
 *   mem_chain_weight      bwamem.c:223-244
 *   mem_chain_flt         bwamem.c:336-396 with klib's introsort by weight
 *                         (ksort.h:146-226, step for step: the sort is not
 *                         stable)
 *   mem_flt_chained_seeds bwamem.c:607-624, mem_seed_sw 580-605 (ksw_align2 of
 *                         the seed +-50 bp: oracle_ksw_align2), bns_fetch_seq
 *                         bntseq.c:421-446
 * Pinned by tests/golden/chain_*.npz (oracle/gen_chain.c: the reference's own
 * mem_chain / mem_chain_flt / mem_flt_chained_seeds), tests/test_chain_oracle.py.
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define BT 5            /* kbtree t: ((512 - 4 - 8) / (8 + sizeof(mem_chain_t)=40) + 1) >> 1 */
#define BN (2 * BT - 1) /* keys per node */
#define SHORT_EXT 50    /* MEM_SHORT_EXT, bwamem.c:573 */
#define SHORT_LEN 200   /* MEM_SHORT_LEN */

typedef struct {
  int64_t pos;
  int rid, is_alt, n, cap, first, kept;
  int w;
  bwagpu_seed_t *s;
} ch_t;

typedef struct node {
  int n, internal;
  int key[BN];            /* chain indices, ordered by chains[].pos */
  struct node *child[BN + 1];
} node_t;

typedef struct {
  node_t *root;
  const ch_t *c;
  int n_keys;
} tree_t;

static node_t *new_node(int internal)
{
  node_t *x = (node_t *)calloc(1, sizeof(node_t));
  x->internal = internal;
  return x;
}

static void free_tree(node_t *x)
{
  if (!x) return;
  if (x->internal)
    for (int i = 0; i <= x->n; ++i) free_tree(x->child[i]);
  free(x);
}

static inline int pcmp(int64_t a, int64_t b) { return (b < a) - (a < b); }

/* the node search of kbtree.h:100-113: the first key >= pos (*r = 0 when
   equal, else -1 after stepping back to the last key < pos); past the end,
   the last key with *r = 1 */
static int node_find(const tree_t *t, const node_t *x, int64_t pos, int *r)
{
  int b = 0, e = x->n;
  if (x->n == 0) { *r = -1; return -1; }
  while (b < e) {
    const int m = (b + e) >> 1;
    if (pcmp(t->c[x->key[m]].pos, pos) < 0) b = m + 1;
    else e = m;
  }
  if (b == x->n) { *r = 1; return x->n - 1; }
  if ((*r = pcmp(pos, t->c[x->key[b]].pos)) < 0) --b;
  return b;
}

/* kb_intervalp's lower (kbtree.h:130-147) */
static int lower_of(const tree_t *t, int64_t pos)
{
  int lower = -1, r = 0;
  for (const node_t *x = t->root; x;) {
    const int i = node_find(t, x, pos, &r);
    if (i >= 0 && r == 0) return x->key[i];
    if (i >= 0) lower = x->key[i];
    if (!x->internal) break;
    x = x->child[i + 1];
  }
  return lower;
}

/* __kb_split (kbtree.h:152-167): child y of x at i splits around its median */
static void split(node_t *x, int i, node_t *y)
{
  node_t *z = new_node(y->internal);
  z->n = BT - 1;
  memcpy(z->key, y->key + BT, sizeof(int) * (BT - 1));
  if (y->internal) memcpy(z->child, y->child + BT, sizeof(node_t *) * BT);
  y->n = BT - 1;
  memmove(x->child + i + 2, x->child + i + 1, sizeof(node_t *) * (size_t)(x->n - i));
  x->child[i + 1] = z;
  memmove(x->key + i + 1, x->key + i, sizeof(int) * (size_t)(x->n - i));
  x->key[i] = y->key[BT - 1];
  ++x->n;
}

/* kb_putp (kbtree.h:168-197) */
static void put(tree_t *t, int k)
{
  const int64_t pos = t->c[k].pos;
  int r;
  ++t->n_keys;
  if (t->root->n == BN) {
    node_t *s = new_node(1);
    s->child[0] = t->root;
    split(s, 0, t->root);
    t->root = s;
  }
  node_t *x = t->root;
  for (;;) {
    if (!x->internal) {
      const int i = node_find(t, x, pos, &r);
      if (i != x->n - 1) memmove(x->key + i + 2, x->key + i + 1, sizeof(int) * (size_t)(x->n - i - 1));
      x->key[i + 1] = k;
      ++x->n;
      return;
    }
    int i = node_find(t, x, pos, &r) + 1;
    if (x->child[i]->n == BN) {
      split(x, i, x->child[i]);
      if (pcmp(pos, t->c[x->key[i]].pos) > 0) ++i;
    }
    x = x->child[i];
  }
}

/* __kb_traverse (kbtree.h:336-358): in-order */
static void traverse(const node_t *x, int *out, int *n)
{
  for (int i = 0; i <= x->n; ++i) {
    if (x->internal) traverse(x->child[i], out, n);
    if (i < x->n) out[(*n)++] = x->key[i];
  }
}

static void ch_push(ch_t *c, const bwagpu_seed_t *s)
{
  if (c->n == c->cap) {
    c->cap = c->cap ? c->cap << 1 : 4;
    c->s = (bwagpu_seed_t *)realloc(c->s, sizeof(bwagpu_seed_t) * (size_t)c->cap);
  }
  c->s[c->n++] = *s;
}

/* test_and_merge, bwamem.c:199-221 */
static int merge(int w, int max_chain_gap, int64_t l_pac, ch_t *c, const bwagpu_seed_t *p, int rid)
{
  const bwagpu_seed_t *last = &c->s[c->n - 1];
  const int64_t qend = last->qbeg + last->len, rend = last->rbeg + last->len;
  if (rid != c->rid) return 0;
  if (p->qbeg >= c->s[0].qbeg && p->qbeg + p->len <= qend && p->rbeg >= c->s[0].rbeg && p->rbeg + p->len <= rend)
    return 1; /* contained: dropped */
  if ((last->rbeg < l_pac || c->s[0].rbeg < l_pac) && p->rbeg >= l_pac) return 0;
  const int64_t x = p->qbeg - last->qbeg, y = p->rbeg - last->rbeg;
  if (y >= 0 && x - y <= w && y - x <= w && x - last->len < max_chain_gap && y - last->len < max_chain_gap) {
    ch_push(c, p);
    return 1;
  }
  return 0;
}

static int pos2rid(const bwagpu_bns_t *bns, int64_t pos_f) /* bns_pos2rid, bntseq.c:349-363 */
{
  int left = 0, mid = 0, right = bns->n_seqs;
  if (pos_f >= bns->l_pac) return -1;
  while (left < right) {
    mid = (left + right) >> 1;
    if (pos_f >= bns->ann_offset[mid]) {
      if (mid == bns->n_seqs - 1) break;
      if (pos_f < bns->ann_offset[mid + 1]) break;
      left = mid + 1;
    } else right = mid;
  }
  return mid;
}

static inline int64_t depos(int64_t l_pac, int64_t pos) { return pos >= l_pac ? (l_pac << 1) - 1 - pos : pos; }

static int intv2rid(const bwagpu_bns_t *bns, int64_t rb, int64_t re) /* bntseq.c:365-373 */
{
  if (rb < bns->l_pac && re > bns->l_pac) return -2;
  const int b = pos2rid(bns, depos(bns->l_pac, rb));
  const int e = rb < re ? pos2rid(bns, depos(bns->l_pac, re - 1)) : b;
  return b == e ? b : -1;
}

static int weight(const ch_t *c) /* mem_chain_weight, bwamem.c:223-244 */
{
  int64_t end;
  int j, w = 0, tmp;
  for (j = 0, end = 0; j < c->n; ++j) {
    const bwagpu_seed_t *s = &c->s[j];
    if (s->qbeg >= end) w += s->len;
    else if (s->qbeg + s->len > end) w += (int)(s->qbeg + s->len - end);
    end = end > s->qbeg + s->len ? end : s->qbeg + s->len;
  }
  tmp = w;
  w = 0;
  for (j = 0, end = 0; j < c->n; ++j) {
    const bwagpu_seed_t *s = &c->s[j];
    if (s->rbeg >= end) w += s->len;
    else if (s->rbeg + s->len > end) w += (int)(s->rbeg + s->len - end);
    end = end > s->rbeg + s->len ? end : s->rbeg + s->len;
  }
  w = w < tmp ? w : tmp;
  return w < 1 << 30 ? w : (1 << 30) - 1;
}

/* klib introsort (ksort.h:146-226) over chain pointers by weight, greater
   first (mem_flt's flt_lt, bwamem.c:333-334) — step for step */
#define FLT_LT(a, b) ((a)->w > (b)->w)
typedef ch_t *cp_t;
static void c_insert_sort(cp_t *s, cp_t *t)
{
  for (cp_t *i = s + 1; i < t; ++i)
    for (cp_t *j = i; j > s && FLT_LT(*j, *(j - 1)); --j) { cp_t x = *j; *j = *(j - 1); *(j - 1) = x; }
}
static void c_comb_sort(size_t n, cp_t *a)
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
    for (cp_t *i = a; i < a + n - gap; ++i) {
      cp_t *j = i + gap;
      if (FLT_LT(*j, *i)) { cp_t x = *i; *i = *j; *j = x; swapped = 1; }
    }
  } while (swapped || gap > 2);
  if (gap != 1) c_insert_sort(a, a + n);
}
static void c_intro_sort(size_t n, cp_t *a)
{
  if (n < 1) return;
  if (n == 2) {
    if (FLT_LT(a[1], a[0])) { cp_t x = a[0]; a[0] = a[1]; a[1] = x; }
    return;
  }
  int d;
  for (d = 2; 1ul << d < n; ++d);
  struct { cp_t *l, *r; int d; } stack[2 * 64 + 2], *top = stack;
  cp_t *s = a, *t = a + (n - 1), *i, *j, *k, rp, x;
  d <<= 1;
  for (;;) {
    if (s < t) {
      if (--d == 0) {
        c_comb_sort((size_t)(t - s + 1), s);
        t = s;
        continue;
      }
      i = s; j = t; k = i + ((j - i) >> 1) + 1;
      if (FLT_LT(*k, *i)) {
        if (FLT_LT(*k, *j)) k = j;
      } else k = FLT_LT(*j, *i) ? i : j;
      rp = *k;
      if (k != t) { x = *k; *k = *t; *t = x; }
      for (;;) {
        do ++i; while (FLT_LT(*i, rp));
        do --j; while (i <= j && FLT_LT(rp, *j));
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
        c_insert_sort(a, a + n);
        return;
      }
      --top; s = top->l; t = top->r; d = top->d;
    }
  }
}

#define CHN_BEG(c) ((c)->s[0].qbeg)
#define CHN_END(c) ((c)->s[(c)->n - 1].qbeg + (c)->s[(c)->n - 1].len)

/* mem_chain_flt, bwamem.c:336-396, over chain pointers; returns the kept count */
static int chain_flt(const oracle_chainopt_t *o, int n_chn, cp_t *a)
{
  int i, k;
  if (n_chn == 0) return 0;
  for (i = k = 0; i < n_chn; ++i) {
    ch_t *c = a[i];
    c->first = -1;
    c->kept = 0;
    c->w = weight(c) & ((1 << 29) - 1); /* the 29-bit field of mem_chain_t */
    if (c->w < o->min_chain_weight) free(c->s), c->s = 0, c->n = 0;
    else a[k++] = c;
  }
  n_chn = k;
  c_intro_sort((size_t)n_chn, a);
  if (n_chn == 0) return 0; /* (the reference indexes a[0] here regardless; nothing is read from it) */
  int *chains = (int *)malloc(sizeof(int) * (size_t)n_chn), nc = 0;
  a[0]->kept = 3;
  chains[nc++] = 0;
  for (i = 1; i < n_chn; ++i) {
    int large_ovlp = 0;
    for (k = 0; k < nc; ++k) {
      const int j = chains[k];
      const int b_max = CHN_BEG(a[j]) > CHN_BEG(a[i]) ? CHN_BEG(a[j]) : CHN_BEG(a[i]);
      const int e_min = CHN_END(a[j]) < CHN_END(a[i]) ? CHN_END(a[j]) : CHN_END(a[i]);
      if (e_min > b_max && (!a[j]->is_alt || a[i]->is_alt)) {
        const int li = CHN_END(a[i]) - CHN_BEG(a[i]), lj = CHN_END(a[j]) - CHN_BEG(a[j]);
        const int min_l = li < lj ? li : lj;
        if (e_min - b_max >= min_l * o->mask_level && min_l < o->max_chain_gap) {
          large_ovlp = 1;
          if (a[j]->first < 0) a[j]->first = i;
          if (a[i]->w < a[j]->w * o->drop_ratio && a[j]->w - a[i]->w >= o->min_seed_len << 1) break;
        }
      }
    }
    if (k == nc) {
      chains[nc++] = i;
      a[i]->kept = large_ovlp ? 2 : 3;
    }
  }
  for (i = 0; i < nc; ++i) {
    const ch_t *c = a[chains[i]];
    if (c->first >= 0) a[c->first]->kept = 1;
  }
  free(chains);
  for (i = k = 0; i < n_chn; ++i) {
    if (a[i]->kept == 0 || a[i]->kept == 3) continue;
    if (++k >= o->max_chain_extend) break;
  }
  for (; i < n_chn; ++i)
    if (a[i]->kept < 3) a[i]->kept = 0;
  for (i = k = 0; i < n_chn; ++i) {
    ch_t *c = a[i];
    if (c->kept == 0) free(c->s), c->s = 0, c->n = 0;
    else a[k++] = a[i];
  }
  return k;
}

/* mem_seed_sw, bwamem.c:580-605 */
static int seed_sw(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const uint8_t *pac, int l_query,
                   const uint8_t *query, const bwagpu_seed_t *s)
{
  const int64_t l_pac = bns->l_pac;
  if (s->len >= SHORT_LEN) return -1;
  int qb = s->qbeg, qe = s->qbeg + s->len;
  int64_t rb = s->rbeg, re = s->rbeg + s->len;
  const int64_t mid = (rb + re) >> 1;
  qb -= SHORT_EXT; qb = qb > 0 ? qb : 0;
  qe += SHORT_EXT; qe = qe < l_query ? qe : l_query;
  rb -= SHORT_EXT; rb = rb > 0 ? rb : 0;
  re += SHORT_EXT; re = re < l_pac << 1 ? re : l_pac << 1;
  if (rb < l_pac && l_pac < re) {
    if (mid < l_pac) re = l_pac;
    else rb = l_pac;
  }
  if (qe - qb >= SHORT_LEN || re - rb >= SHORT_LEN) return -1;
  /* bns_fetch_seq (bntseq.c:421-446): clip to the contig holding mid */
  {
    const int is_rev = mid >= l_pac;
    const int rid = pos2rid(bns, depos(l_pac, mid));
    int64_t fb = bns->ann_offset[rid], fe = fb + bns->ann_len[rid];
    if (is_rev) {
      const int64_t t = fb;
      fb = (l_pac << 1) - fe;
      fe = (l_pac << 1) - t;
    }
    rb = rb > fb ? rb : fb;
    re = re < fe ? re : fe;
  }
  uint8_t rseq[SHORT_LEN];
  oracle_get_window(l_pac, pac, rb, re, rseq);
  bwagpu_kswr_t x;
  oracle_ksw_align2(qe - qb, query + qb, (int)(re - rb), rseq, opt->mat, opt->o_del, opt->e_del, opt->o_ins,
                    opt->e_ins, BWAGPU_KSW_XSTART, &x, 0);
  return x.score;
}

/* mem_flt_chained_seeds, bwamem.c:607-624 */
static void flt_chained_seeds(const bwagpu_opt_t *opt, const oracle_chainopt_t *o, const bwagpu_bns_t *bns,
                              const uint8_t *pac, int l_query, const uint8_t *query, int n_chn, cp_t *a)
{
  const double min_l = o->min_chain_weight ? 1.1f * o->min_chain_weight : 5.5f * log(l_query);
  const int min_HSP_score = (int)(opt->a * min_l + .499);
  if (min_l > 0.05f * l_query) return;
  for (int i = 0; i < n_chn; ++i) {
    ch_t *c = a[i];
    int j, k;
    for (j = k = 0; j < c->n; ++j) {
      bwagpu_seed_t *s = &c->s[j];
      s->score = seed_sw(opt, bns, pac, l_query, query, s);
      if (s->score < 0 || s->score >= min_HSP_score) {
        s->score = s->score < 0 ? s->len * opt->a : s->score;
        c->s[k++] = *s;
      }
    }
    c->n = k;
  }
}

static void emit(ch_t *c, float frac_rep, oracle_chains_t *out)
{
  if (out->n_chains < out->cap_chains) {
    bwagpu_chain_t *d = &out->chains[out->n_chains];
    d->pos = c->pos;
    d->rid = c->rid;
    d->n = c->n;
    d->w = c->w;
    d->kept = c->kept;
    d->first = c->first;
    d->is_alt = c->is_alt;
    d->frac_rep = frac_rep;
    d->pad_ = 0;
  }
  for (int j = 0; j < c->n; ++j) {
    if (out->n_seeds + j < out->cap_seeds) out->seeds[out->n_seeds + j] = c->s[j];
  }
  out->n_seeds += c->n;
  ++out->n_chains;
}

/* one read: mem_chain's body (raw != 0: stop there, chains in traversal
   order with w/kept/first unset) or the whole SeqsToChains chaining */
static void chain_read(const oracle_chain_env_t *env, int len, const uint8_t *seq, int raw, oracle_chains_t *out)
{
  const oracle_chainopt_t *o = env->copt;
  const int64_t l_pac = env->bns->l_pac;
  if (len < o->min_seed_len) return;
  int cap = 64;
  uint64_t *iv = (uint64_t *)malloc(sizeof(uint64_t) * 4 * (size_t)cap);
  int n_iv = oracle_collect_intv(env->bwt_hdr, env->bwt_words, env->seedopt, env->split_factor, len, seq, iv, cap);
  if (n_iv > cap) {
    cap = n_iv;
    iv = (uint64_t *)realloc(iv, sizeof(uint64_t) * 4 * (size_t)cap);
    oracle_collect_intv(env->bwt_hdr, env->bwt_words, env->seedopt, env->split_factor, len, seq, iv, cap);
  }
  int i, b, e, l_rep;
  for (i = 0, b = e = l_rep = 0; i < n_iv; ++i) { /* frac_rep, bwamem.c:277-283 */
    const uint64_t *p = iv + 4 * i;
    const int sb = (int)(p[3] >> 32), se = (int)(uint32_t)p[3];
    if (p[2] <= (uint64_t)o->max_occ) continue;
    if (sb > e) l_rep += e - b, b = sb, e = se;
    else e = e > se ? e : se;
  }
  l_rep += e - b;
  int n_ch = 0, cap_ch = 16;
  ch_t *ch = (ch_t *)malloc(sizeof(ch_t) * (size_t)cap_ch);
  tree_t t = {new_node(0), 0, 0};
  for (i = 0; i < n_iv; ++i) {
    const uint64_t *p = iv + 4 * i;
    const int slen = (int)((uint32_t)p[3] - (p[3] >> 32));
    const int step = p[2] > (uint64_t)o->max_occ ? (int)(p[2] / (uint64_t)o->max_occ) : 1;
    int64_t k;
    int count;
    for (k = count = 0; (uint64_t)k < p[2] && count < o->max_occ; k += step, ++count) {
      bwagpu_seed_t s;
      s.rbeg = (int64_t)oracle_bwt_sa(env->bwt_hdr, env->bwt_words, env->sa, env->sa_intv, p[0] + (uint64_t)k);
      s.qbeg = (int32_t)(p[3] >> 32);
      s.score = s.len = slen;
      s.pad_ = 0;
      const int rid = intv2rid(env->bns, s.rbeg, s.rbeg + s.len);
      if (rid < 0) continue;
      int add = 1;
      if (t.n_keys) {
        t.c = ch;
        const int lo = lower_of(&t, s.rbeg);
        if (lo >= 0 && merge(env->opt->w, o->max_chain_gap, l_pac, &ch[lo], &s, rid)) add = 0;
      }
      if (add) {
        if (n_ch == cap_ch) {
          cap_ch <<= 1;
          ch = (ch_t *)realloc(ch, sizeof(ch_t) * (size_t)cap_ch);
        }
        ch_t *c = &ch[n_ch];
        memset(c, 0, sizeof *c);
        c->pos = s.rbeg;
        c->rid = rid;
        c->is_alt = env->is_alt ? !!env->is_alt[rid] : 0;
        c->first = -1;
        ch_push(c, &s);
        t.c = ch;
        put(&t, n_ch++);
      }
    }
  }
  free(iv);
  int *order = (int *)malloc(sizeof(int) * (size_t)(n_ch > 0 ? n_ch : 1)), n_ord = 0;
  traverse(t.root, order, &n_ord);
  free_tree(t.root);
  const float frac_rep = (float)l_rep / len;
  cp_t *a = (cp_t *)malloc(sizeof(cp_t) * (size_t)(n_ch > 0 ? n_ch : 1));
  for (i = 0; i < n_ord; ++i) a[i] = &ch[order[i]];
  int n = n_ord;
  if (!raw) {
    n = chain_flt(o, n, a);
    flt_chained_seeds(env->opt, o, env->bns, env->pac, len, seq, n, a);
  }
  for (i = 0; i < n; ++i) emit(a[i], frac_rep, out);
  for (i = 0; i < n_ch; ++i) free(ch[i].s);
  free(ch);
  free(order);
  free(a);
}

int oracle_seqs2chains(const oracle_chain_env_t *env, int32_t n_reads, const int64_t *seq_off, const uint8_t *seq,
                       int raw, int32_t *read_chain_off, oracle_chains_t *out)
{
  out->n_chains = 0;
  out->n_seeds = 0;
  read_chain_off[0] = 0;
  for (int32_t r = 0; r < n_reads; ++r) {
    chain_read(env, (int)(seq_off[r + 1] - seq_off[r]), seq + seq_off[r], raw, out);
    read_chain_off[r + 1] = out->n_chains;
  }
  return out->n_chains <= out->cap_chains && out->n_seeds <= out->cap_seeds ? 0 : 1;
}
