/*
 * fpga_stream.c — TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * The FPGA back end's wire format, restated:
 *   oracle_fpga_pack  packReadData + getChainRef (src/fpga/FPGAPipeline.cpp:
 *                     143-192, 194-343) with bns_fetch_seq_fpga's window clip
 *                     (src/bwa_wrapper.cpp:790-809) — the input stream of
 *                     sw_top;
 *   oracle_fpga_sw    what bwagpu_sw_stream must return for such a stream:
 *                     every task one seed extended as mem_chain2aln extends a
 *                     seed (bwa/bwamem.c:717-792, oracle_seed_extend) in its
 *                     chain's window, written as the per-task record
 *                     processOutput reads (FPGAPipeline.cpp:90-105).
 * The FPGA kernel itself (src/fpga/kernel/smithwaterman.cpp) is not the
 * semantics here: it has no z-drop and fixed scoring;
 * the records carry bwa's own extension, so processOutput rebuilds the region
 * mem_chain2aln would build for that seed.
 */
#include <stdlib.h>
#include <string.h>
#include "oracle.h"

#define MAX_CHAINS_PACKED 2000 /* FPGAPipeline.cpp:208 */

static void put32(int32_t *out, int64_t at, int32_t v) { out[at] = v; }
static void put64(int32_t *out, int64_t at, int64_t v)
{ /* *(int64_t *)&buffer[4 at] on a little-endian host */
  out[at] = (int32_t)(uint32_t)(uint64_t)v;
  out[at + 1] = (int32_t)(uint32_t)((uint64_t)v >> 32);
}
static int64_t get64(const int32_t *in, int64_t at)
{
  return (int64_t)((uint64_t)(uint32_t)in[at] | (uint64_t)(uint32_t)in[at + 1] << 32);
}

/* bns_pos2rid (bwa/bntseq.c:370-385): the last contig starting at or before pos_f */
static int pos2rid(const bwagpu_bns_t *bns, int64_t pos_f)
{
  int lo = 0, hi = bns->n_seqs - 1;
  if (pos_f >= bns->l_pac) return -1;
  while (lo < hi) {
    int mid = (lo + hi + 1) >> 1;
    if (bns->ann_offset[mid] <= pos_f) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

/* getChainRef's window for one chain (FPGAPipeline.cpp:158-190) */
static void chain_window(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, int lq, const bwagpu_seed_t *sd, int ns,
                         int64_t *lo_, int64_t *hi_)
{
  const int64_t l_pac = bns->l_pac, two = l_pac << 1;
  int64_t lo = two, hi = 0, mid, pos_f, fb, fe;
  int i, rid, is_rev;
  for (i = 0; i < ns; ++i) {
    const bwagpu_seed_t *t = &sd[i];
    int64_t b = t->rbeg - (t->qbeg + oracle_max_gap_len(opt, t->qbeg));
    int tail = lq - t->qbeg - t->len;
    int64_t e = t->rbeg + t->len + (tail + oracle_max_gap_len(opt, tail));
    if (b < lo) lo = b;
    if (e > hi) hi = e;
  }
  if (lo < 0) lo = 0;
  if (hi > two) hi = two;
  if (lo < l_pac && l_pac < hi) {
    if (sd[0].rbeg < l_pac) hi = l_pac;
    else lo = l_pac;
  }
  /* bns_fetch_seq_fpga: clip to the contig of the first seed */
  mid = sd[0].rbeg;
  is_rev = mid >= l_pac;
  pos_f = is_rev ? two - 1 - mid : mid;
  rid = pos2rid(bns, pos_f);
  if (rid >= 0) {
    fb = bns->ann_offset[rid];
    fe = fb + bns->ann_len[rid];
    if (is_rev) { int64_t t0 = fb; fb = two - fe; fe = two - t0; }
    if (lo < fb) lo = fb;
    if (hi > fe) hi = fe;
  }
  *lo_ = lo;
  *hi_ = hi;
}

int64_t oracle_fpga_pack(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const bwagpu_batch_t *b, int32_t *out,
                         int64_t cap_words, int32_t cap_tasks, int32_t *n_tasks, int32_t *packed, int32_t *task_seed)
{
  int64_t p = 0;
  int32_t nt = 0;
  for (int r = 0; r < b->n_reads; ++r) {
    const int c0 = b->read_chain_off[r], nch = b->read_chain_off[r + 1] - c0;
    const int lq = (int)(b->seq_off[r + 1] - b->seq_off[r]);
    const uint8_t *q = b->seq + b->seq_off[r];
    const int total = b->chain_seed_off[c0 + nch] - b->chain_seed_off[c0];
    int64_t need = 4 + (lq + 7) / 8 + 5 * (int64_t)nch + 5 * (int64_t)total, at_end, at_nch;
    packed[r] = 0;
    if (nch == 0 || total == 0 || nch >= MAX_CHAINS_PACKED) continue;
    if (p + need > cap_words) return -1;
    packed[r] = 1;
    at_end = p++;
    put32(out, p++, lq);
    { /* 8 bases per word, 4 bits each, first base in the high nibble */
      uint32_t w = 0;
      int i;
      for (i = 0; i < lq; ++i) {
        w = w << 4 | q[i];
        if ((i & 7) == 7) { put32(out, p++, (int32_t)w); w = 0; }
      }
      if (lq & 7) put32(out, p++, (int32_t)(w << (4 * (8 - (lq & 7)))));
    }
    at_nch = p++;
    for (int c = c0; c < c0 + nch; ++c) {
      const bwagpu_seed_t *sd = b->seeds + b->chain_seed_off[c];
      const int ns = b->chain_seed_off[c + 1] - b->chain_seed_off[c];
      int64_t lo = 0, hi = 0, at_ns;
      int n_put = 0;
      if (ns) chain_window(opt, bns, lq, sd, ns, &lo, &hi);
      put64(out, p, lo);
      put64(out, p + 2, hi);
      p += 4;
      at_ns = p++;
      for (int k = ns - 1; k >= 0; --k) { /* FPGAPipeline.cpp:296-331 */
        const bwagpu_seed_t *s = &sd[k];
        if (!(s->qbeg > 0 || s->qbeg + s->len != lq)) continue; /* the whole read: no task */
        if (nt >= cap_tasks) return -1;
        if (task_seed) task_seed[nt] = b->chain_seed_off[c] + k;
        put32(out, p, nt++);
        put64(out, p + 1, s->rbeg);
        put32(out, p + 3, s->qbeg);
        put32(out, p + 4, s->len);
        p += 5;
        ++n_put;
      }
      put32(out, at_ns, n_put);
    }
    put32(out, at_nch, nch);
    put32(out, at_end, (int32_t)p);
  }
  *n_tasks = nt;
  return p;
}

int oracle_fpga_sw(const bwagpu_opt_t *opt, const bwagpu_bns_t *bns, const uint8_t *pac, const int32_t *in,
                   int64_t n_words, int16_t *out, int32_t cap_tasks, int32_t *n_tasks)
{
  const int64_t two = bns->l_pac << 1;
  uint8_t q[BWAGPU_MAX_READ_LEN + 1], qrev[BWAGPU_MAX_READ_LEN + 1];
  uint8_t *seen = (uint8_t *)calloc((size_t)cap_tasks + 1, 1);
  int32_t nt = 0, n_max = 0;
  int bad = 0;
  int64_t p = 0;
  while (p < n_words && !bad) {
    const int64_t end = in[p];
    int lq, nch, i;
    int64_t c;
    if (end <= p + 2 || end > n_words) { bad = 1; break; }
    lq = in[p + 1];
    if (lq < 0 || lq > BWAGPU_MAX_READ_LEN || p + 3 + (lq + 7) / 8 > end) { bad = 1; break; }
    for (i = 0; i < lq; ++i) {
      q[i] = (uint8_t)((uint32_t)in[p + 2 + i / 8] >> (28 - 4 * (i & 7)) & 15);
      if (q[i] > 4) bad = 1;
    }
    c = p + 2 + (lq + 7) / 8;
    nch = in[c++];
    for (int ch = 0; ch < nch && !bad; ++ch) {
      int64_t lo, hi;
      int ns;
      uint8_t *win, *trev;
      if (c + 5 > end) { bad = 1; break; }
      lo = get64(in, c);
      hi = get64(in, c + 2);
      ns = in[c + 4];
      c += 5;
      if (ns < 0 || c + 5 * (int64_t)ns > end) { bad = 1; break; }
      if (ns == 0) continue;
      if (lo < 0 || hi > two || lo > hi || (lo < bns->l_pac && bns->l_pac < hi)) { bad = 1; break; }
      win = (uint8_t *)malloc((size_t)(hi - lo) + 1);
      trev = (uint8_t *)malloc((size_t)(hi - lo) + 1);
      oracle_get_window(bns->l_pac, pac, lo, hi, win);
      for (int k = 0; k < ns && !bad; ++k, c += 5) {
        const int32_t t = in[c];
        bwagpu_seed_t s;
        bwagpu_alnreg_t a;
        int64_t cells[2] = {0, 0}, calls = 0;
        int16_t *o;
        s.rbeg = get64(in, c + 1);
        s.qbeg = in[c + 3];
        s.len = in[c + 4];
        s.score = s.pad_ = 0;
        if (t < 0 || t >= cap_tasks || seen[t]) { bad = 1; break; }
        if (s.qbeg < 0 || s.len <= 0 || s.qbeg + s.len > lq || s.rbeg < lo || s.rbeg + s.len > hi) { bad = 1; break; }
        seen[t] = 1;
        ++nt;
        if (t + 1 > n_max) n_max = t + 1;
        memset(&a, 0, sizeof a);
        oracle_seed_extend(opt, lq, q, &s, lo, hi, win, qrev, trev, &a, cells, &calls);
        o = out + 10 * (int64_t)t;
        o[0] = (int16_t)(t & 0xffff);
        o[1] = (int16_t)(t >> 16);
        o[2] = (int16_t)a.qb;
        o[3] = (int16_t)(a.qe - (s.qbeg + s.len));
        o[4] = (int16_t)(a.rb - s.rbeg);
        o[5] = (int16_t)(a.re - (s.rbeg + s.len));
        o[6] = (int16_t)a.score;
        o[7] = (int16_t)a.truesc;
        o[8] = (int16_t)a.w;
        o[9] = 0;
      }
      free(win);
      free(trev);
    }
    if (!bad && c != end) bad = 1;
    p = end;
  }
  free(seen);
  if (!bad && nt != n_max) bad = 1; /* processOutput: total == max index + 1 (FPGAPipeline.cpp:54) */
  *n_tasks = bad ? 0 : nt;
  return bad ? -1 : 0;
}
