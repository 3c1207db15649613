// seed.hip — seeding's interval collection on the device: mem_collect_intv
// (bwa/bwamem.c:120-167) for every read of a batch.
//
// One lane per read.  The work is a chain of dependent FM-index lookups — each
// bwt_extend is two occurrence-block reads of 64 bytes at data-dependent
// positions — so the kernel is bound by memory latency, not by ALU or HBM
// bandwidth: it keeps as many reads in flight as the device holds lanes, and
// each lookup is one 64-byte block fetched with four 16-byte loads issued
// together.  The occurrence counts are computed in registers (three
// equality-popcounts per 2-bit base word; A from the position count) instead
// of bwa's 256-entry byte table.  The intermediate interval lists live in a
// per-read scratch region of global memory (L1/L2 resident while a read works
// on them); the read's own intervals are built in its output slots and sorted
// there with klib's introsort restated step for step (the order of intervals
// with equal info is the algorithm's).
#include <hip/hip_runtime.h>
#include <stdlib.h>

#include "seed.h"

namespace bwagpu {
namespace {

struct Ivl {
  uint64_t x[3], info;
};
static_assert(sizeof(Ivl) == sizeof(bwagpu_intv_t), "interval layout");

// ---- occurrence counting on the device layout
// bwa's interleaved array (bwt.h:46-57) stores, per 128 positions, four
// uint64 counts and 8 words of 2-bit bases: 64 B fetched and 8 words counted
// per lookup.  bwagpu_set_bwt re-lays it out once (build_occ64_kernel): per
// 64 positions one 32-byte record {uint32 count of A/C/G/T before the block,
// relative to its 2^32-position superblock (sup_shift); 4 words of bases}, plus 4 uint64
// counts per superblock.  A lookup is one 32-byte fetch and 4 words counted
// (three equality-popcounts each, A from the position count); the counts are
// bwa's exactly (bwt_occ4, bwt.c:169-187).
__device__ __forceinline__ void block_counts64(uint64_t k, const uint4 hdr, const uint4 w4, const uint64_t* sup,
                                               int sup_shift, uint64_t cnt[4]) {
  const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
  const int nfull = (int)((k & 63) >> 4);
  const uint32_t tail = ~((1u << ((~(uint32_t)k & 15) << 1)) - 1);  // fields 0..(k & 15) of word nfull
  uint32_t c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = (i < nfull ? 0xffffffffu : i == nfull ? tail : 0u) & 0x55555555u;
    const uint32_t x1 = w[i] ^ 0x55555555u, x2 = w[i] ^ 0xaaaaaaaau, x3 = ~w[i];
    c1 += __popc(~(x1 | x1 >> 1) & m);
    c2 += __popc(~(x2 | x2 >> 1) & m);
    c3 += __popc(~(x3 | x3 >> 1) & m);
  }
  const uint32_t c0 = (uint32_t)(k & 63) + 1 - c1 - c2 - c3;
  const uint64_t* sp = sup + 4 * (k >> sup_shift);
  cnt[0] = sp[0] + hdr.x + c0;
  cnt[1] = sp[1] + hdr.y + c1;
  cnt[2] = sp[2] + hdr.z + c2;
  cnt[3] = sp[3] + hdr.w + c3;
}

// bwt_occ4 (bwt.c:169-187): occurrences of A/C/G/T in bwt[0..k], $ removed
__device__ __forceinline__ void occ4(const DevBwt& b, uint64_t k, uint64_t cnt[4]) {
  if (k == ~0ull) {
    cnt[0] = cnt[1] = cnt[2] = cnt[3] = 0;
    return;
  }
  k -= (k >= b.primary);
  const uint4* p = b.occ + 2 * (k >> 6);
  block_counts64(k, p[0], p[1], b.sup, b.sup_shift, cnt);
}

// bwt_2occ4 (bwt.c:189-214): both ends of an interval; when they fall in the
// same block it is fetched once (the second fetch is issued only by the lanes
// whose ends lie in different blocks)
__device__ __forceinline__ void occ4x2(const DevBwt& b, uint64_t k, uint64_t l, uint64_t tk[4], uint64_t tl[4]) {
  if (k == ~0ull || l == ~0ull) {
    occ4(b, k, tk);
    occ4(b, l, tl);
    return;
  }
  const uint64_t kk = k - (k >= b.primary), ll = l - (l >= b.primary);
  const uint4* pk = b.occ + 2 * (kk >> 6);
  const uint4 a0 = pk[0], a1 = pk[1];
  uint4 d0 = a0, d1 = a1;
  if ((kk >> 6) != (ll >> 6)) {
    const uint4* pl = b.occ + 2 * (ll >> 6);
    d0 = pl[0];
    d1 = pl[1];
  }
  block_counts64(kk, a0, a1, b.sup, b.sup_shift, tk);
  block_counts64(ll, d0, d1, b.sup, b.sup_shift, tl);
}

// bwt_B0 (bwt.h:86): the base at $-free position x
__device__ __forceinline__ int base_at(const DevBwt& b, uint64_t x) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(b.occ + 2 * (x >> 6) + 1);
  return (int)(w[(x & 63) >> 4] >> ((~x & 15) << 1) & 3);
}

// one lane per 64-position block: its record from bwa's array (the bwa block
// header's counts + the bases of the block's first half before it)
__global__ void __launch_bounds__(256) build_occ64_kernel(DevBwt b, uint4* __restrict__ occ, uint64_t* __restrict__ sup,
                                                          uint64_t n_blocks, uint64_t n_sup) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_sup) {  // superblock s starts at position s << sup_shift, a bwa block boundary
    const uint64_t pos = i << b.sup_shift;
    const uint64_t* hb = reinterpret_cast<const uint64_t*>(b.bwt + ((pos >> 7) << 4));
    for (int c = 0; c < 4; ++c) sup[4 * i + c] = pos < b.seq_len ? hb[c] : 0;
  }
  if (i >= n_blocks) return;
  const uint64_t pos = i << 6;  // first position of the block
  if (pos >= b.seq_len) return;  // (the spare record is never read)
  const uint32_t* bb = b.bwt + ((pos >> 7) << 4);
  const uint64_t* hb = reinterpret_cast<const uint64_t*>(bb);
  const uint64_t* hs = reinterpret_cast<const uint64_t*>(b.bwt + (((pos >> b.sup_shift) << b.sup_shift >> 7) << 4));
  uint64_t cnt[4] = {hb[0], hb[1], hb[2], hb[3]};
  const int half = (int)((pos >> 6) & 1);
  const uint32_t* w = bb + 8 + 4 * half;
  if (half) {  // the block's first 64 bases (words 0-3) come before it
    for (int j = 0; j < 4; ++j) {
      const uint32_t v = bb[8 + j];
      const uint32_t x1 = v ^ 0x55555555u, x2 = v ^ 0xaaaaaaaau, x3 = ~v;
      const uint32_t n1 = __popc(~(x1 | x1 >> 1) & 0x55555555u), n2 = __popc(~(x2 | x2 >> 1) & 0x55555555u),
                     n3 = __popc(~(x3 | x3 >> 1) & 0x55555555u);
      cnt[0] += 16 - n1 - n2 - n3;
      cnt[1] += n1;
      cnt[2] += n2;
      cnt[3] += n3;
    }
  }
  uint4 hdr;
  hdr.x = (uint32_t)(cnt[0] - hs[0]);
  hdr.y = (uint32_t)(cnt[1] - hs[1]);
  hdr.z = (uint32_t)(cnt[2] - hs[2]);
  hdr.w = (uint32_t)(cnt[3] - hs[3]);
  occ[2 * i] = hdr;
  occ[2 * i + 1] = make_uint4(w[0], w[1], w[2], w[3]);
}

// bwt_extend (bwt.c:262-276)
__device__ __forceinline__ void extend(const DevBwt& b, const Ivl& ik, Ivl ok[4], int is_back) {
  uint64_t tk[4], tl[4];
  const int nb = !is_back;
  occ4x2(b, ik.x[nb] - 1, ik.x[nb] - 1 + ik.x[2], tk, tl);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ok[i].x[nb] = b.L2[i] + 1 + tk[i];
    ok[i].x[2] = tl[i] - tk[i];
    ok[i].info = 0;
  }
  ok[3].x[is_back] = ik.x[is_back] + (ik.x[nb] <= b.primary && ik.x[nb] + ik.x[2] - 1 >= b.primary);
  ok[2].x[is_back] = ok[3].x[is_back] + ok[3].x[2];
  ok[1].x[is_back] = ok[2].x[is_back] + ok[2].x[2];
  ok[0].x[is_back] = ok[1].x[is_back] + ok[1].x[2];
}

// bwt_extend's interval for one base c only (ok[c] of bwt.c:262-276).  The
// callers index ok[] with a per-lane base, which would put the 4-entry array
// in scratch memory; here the entry is picked with selects instead.
__device__ __forceinline__ Ivl extend1(const DevBwt& b, const Ivl& ik, int c, int is_back) {
  uint64_t tk[4], tl[4];
  const int nb = !is_back;
  occ4x2(b, ik.x[nb] - 1, ik.x[nb] - 1 + ik.x[2], tk, tl);
  const uint64_t s0 = tl[0] - tk[0], s1 = tl[1] - tk[1], s2 = tl[2] - tk[2], s3 = tl[3] - tk[3];
  const uint64_t tkc = c == 0 ? tk[0] : c == 1 ? tk[1] : c == 2 ? tk[2] : tk[3];
  const uint64_t l2c = c == 0 ? b.L2[0] : c == 1 ? b.L2[1] : c == 2 ? b.L2[2] : b.L2[3];
  const uint64_t sc = c == 0 ? s0 : c == 1 ? s1 : c == 2 ? s2 : s3;
  // ok[c].x[is_back] = ok[3].x[is_back] + sizes of the bases above c (bwt.c:272-275)
  const uint64_t above = (c < 3 ? s3 : 0) + (c < 2 ? s2 : 0) + (c < 1 ? s1 : 0);
  Ivl o;
  o.x[nb] = l2c + 1 + tkc;
  o.x[2] = sc;
  o.x[is_back] = ik.x[is_back] + (ik.x[nb] <= b.primary && ik.x[nb] + ik.x[2] - 1 >= b.primary) + above;
  o.info = 0;
  return o;
}

__device__ __forceinline__ uint64_t l2_at(const DevBwt& b, int i) {  // L2[i] by selects, not a scratch copy
  // (the empty asm keeps the compiler from turning the selects back into an
  // indexed copy of the kernel argument in scratch memory)
  uint64_t l0 = b.L2[0], l1 = b.L2[1], l2 = b.L2[2], l3 = b.L2[3], l4 = b.L2[4];
  asm volatile("" : "+s"(l0), "+s"(l1), "+s"(l2), "+s"(l3), "+s"(l4));
  return i == 0 ? l0 : i == 1 ? l1 : i == 2 ? l2 : i == 3 ? l3 : l4;
}

// bwt_extend's ok[c] in the backward form (is_back = 1; a forward extension
// runs on the swapped interval), counting only what ok[c] needs: the
// occurrences of c at both ends and those of the bases above c (bwt.c:
// 272-275 sums their sizes) — an equality and a comparison popcount per word
// instead of three equality ones, 32-bit arithmetic inside a superblock, and
// the superblock table read only when the BWT has positions past 2^32.
// Intervals always start at row >= 1 (set_intv and every extension give
// L2[c] + 1 + ...), so k = x[0] - 1 is never bwt_occ's (bwtint_t)-1.
struct CountsC {
  uint32_t eq, gt;  // occurrences of c / of bases above c in [superblock start, position]
};
__device__ __forceinline__ CountsC counts_c(uint64_t k, const uint4 hdr, const uint4 w4, uint32_t pe_hi, uint32_t pe_lo,
                                            uint32_t g_or, uint32_t g_lo, int c) {
  const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
  const int nfull = (int)((k & 63) >> 4);
  const uint32_t tail = ~((1u << ((~(uint32_t)k & 15) << 1)) - 1);
  uint32_t eq = c == 0 ? hdr.x : c == 1 ? hdr.y : c == 2 ? hdr.z : hdr.w;
  uint32_t gt = (c < 1 ? hdr.y : 0u) + (c < 2 ? hdr.z : 0u) + (c < 3 ? hdr.w : 0u);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t m = (i < nfull ? 0xffffffffu : i == nfull ? tail : 0u) & 0x55555555u;
    const uint32_t hi = (w[i] >> 1) & m, lo = w[i] & m;
    eq += __popc(~((hi ^ pe_hi) | (lo ^ pe_lo)) & m);  // fields equal to c
    gt += __popc((hi & (lo | g_or)) | (lo & g_lo));    // fields above c
  }
  return CountsC{eq, gt};
}

// the superblock's counts of c and of the bases above c (zero below 2^32)
__device__ __forceinline__ void sup_c(const DevBwt& b, uint64_t k, int c, uint64_t& eq, uint64_t& gt) {
  const ulonglong2* sp = reinterpret_cast<const ulonglong2*>(b.sup + 4 * (k >> b.sup_shift));
  const ulonglong2 s01 = sp[0], s23 = sp[1];
  eq = c == 0 ? s01.x : c == 1 ? s01.y : c == 2 ? s23.x : s23.y;
  gt = (c < 1 ? s01.y : 0ull) + (c < 2 ? s23.x : 0ull) + (c < 3 ? s23.y : 0ull);
}

// extend_c in two halves, so that a caller can issue other loads between the
// fetch of the occurrence records and the first use of their data
struct OccRecs {
  uint64_t kk, ll;
  uint4 a0, a1, d0, d1;
};
__device__ __forceinline__ OccRecs extend_fetch(const DevBwt& b, const Ivl& ik) {
  OccRecs o;
  const uint64_t k = ik.x[0] - 1, l = k + ik.x[2];
  o.kk = k - (k >= b.primary);
  o.ll = l - (l >= b.primary);
  const uint4* pk = b.occ + 2 * (o.kk >> 6);
  o.a0 = pk[0];
  o.a1 = pk[1];
  o.d0 = o.a0;
  o.d1 = o.a1;
  if ((o.kk >> 6) != (o.ll >> 6)) {  // the second block only when the ends do not share one
    const uint4* pl = b.occ + 2 * (o.ll >> 6);
    o.d0 = pl[0];
    o.d1 = pl[1];
  }
  return o;
}

__device__ __forceinline__ Ivl extend_finish(const DevBwt& b, const Ivl& ik, int c, const OccRecs& f) {
  const uint32_t pe_hi = (c & 2) ? 0x55555555u : 0u, pe_lo = (c & 1) ? 0x55555555u : 0u;
  // field > c: c = 0 -> hi | lo, 1 -> hi, 2 -> hi & lo, 3 -> none
  const uint32_t g_or = c <= 1 ? 0x55555555u : 0u, g_lo = c == 0 ? 0x55555555u : 0u;
  const uint32_t g_on = c == 3 ? 0u : 0xffffffffu;
  const CountsC ck = counts_c(f.kk, f.a0, f.a1, pe_hi, pe_lo, g_or, g_lo, c);
  const CountsC cl = counts_c(f.ll, f.d0, f.d1, pe_hi, pe_lo, g_or, g_lo, c);
  uint64_t tk = ck.eq, tl = cl.eq, gk = ck.gt & g_on, gl = cl.gt & g_on;
  if (b.seq_len >> b.sup_shift) {  // wave-uniform: the BWT has superblocks past the first
    uint64_t se, sg;
    sup_c(b, f.kk, c, se, sg);
    tk += se;
    gk += c == 3 ? 0ull : sg;
    sup_c(b, f.ll, c, se, sg);
    tl += se;
    gl += c == 3 ? 0ull : sg;
  }
  Ivl o;
  o.x[0] = l2_at(b, c) + 1 + tk;
  o.x[2] = tl - tk;
  o.x[1] = ik.x[1] + (ik.x[0] <= b.primary && ik.x[0] + ik.x[2] - 1 >= b.primary) + (gl - gk);
  o.info = 0;
  return o;
}

__device__ __forceinline__ Ivl extend_c(const DevBwt& b, const Ivl& ik, int c) {
  return extend_finish(b, ik, c, extend_fetch(b, ik));
}


__device__ __forceinline__ Ivl set_intv(const DevBwt& b, int c) {  // bwt.h:80
  Ivl ik;
  ik.x[0] = l2_at(b, c) + 1;
  ik.x[2] = l2_at(b, c + 1) - l2_at(b, c);
  ik.x[1] = l2_at(b, 3 - c) + 1;
  ik.info = 0;
  return ik;
}

struct List {
  Ivl* a;
  int n, cap;
  __device__ void push(const Ivl& v) {
    if (n < cap) a[n] = v;
    ++n;
  }
};

// tier 1 gives up on a read after this many bwt_extend calls (its wave would
// otherwise wait for the slowest lane); tier 2 redoes it wave-parallel
struct Budget {
  int left;
  __device__ bool spend() { return --left < 0; }
};

__device__ __forceinline__ void reverse(List& v) {
  for (int j = 0; j < v.n >> 1; ++j) {
    const Ivl t = v.a[v.n - 1 - j];
    v.a[v.n - 1 - j] = v.a[j];
    v.a[j] = t;
  }
}

// bwt_smem1a with max_intv = 0 (bwt.c:289-356)
__device__ int smem1(const DevBwt& b, int len, const uint8_t* q, int x, int min_intv, List& mem, List& prev,
                     List& curr, Budget& bg) {
  int i;
  mem.n = 0;
  if (q[x] > 3) return x + 1;
  if (min_intv < 1) min_intv = 1;
  Ivl ik = set_intv(b, q[x]);
  ik.info = (uint64_t)(x + 1);
  curr.n = 0;
  for (i = x + 1; i < len; ++i) {  // forward
    const int qi = q[i];
    if (qi < 4) {
      const int c = 3 - qi;
      if (bg.spend()) return -1;
      const Ivl okc = extend1(b, ik, c, 0);
      if (okc.x[2] != ik.x[2]) {
        curr.push(ik);
        if (okc.x[2] < (uint64_t)min_intv) break;
      }
      ik = okc;
      ik.info = (uint64_t)(i + 1);
    } else {
      curr.push(ik);
      break;
    }
  }
  if (i == len) curr.push(ik);
  reverse(curr);  // longest matches first
  const int ret = (int)curr.a[0].info;
  {  // the two lists trade places (values, not pointers: no addressable locals)
    const List t = curr;
    curr = prev;
    prev = t;
  }
  for (i = x - 1; i >= -1; --i) {  // backward
    const int c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
    curr.n = 0;
    Ivl pn{};
    if (prev.n > 0) pn = prev.a[0];
    for (int j = 0; j < prev.n; ++j) {
      const Ivl p = pn;
      if (j + 1 < prev.n) pn = prev.a[j + 1];  // the next candidate's load overlaps this extension
      Ivl okc{};
      if (c >= 0) {
        if (bg.spend()) return -1;
        okc = extend1(b, p, c, 1);
      }
      if (c < 0 || okc.x[2] < (uint64_t)min_intv) {
        if (curr.n == 0 && (mem.n == 0 || (uint64_t)(i + 1) < mem.a[mem.n - 1].info >> 32)) {
          Ivl h = p;
          h.info |= (uint64_t)(i + 1) << 32;
          mem.push(h);
        }
      } else if (curr.n == 0 || okc.x[2] != curr.a[curr.n - 1].x[2]) {
        okc.info = p.info;
        curr.push(okc);
      }
    }
    if (curr.n == 0) break;
    const List t2 = curr;
    curr = prev;
    prev = t2;
  }
  reverse(mem);  // by start
  return ret;
}

// bwt_seed_strategy1 (bwt.c:358-378)
template <class B>
__device__ int seed_strategy1(const DevBwt& b, int len, const uint8_t* q, int x, int min_len, int max_intv, Ivl& m,
                              B& bg) {
  m.x[0] = m.x[1] = m.x[2] = m.info = 0;
  if (q[x] > 3) return x + 1;
  Ivl ik = set_intv(b, q[x]);
  for (int i = x + 1; i < len; ++i) {
    const int qi = q[i];
    if (qi < 4) {
      const int c = 3 - qi;
      if (bg.spend()) return -1;
      const Ivl okc = extend1(b, ik, c, 0);
      if (okc.x[2] < (uint64_t)max_intv && i - x >= min_len) {
        m = okc;
        m.info = (uint64_t)x << 32 | (uint64_t)(i + 1);
        return i + 1;
      }
      ik = okc;
    } else {
      return i + 1;
    }
  }
  return len;
}

// klib's introsort by info (ksort.h:146-226, bwamem.c:90-91), step for step
__device__ __forceinline__ bool lt(const Ivl& a, const Ivl& b) { return a.info < b.info; }
__device__ __forceinline__ void swp(Ivl* a, int i, int j) {
  const Ivl t = a[i];
  a[i] = a[j];
  a[j] = t;
}
__device__ void insert_sort(Ivl* a, int s, int t) {  // [s, t)
  for (int i = s + 1; i < t; ++i)
    for (int j = i; j > s && lt(a[j], a[j - 1]); --j) swp(a, j, j - 1);
}
__device__ void comb_sort(Ivl* a, int n) {
  const double shrink = 1.2473309501039786540366528676643;
  int gap = n;
  bool swapped;
  do {
    if (gap > 2) {
      gap = (int)(gap / shrink);
      if (gap == 9 || gap == 10) gap = 11;
    }
    swapped = false;
    for (int i = 0; i < n - gap; ++i)
      if (lt(a[i + gap], a[i])) {
        swp(a, i, i + gap);
        swapped = true;
      }
  } while (swapped || gap > 2);
  if (gap != 1) insert_sort(a, 0, n);
}
__device__ void intro_sort(Ivl* a, int n) {
  if (n < 1) return;
  if (n == 2) {
    if (lt(a[1], a[0])) swp(a, 0, 1);
    return;
  }
  int d = 2;
  while ((1 << d) < n) ++d;
  struct Frame {
    int l, r, d;
  } stack[40];
  int top = 0, s = 0, t = n - 1;
  d <<= 1;
  for (;;) {
    if (s < t) {
      if (--d == 0) {
        comb_sort(a + s, t - s + 1);
        t = s;
        continue;
      }
      int i = s, j = t, k = i + ((j - i) >> 1) + 1;
      if (lt(a[k], a[i])) {
        if (lt(a[k], a[j])) k = j;
      } else {
        k = lt(a[j], a[i]) ? i : j;
      }
      const Ivl rp = a[k];
      if (k != t) swp(a, k, t);
      for (;;) {
        do ++i; while (lt(a[i], rp));
        do --j; while (i <= j && lt(rp, a[j]));
        if (j <= i) break;
        swp(a, i, j);
      }
      swp(a, i, t);
      if (i - s > t - i) {
        if (i - s > 16) stack[top++] = Frame{s, i - 1, d};
        s = t - i > 16 ? i + 1 : t;
      } else {
        if (t - i > 16) stack[top++] = Frame{i + 1, t, d};
        t = i - s > 16 ? i - 1 : s;
      }
    } else {
      if (top == 0) {
        insert_sort(a, 0, n);
        return;
      }
      --top;
      s = stack[top].l;
      t = stack[top].r;
      d = stack[top].d;
    }
  }
}

// ---- tier 1: two lanes per read, within an extension budget each
// The LAST-like pass does not read the first two passes' results, so it runs
// on a lane of its own (threads [n, 2n)) beside the SMEM + re-seeding lane
// (threads [0, n)); tier1_merge_kernel appends its intervals after theirs —
// mem_collect_intv's push order — and sorts.  A lane out of budget hands the
// whole read to tier 2 (the first of the two to give up lists it).
__global__ void __launch_bounds__(256) collect_intv_kernel(DevBwt b, SeedArgs a) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= 2 * a.n_reads) return;
  const bool last_like = t >= a.n_reads;
  const int r = last_like ? t - a.n_reads : t;
  const int64_t q0 = a.seq_off[r];
  const int len = (int)(a.seq_off[r + 1] - q0);
  const uint8_t* q = a.seq + q0;
  Ivl* base = reinterpret_cast<Ivl*>(a.scratch) + 4 * (q0 + 2 * (int64_t)r);
  Budget bg{a.budget};
  auto give_up = [&]() {  // tier 2 takes the read
    if (atomicCAS(a.flags + r, 0, 1) == 0) a.heavy[atomicAdd(a.n_heavy, 1)] = r;
  };
  if (last_like) {  // bwamem.c:150-165 into the read's fourth list
    List p3{base + 3 * (len + 2), 0, len + 2};
    if (a.max_mem_intv > 0) {
      int x = 0;
      while (x < len) {
        if (q[x] < 4) {
          Ivl m;
          x = seed_strategy1(b, len, q, x, a.min_seed_len, a.max_mem_intv, m, bg);
          if (x < 0) return give_up();
          if (m.x[2] > 0) p3.push(m);
        } else {
          ++x;
        }
      }
    }
    a.p3_n[r] = p3.n;
    return;
  }
  List la{base, 0, len + 2}, lb{base + (len + 2), 0, len + 2}, mem1{base + 2 * (len + 2), 0, len + 2};
  List mem{reinterpret_cast<Ivl*>(a.out) + (int64_t)r * a.max_per_read, 0, a.max_per_read};
  int x = 0;
  while (x < len) {  // SMEMs
    if (q[x] < 4) {
      x = smem1(b, len, q, x, 1, mem1, la, lb, bg);
      if (x < 0) return give_up();
      for (int i = 0; i < mem1.n; ++i)
        if ((int)((uint32_t)mem1.a[i].info - (uint32_t)(mem1.a[i].info >> 32)) >= a.min_seed_len) mem.push(mem1.a[i]);
    } else {
      ++x;
    }
  }
  const int old_n = min(mem.n, mem.cap);
  for (int k = 0; k < old_n; ++k) {  // re-seeding inside long SMEMs
    const Ivl p = mem.a[k];
    const int start = (int)(p.info >> 32), end = (int)(int32_t)p.info;
    if (end - start < a.split_len || p.x[2] > (uint64_t)a.split_width) continue;
    if (smem1(b, len, q, (start + end) >> 1, (int)(p.x[2] + 1), mem1, la, lb, bg) < 0) return give_up();
    for (int i = 0; i < mem1.n; ++i)
      if ((uint32_t)mem1.a[i].info - (uint32_t)(mem1.a[i].info >> 32) >= (uint32_t)a.min_seed_len) mem.push(mem1.a[i]);
  }
  a.out_n[r] = mem.n;  // passes 1-2; the merge adds pass 3 and sorts
}

// ---- tier 1, one extension per step: the same two lanes per read as
// collect_intv_kernel, written so that every iteration of a lane's loop is
// exactly one bwt_extend followed by a few lines of bookkeeping.  In the
// nested form (bwt_smem1a's forward loop, its backward rows, the loop over a
// row's items, mem_collect_intv's passes) the lanes of a wave sit in
// different loops, and a structured loop nest costs the slowest lane's trip
// count at every level.  Per-lane stamps (BWAGPU_SEED_DBG,
// tools_dev/seed_lanes.py) and tools_dev/micro/ext_{chain,real}.hip priced
// it: a lone wave's dependent fetch is 0.6 us, seed.hip's extension 1.2 us,
// a nested-form step 3.6 us.  Here the loop carries three intervals (the
// one being extended, the result, the next one fetched during this
// extension: the row's next item, or the next row's first item, which is
// the current row's first push), the base the next step needs is fetched
// during the extension too, and only the rare transitions (an SMEM's end or
// start, the forward walk's end, the passes) leave the common path.
// Results, push orders and the tier-2 hand-over rule are the nested
// kernel's exactly.
enum : int { kDone, kFwd, kBwd, kS1 };
enum : int { gNone, gFwdEnd, gSmemEnd, gNextSmem, gS1Next };

__device__ __forceinline__ void swap01(Ivl& v) {
  const uint64_t t = v.x[0];
  v.x[0] = v.x[1];
  v.x[1] = t;
}

__global__ void __launch_bounds__(256) collect_intv_step_kernel(DevBwt b, SeedArgs a) {
  const int t = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (t >= 2 * a.n_reads) return;
  const bool last_like = t >= a.n_reads;
  const int r = last_like ? t - a.n_reads : t;
  const int64_t q0 = a.seq_off[r];
  const int len = (int)(a.seq_off[r + 1] - q0);
  const uint8_t* q = a.seq + q0;
  Ivl* const base = reinterpret_cast<Ivl*>(a.scratch) + 4 * (q0 + 2 * (int64_t)r);
  const int lcap = len + 2;
  Ivl* const m1 = base + 2 * lcap;  // bwt_smem1a's own result list
  Ivl* const p3 = base + 3 * lcap;  // the LAST-like pass's list
  Ivl* const mem = reinterpret_cast<Ivl*>(a.out) + (int64_t)r * a.max_per_read;
  const int cap = a.max_per_read;
  int left = a.budget;
  const int64_t t_start = a.dbg ? (int64_t)wall_clock64() : 0;
  int n_steps = 0;

  int mode = kFwd;
  int pass = 1, x = 0, k = 0, old_n = 0, mem_n = 0, p3_n = 0;
  int x0 = 0, i = 0, min_intv = 1, ret = 0;
  int prv = 0, prev_n = 0, curr_n = 0, m1_n = 0, j = 0, qc = 4;  // qc: the base the next extension adds
  bool prev_rev = false;
  uint64_t last_sz = 0, m1_last = 0;
  Ivl cur{};

  // the rare transitions; on return mode is set for the next extension, or kDone
  auto rare = [&](int go) {
    while (go != gNone) {
      if (go == gFwdEnd) {  // bwt.c:318-324: the list reversed (walked from its end), the lists trade places
        prv ^= 1;
        prev_n = curr_n;
        prev_rev = true;
        curr_n = 0;
        j = 0;
        i = x0 - 1;
        qc = i >= 0 ? (int)q[i] : 4;
        if (qc > 3) {  // no extension: only the row's first item (cur, the last push) can reach mem
          if (m1_n == 0 || (uint64_t)(i + 1) < m1_last) {
            Ivl h = cur;
            h.info |= (uint64_t)(i + 1) << 32;
            m1[m1_n++] = h;
            m1_last = (uint64_t)(i + 1);
          }
          go = gSmemEnd;
        } else {
          mode = kBwd;
          go = gNone;
        }
      } else if (go == gSmemEnd) {  // bwt.c:352 (mem reversed) and mem_collect_intv's length filter
        for (int e = m1_n - 1; e >= 0; --e) {
          const Ivl v = m1[e];
          if ((int)((uint32_t)v.info - (uint32_t)(v.info >> 32)) >= a.min_seed_len) {
            if (mem_n < cap) mem[mem_n] = v;
            ++mem_n;
          }
        }
        if (pass == 1) x = ret;
        go = gNextSmem;
      } else if (go == gNextSmem) {  // mem_collect_intv's passes 1 and 2 (bwamem.c:128-149)
        int xs = -1, mi = 1;
        if (pass == 1) {
          while (x < len && q[x] > 3) ++x;
          if (x < len) {
            xs = x;
          } else {
            pass = 2;
            old_n = min(mem_n, cap);
            k = 0;
            n_steps = a.budget - left;  // (debug stamps: pass 1's share)
          }
        } else if (k >= old_n) {
          a.out_n[r] = mem_n;  // passes 1-2; the merge adds pass 3 and sorts
          mode = kDone;
          go = gNone;
        } else {
          const Ivl pk = mem[k++];
          const int start = (int)(pk.info >> 32), end = (int)(int32_t)pk.info;
          if (end - start >= a.split_len && pk.x[2] <= (uint64_t)a.split_width) {
            xs = (start + end) >> 1;
            mi = (int)(pk.x[2] + 1);
          }
        }
        if (xs >= 0) {  // bwt_smem1a's start (bwt.c:298-304)
          m1_n = 0;
          x0 = xs;
          const int c0 = q[xs];
          if (c0 > 3) {
            ret = xs + 1;
            go = gSmemEnd;
          } else {
            min_intv = mi < 1 ? 1 : mi;
            cur = set_intv(b, c0);
            cur.info = (uint64_t)(xs + 1);
            curr_n = 0;
            i = xs + 1;
            qc = i < len ? (int)q[i] : 4;
            if (qc > 3) {
              base[(prv ^ 1) * lcap] = cur;
              curr_n = 1;
              ret = (int)cur.info;
              go = gFwdEnd;
            } else {
              mode = kFwd;
              go = gNone;
            }
          }
        }
      } else {  // gS1Next: bwamem.c:150-165 around bwt_seed_strategy1 (bwt.c:358-378)
        if (a.max_mem_intv > 0)
          while (x < len && q[x] > 3) ++x;
        if (a.max_mem_intv <= 0 || x >= len) {
          a.p3_n[r] = p3_n;
          mode = kDone;
          go = gNone;
        } else {
          cur = set_intv(b, q[x]);
          x0 = x;
          i = x + 1;
          qc = i < len ? (int)q[i] : 4;
          if (qc > 3) {
            x = i < len ? i + 1 : len;
          } else {
            mode = kS1;
            go = gNone;
          }
        }
      }
    }
  };

  Ivl pre{};
  int go = last_like ? gS1Next : gNextSmem;
  for (;;) {
    if (go != gNone) rare(go);
    if (mode == kDone) break;
    const bool back = mode == kBwd;
    if (--left < 0) {  // tier 2 takes the read
      if (atomicCAS(a.flags + r, 0, 1) == 0) a.heavy[atomicAdd(a.n_heavy, 1)] = r;
      break;
    }
    // fetched during the extension: the base after this one, and (backward)
    // the row's next item or the next row's first one
    // (issued after the extension's fetch, unconditionally, from clamped
    // addresses, so that nothing waits for them before that fetch is out)
    Ivl in = cur;
    if (!back) swap01(in);
    const OccRecs recs = extend_fetch(b, in);
    const int qn_pos = back ? i - 1 : i + 1;
    const int qn_raw = q[min(max(qn_pos, 0), len - 1)];
    const int pre_at = j + 1 < prev_n ? prv * lcap + (prev_rev ? prev_n - 2 - j : j + 1) : (prv ^ 1) * lcap;
    pre = base[back ? pre_at : 0];
    Ivl res = extend_finish(b, in, back ? qc : 3 - qc, recs);
    if (!back) swap01(res);
    const int qn = qn_pos >= 0 && qn_pos < len ? qn_raw : 4;
    go = gNone;
    if (mode == kBwd) {  // bwt.c:327-349
      bool first_push = false;
      if (res.x[2] < (uint64_t)min_intv) {
        if (curr_n == 0 && (m1_n == 0 || (uint64_t)(i + 1) < m1_last)) {
          Ivl h = cur;
          h.info |= (uint64_t)(i + 1) << 32;
          m1[m1_n++] = h;
          m1_last = (uint64_t)(i + 1);
        }
      } else if (curr_n == 0 || res.x[2] != last_sz) {
        res.info = cur.info;
        base[(prv ^ 1) * lcap + curr_n] = res;
        first_push = curr_n == 0;
        ++curr_n;
        last_sz = res.x[2];
      }
      if (++j < prev_n) {
        cur = pre;
      } else if (curr_n == 0) {
        go = gSmemEnd;
      } else {  // the next row
        cur = first_push ? res : pre;
        prv ^= 1;
        prev_n = curr_n;
        prev_rev = false;
        curr_n = 0;
        j = 0;
        --i;
        qc = qn;
        if (qc > 3) {  // an ambiguous base or the read's start: as in rare(gFwdEnd)
          if (m1_n == 0 || (uint64_t)(i + 1) < m1_last) {
            Ivl h = cur;
            h.info |= (uint64_t)(i + 1) << 32;
            m1[m1_n++] = h;
            m1_last = (uint64_t)(i + 1);
          }
          go = gSmemEnd;
        }
      }
    } else if (mode == kFwd) {  // bwt.c:305-317
      if (res.x[2] != cur.x[2]) {
        base[(prv ^ 1) * lcap + curr_n++] = cur;
        ret = (int)cur.info;
        if (res.x[2] < (uint64_t)min_intv) go = gFwdEnd;
      }
      if (go == gNone) {
        cur = res;
        cur.info = (uint64_t)(i + 1);
        ++i;
        qc = qn;
        if (qc > 3) {  // an ambiguous base or the read's end
          base[(prv ^ 1) * lcap + curr_n++] = cur;
          ret = (int)cur.info;
          go = gFwdEnd;
        }
      }
    } else {  // kS1 (bwt.c:365-377)
      if (res.x[2] < (uint64_t)a.max_mem_intv && i - x0 >= a.min_seed_len) {
        if (res.x[2] > 0) {
          res.info = (uint64_t)x0 << 32 | (uint64_t)(i + 1);
          if (p3_n < lcap) p3[p3_n] = res;
          ++p3_n;
        }
        x = i + 1;
        go = gS1Next;
      } else {
        cur = res;
        ++i;
        qc = qn;
        if (qc > 3) {
          x = i < len ? i + 1 : len;
          go = gS1Next;
        }
      }
    }
  }
  if (a.dbg) {
    int64_t* d = a.dbg + 4 * (int64_t)t;
    d[0] = a.budget - left;
    d[1] = n_steps;
    d[2] = t_start;
    d[3] = (int64_t)wall_clock64();
  }
}

// tier 1's two halves of a read joined (bwamem.c:166: the sort of all)
__global__ void __launch_bounds__(256) tier1_merge_kernel(SeedArgs a) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads || a.flags[r]) return;
  const int64_t q0 = a.seq_off[r];
  const int len = (int)(a.seq_off[r + 1] - q0);
  const Ivl* p3 = reinterpret_cast<const Ivl*>(a.scratch) + 4 * (q0 + 2 * (int64_t)r) + 3 * (len + 2);
  List mem{reinterpret_cast<Ivl*>(a.out) + (int64_t)r * a.max_per_read, a.out_n[r], a.max_per_read};
  const int n3 = a.p3_n[r];
  for (int i = 0; i < n3; ++i) mem.push(p3[i]);
  if (mem.n <= mem.cap) {
    intro_sort(mem.a, mem.n);
    a.out_n[r] = mem.n;
  } else {
    a.out_n[r] = -mem.n;  // does not fit: flagged, left unsorted
  }
}

// ---- tier 2: one wave per read, the backward search lane-parallel
// Every scalar (interval under forward extension, list lengths, positions) is
// wave-uniform; list entries written by lane 0 (or by their owner lane) are
// published with a workgroup fence before other lanes read them.
struct NoBudget {
  __device__ bool spend() { return false; }
};

struct WList {
  Ivl* a;
  int n, cap;
  __device__ void push(const Ivl& v, bool lane0) {
    if (n < cap && lane0) a[n] = v;
    ++n;
  }
};

__device__ __forceinline__ void publish() { __threadfence_block(); }

__device__ __forceinline__ void wreverse(WList& v, int lane) {
  for (int j0 = 0; j0 < v.n >> 1; j0 += 64) {
    const int j = j0 + lane;
    const bool on = j < v.n >> 1;
    Ivl lo, hi;
    if (on) {
      lo = v.a[j];
      hi = v.a[v.n - 1 - j];
    }
    publish();
    if (on) {
      v.a[j] = hi;
      v.a[v.n - 1 - j] = lo;
    }
    publish();
  }
}

__device__ __forceinline__ uint64_t bperm64(int src_lane, uint64_t v) {
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)v);
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(uint32_t)(v >> 32));
  return (uint64_t)(uint32_t)hi << 32 | (uint32_t)lo;
}

// bwt_smem1a with max_intv = 0 (bwt.c:289-356), one wave
__device__ int smem1_wave(const DevBwt& b, int len, const uint8_t* q, int x, int min_intv, WList& mem, WList& prev,
                          WList& curr, int lane) {
  const bool l0 = lane == 0;
  int i;
  mem.n = 0;
  if (q[x] > 3) return x + 1;
  if (min_intv < 1) min_intv = 1;
  Ivl ik = set_intv(b, q[x]);
  ik.info = (uint64_t)(x + 1);
  curr.n = 0;
  for (i = x + 1; i < len; ++i) {  // forward: one interval, every lane alike
    const int qi = q[i];
    if (qi < 4) {
      const int c = 3 - qi;
      const Ivl okc = extend1(b, ik, c, 0);
      if (okc.x[2] != ik.x[2]) {
        curr.push(ik, l0);
        if (okc.x[2] < (uint64_t)min_intv) break;
      }
      ik = okc;
      ik.info = (uint64_t)(i + 1);
    } else {
      curr.push(ik, l0);
      break;
    }
  }
  if (i == len) curr.push(ik, l0);
  publish();
  wreverse(curr, lane);
  const int ret = (int)curr.a[0].info;
  {
    const WList t = curr;
    curr = prev;
    prev = t;
  }
  const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
  for (i = x - 1; i >= -1; --i) {  // backward: lane j extends prev[j]
    const int c = i < 0 ? -1 : q[i] < 4 ? q[i] : -1;
    curr.n = 0;
    bool have_last = false;  // a kept (pushed) entry exists in curr
    uint64_t last_sz = 0;
    for (int j0 = 0; j0 < prev.n; j0 += 64) {
      const int j = j0 + lane;
      const bool valid = j < prev.n;
      Ivl p{};
      if (valid) p = prev.a[j];
      Ivl okc{};
      if (valid && c >= 0) okc = extend1(b, p, c, 1);
      const bool A = valid && (c < 0 || okc.x[2] < (uint64_t)min_intv);
      const bool nA = valid && !A;
      // bwt.c:333-338: only entry 0 can reach mem (curr is empty before the
      // first non-A entry; after a push the containment test fails)
      if (j0 == 0) {
        const bool a0 = __builtin_amdgcn_readfirstlane((int)A) != 0;
        if (a0) {
          const Ivl p0 = prev.a[0];
          if (mem.n == 0 || (uint64_t)(i + 1) < mem.a[mem.n - 1].info >> 32) {
            Ivl h = p0;
            h.info |= (uint64_t)(i + 1) << 32;
            mem.push(h, l0);
            publish();
          }
        }
      }
      // bwt.c:339-342: a non-A entry is pushed unless its size equals the last
      // pushed one, i.e. that of the previous non-A entry
      const uint64_t nA_m = __builtin_amdgcn_ballot_w64(nA);
      const uint64_t prev_m = nA_m & below;
      const int pl = prev_m ? 63 - (int)__builtin_clzll(prev_m) : 0;
      const uint64_t psz = bperm64(pl, okc.x[2]);
      const bool keep = nA && (prev_m ? okc.x[2] != psz : (!have_last || okc.x[2] != last_sz));
      const uint64_t keep_m = __builtin_amdgcn_ballot_w64(keep);
      if (keep) {
        Ivl v = okc;
        v.info = p.info;
        curr.a[curr.n + (int)__builtin_popcountll(keep_m & below)] = v;
      }
      curr.n += (int)__builtin_popcountll(keep_m);
      if (nA_m) {
        const int hl = 63 - (int)__builtin_clzll(nA_m);
        last_sz = bperm64(hl, okc.x[2]);
        have_last = true;
      }
      publish();
    }
    if (curr.n == 0) break;
    const WList t2 = curr;
    curr = prev;
    prev = t2;
  }
  wreverse(mem, lane);
  return ret;
}

__global__ void __launch_bounds__(256) collect_intv_wave_kernel(DevBwt b, SeedArgs a) {
  const int lane = (int)(threadIdx.x & 63);
  const bool l0 = lane == 0;
  const int nw = (int)(gridDim.x * (blockDim.x >> 6));
  const int n_heavy = *a.n_heavy;
  NoBudget nb;
  for (int h = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6); h < n_heavy; h += nw) {
    const int r = __builtin_amdgcn_readfirstlane(a.heavy[h]);
    const int64_t q0 = a.seq_off[r];
    const int len = (int)(a.seq_off[r + 1] - q0);
    const uint8_t* q = a.seq + q0;
    Ivl* base = reinterpret_cast<Ivl*>(a.scratch) + 4 * (q0 + 2 * (int64_t)r);
    WList la{base, 0, len + 2}, lb{base + (len + 2), 0, len + 2}, mem1{base + 2 * (len + 2), 0, len + 2};
    WList mem{reinterpret_cast<Ivl*>(a.out) + (int64_t)r * a.max_per_read, 0, a.max_per_read};
    int x = 0;
    while (x < len) {  // SMEMs
      if (q[x] < 4) {
        x = smem1_wave(b, len, q, x, 1, mem1, la, lb, lane);
        for (int i = 0; i < mem1.n; ++i) {
          const Ivl v = mem1.a[i];
          if ((int)((uint32_t)v.info - (uint32_t)(v.info >> 32)) >= a.min_seed_len) mem.push(v, l0);
        }
        publish();
      } else {
        ++x;
      }
    }
    const int old_n = min(mem.n, mem.cap);
    for (int k = 0; k < old_n; ++k) {  // re-seeding inside long SMEMs
      const Ivl p = mem.a[k];
      const int start = (int)(p.info >> 32), end = (int)(int32_t)p.info;
      if (end - start < a.split_len || p.x[2] > (uint64_t)a.split_width) continue;
      smem1_wave(b, len, q, (start + end) >> 1, (int)(p.x[2] + 1), mem1, la, lb, lane);
      for (int i = 0; i < mem1.n; ++i) {
        const Ivl v = mem1.a[i];
        if ((uint32_t)v.info - (uint32_t)(v.info >> 32) >= (uint32_t)a.min_seed_len) mem.push(v, l0);
      }
      publish();
    }
    if (a.max_mem_intv > 0) {  // LAST-like
      x = 0;
      while (x < len) {
        if (q[x] < 4) {
          Ivl m;
          x = seed_strategy1(b, len, q, x, a.min_seed_len, a.max_mem_intv, m, nb);
          if (m.x[2] > 0) mem.push(m, l0);
        } else {
          ++x;
        }
      }
      publish();
    }
    if (l0) {
      if (mem.n <= mem.cap) {
        intro_sort(mem.a, mem.n);
        a.out_n[r] = mem.n;
      } else {
        a.out_n[r] = -mem.n;
      }
    }
    publish();
  }
}

// one wave per read: its intervals (32 B each) copied lane-parallel
__global__ void __launch_bounds__(256) pack_intv_kernel(SeedArgs a, const int64_t* __restrict__ off,
                                                        bwagpu_intv_t* __restrict__ dst) {
  const int r = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = (int)(threadIdx.x & 63);
  if (r >= a.n_reads) return;
  const int n = a.out_n[r];
  const ulonglong4* src = reinterpret_cast<const ulonglong4*>(a.out) + (int64_t)r * a.max_per_read;
  ulonglong4* d = reinterpret_cast<ulonglong4*>(dst) + off[r];
  for (int i = lane; i < n; i += 64) d[i] = src[i];
}

// bwt_sa (bwt.c:86-96): one lane per position; every LF step reads one
// 64-byte occurrence block (bwt_B0 and bwt_occ of a step fall in the same one)
// one step of bwt_sa's walk: bwt_invPsi (bwt.c:53-59), the row whose suffix
// starts one position earlier (its SA entry is this row's minus one)
__device__ __forceinline__ uint64_t sa_step(const DevBwt& b, uint64_t k) {
  if (k == b.primary) return 0;
  const uint64_t x = k - (k > b.primary);
  const int c = base_at(b, x);  // bwt_B0
  uint64_t cnt[4];
  occ4(b, k, cnt);  // bwt_occ(k, c); k == seq_len gives the column total
  return b.L2[c] + cnt[c];
}

__global__ void __launch_bounds__(256) bwt_sa_kernel(DevBwt b, int64_t n, const uint64_t* __restrict__ kin,
                                                     uint64_t* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint64_t k = kin[i], steps = 0;
  if (b.sa_full32) {  // the expanded suffix array: one load (row 0's stored -1 comes back 64-bit)
    const uint32_t v = b.sa_full32[k];
    out[i] = v == 0xffffffffu ? ~0ull : (uint64_t)v;
    return;
  }
  if (b.sa_full64) {
    out[i] = b.sa_full64[k];
    return;
  }
  while (k & b.sa_mask) {  // bwt_sa (bwt.c:86-96): walk to a sampled row
    ++steps;
    k = sa_step(b, k);
  }
  out[i] = steps + b.sa[k >> b.sa_shift];
}

// The whole suffix array from the sample: a thread per sampled row walks
// bwt_sa's steps from it — each step's row has the entry one smaller — and
// writes every row it passes until the next sampled row.  The step is a
// permutation of the rows, so every row is written exactly once; the rows an
// unsampled row's walk in bwt_sa_kernel would reach give the same value.  Row
// 0 (the sentinel's suffix) keeps its stored entry, -1 (bwt_cal_sa sets it,
// bwt.c:181), while the walk from it counts down from its true entry, seq_len.
__global__ void __launch_bounds__(256) sa_expand_kernel(DevBwt b, uint64_t n_sampled, uint32_t* __restrict__ o32,
                                                        uint64_t* __restrict__ o64) {
  const uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= n_sampled) return;
  uint64_t k = s << b.sa_shift, v = s == 0 ? b.seq_len : b.sa[s];
  for (;;) {
    const uint64_t w = k == 0 ? b.sa[0] : v;
    if (o32) o32[k] = (uint32_t)w;
    else o64[k] = w;
    k = sa_step(b, k);
    if (!(k & b.sa_mask)) break;
    --v;
  }
}

}  // namespace

hipError_t launch_build_occ64(const DevBwt& b, uint4* occ, uint64_t* sup, hipStream_t st) {
  const uint64_t nb = occ64_blocks(b.seq_len), ns = occ64_supers(b.seq_len, b.sup_shift);
  const uint64_t n = nb > ns ? nb : ns;
  hipLaunchKernelGGL(build_occ64_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, b, occ, sup, nb, ns);
  return hipGetLastError();
}

hipError_t launch_bwt_sa(const DevBwt& b, int64_t n, const uint64_t* k, uint64_t* out, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(bwt_sa_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, b, n, k, out);
  return hipGetLastError();
}

hipError_t launch_sa_expand(const DevBwt& b, uint32_t* o32, uint64_t* o64, hipStream_t st) {
  const uint64_t n = (b.seq_len >> b.sa_shift) + 1;  // sampled rows 0, sa_intv, ... <= seq_len
  hipLaunchKernelGGL(sa_expand_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, b, n, o32, o64);
  return hipGetLastError();
}

hipError_t launch_pack_intv(const SeedArgs& a, const int64_t* off, bwagpu_intv_t* dst, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  const int blocks = (a.n_reads + 3) / 4;
  hipLaunchKernelGGL(pack_intv_kernel, dim3(blocks), dim3(256), 0, st, a, off, dst);
  return hipGetLastError();
}

hipError_t launch_collect_intv(const DevBwt& b, const SeedArgs& a, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(a.n_heavy, 0, sizeof(int32_t), st);
  if (e == hipSuccess) e = hipMemsetAsync(a.flags, 0, sizeof(int32_t) * (size_t)a.n_reads, st);
  if (e != hipSuccess) return e;
  // BWAGPU_SEED_STEP=1: the one-extension-per-step form (A/B)
  static const bool step = getenv("BWAGPU_SEED_STEP") && atoi(getenv("BWAGPU_SEED_STEP"));
  if (step)
    hipLaunchKernelGGL(collect_intv_step_kernel, dim3((2 * a.n_reads + 255) / 256), dim3(256), 0, st, b, a);
  else
    hipLaunchKernelGGL(collect_intv_kernel, dim3((2 * a.n_reads + 255) / 256), dim3(256), 0, st, b, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  hipLaunchKernelGGL(tier1_merge_kernel, dim3((a.n_reads + 255) / 256), dim3(256), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the reads tier 1 gave up on, one wave each (the count is read on the device)
  const int waves = a.n_reads < 4096 ? a.n_reads : 4096;
  hipLaunchKernelGGL(collect_intv_wave_kernel, dim3((waves + 3) / 4), dim3(256), 0, st, b, a);
  return hipGetLastError();
}

}  // namespace bwagpu
