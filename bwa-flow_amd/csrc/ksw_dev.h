// ksw_dev.h — device building blocks shared by the extension kernels
// (sw_kernels.hip: per-read path and bare task lists; spec.hip: the
// speculative mem_chain2aln; stream.hip: the FPGA wire format).
//
// ksw_extend2 (bwa/ksw.c:380-479) in three lane mappings, all integer VALU
// work (no MFMA):
//  * extend_wave   one call per wave, the query columns in contiguous blocks of
//                  C = ceil((qlen+1)/64) per lane;
//  * extend_pair   two calls per wave, one per 32-lane half;
//  * extend_quad   four calls per wave: two per half, packed in the 16-bit
//                  halves of every DP register (v_pk_* ops).
// In each, everything the reference keeps in eh[] lives in registers; the
// horizontal-gap recurrence F is a max-plus prefix scan over the lanes; the
// row max + LAST argmax is one reduction of the key H << 10 | j; the band trim
// (ksw.c:466-469) is a min / max reduction of the non-zero columns.  Target
// rows are gathered from the HBM-resident 2-bit pac (bntseq.c:225 bit order;
// reverse strand = complement of the mirrored forward, bntseq.c:405-411) into
// LDS row buffers.  Then: one seed's extension (extend_seed, bwamem.c:717-792),
// the sharded work queues and wave-aggregated appends of the persistent grids.
#pragma once
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>

#include "engine.h"
#include "wave_ops.h"

namespace bwagpu {

// wave-uniform max of a group-uniform value over the wave's ACTIVE groups (for
// loop bounds every active group of the wave can share: a scalar branch
// instead of per-lane masking).  Groups of one wave may be at different points
// of the read loop, so inactive groups' registers hold unrelated values: read
// each group's lane 0 with v_readlane and keep it only if EXEC says it is live.
template <int G>
__device__ __forceinline__ int wave_umax(int v) {
  const unsigned long long ex = __builtin_amdgcn_read_exec();
  int m = 0;
#pragma unroll
  for (int k = 0; k < 64 / G; ++k)
    if ((ex >> (k * G)) & 1ull) m = max(m, __builtin_amdgcn_readlane(v, k * G));
  return m;
}

__device__ __forceinline__ long long grp_sum64(long long v, int G) {
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, G);
  return v;
}

__device__ __forceinline__ int pac_base2(const uint8_t* __restrict__ pac, int64_t l_pac, int64_t x) {
  // 2-strand coordinate -> base (bns_get_seq, bntseq.c:398-419)
  if (x < l_pac) return (pac[x >> 2] >> ((~x & 3) << 1)) & 3;
  int64_t f = (l_pac << 1) - 1 - x;
  return 3 - ((pac[f >> 2] >> ((~f & 3) << 1)) & 3);
}

// a wave-uniform value kept in a VGPR: arithmetic on it issues on the VALU
__device__ __forceinline__ int vgpr(int x) {
  int y;
  asm("v_mov_b32 %0, %1" : "=v"(y) : "v"(x));
  return y;
}
__device__ __forceinline__ int usat32(int a, int b) {  // max(a - b, 0) for a, b >= 0
  return (int)__builtin_elementwise_sub_sat((unsigned)a, (unsigned)b);
}

// (int)((double)x / e + 1.) exactly, for e >= 1 and |x| < 2^21 (make_opt
// bounds every input): the real value is (x+e)/e, so it is C's truncating
// quotient.  A float reciprocal gives it to within one; one remainder check
// fixes it — instead of the f64 division the reference's expression compiles to.
__device__ __forceinline__ int trunc_div1(int x, int e) {
  const int n = x + e;
  const int an = n < 0 ? -n : n;
  int q = (int)((float)an * __builtin_amdgcn_rcpf((float)e));
  const int r = an - q * e;
  q = r >= e ? q + 1 : (r < 0 ? q - 1 : q);
  return n < 0 ? -q : q;
}

// cal_max_gap, bwamem.c:630-637
__device__ __forceinline__ int max_gap_len(const DevOpt& o, int qlen) {
  int ld = trunc_div1(qlen * o.a - o.o_del, o.e_del);
  int li = trunc_div1(qlen * o.a - o.o_ins, o.e_ins);
  int l = ld > li ? ld : li;
  l = l > 1 ? l : 1;
  return l < (o.w << 1) ? l : (o.w << 1);
}

// band clamp of ksw_extend2 (ksw.c:399-407), device form of band_cap
__device__ __forceinline__ int band_cap_dev(int qlen, int max_mat, int end_bonus, int o, int e) {
  const int l = trunc_div1(qlen * max_mat + end_bonus - o, e);
  return l > 1 ? l : 1;
}

// query profile of base q (0..4): byte t = mat[t*5 + q]; selects over kernel
// arguments (SGPRs).  The empty asm makes the five words opaque so that the
// select chain is not turned back into an indexed load from the kernarg
// segment (a global load per extension whose wait also drained the table DMA).
__device__ __forceinline__ uint32_t qprof_word(const DevOpt& o, int q) {
  uint32_t p0 = o.qprof[0], p1 = o.qprof[1], p2 = o.qprof[2], p3 = o.qprof[3], p4 = o.qprof[4];
  asm volatile("" : "+s"(p0), "+s"(p1), "+s"(p2), "+s"(p3), "+s"(p4));
  uint32_t v = p0;
  v = q == 1 ? p1 : v;
  v = q == 2 ? p2 : v;
  v = q == 3 ? p3 : v;
  v = q == 4 ? p4 : v;
  return v;
}
__device__ __forceinline__ int qprof4_val(const DevOpt& o, int q) {
  int p0 = o.qprof4[0], p1 = o.qprof4[1], p2 = o.qprof4[2], p3 = o.qprof4[3], p4 = o.qprof4[4];
  asm volatile("" : "+s"(p0), "+s"(p1), "+s"(p2), "+s"(p3), "+s"(p4));
  int v = p0;
  v = q == 1 ? p1 : v;
  v = q == 2 ? p2 : v;
  v = q == 3 ? p3 : v;
  v = q == 4 ? p4 : v;
  return v;
}


struct ExtOut {
  int score, qle, tle, gtle, gscore, max_off;
};

struct Tally {
  long long cells, rows, calls;
};

constexpr int NEG = -(1 << 29);

// ------------------------------------------------ ksw_extend2, one read per wave
// The G = 64 form used by every production kernel.  Columns are STRIDED over
// the wave: lane r holds columns j = 64c + r of segments c < CD (CD =
// ceil((qlen+1)/64), a compile-time constant picked by extend_wave_dispatch).
// Consequences:
//  * each segment is one wave-wide row slice: the in-band test, the non-zero
//    test and the row-max key are 64-bit lane masks / one wave reduction, and
//    every band/maximum/break quantity is a scalar (SGPR) value;
//  * the F scan runs segment after segment, each segment's exclusive prefix
//    seeded with the running maximum (a scalar carry) of the ones before it;
//    columns past qlen sit after every real column and need no masking;
//  * the reference's special eh[] writes (eh[lo].h = first-column value,
//    eh[hi] = {h1, 0}, ksw.c:420-429,449) are single-lane selects.
// x <- inclusive max-scan over the wave (row_shr 1/2/4/8, row_bcast 15/31)
// and r <- wave max in lane 63 (row_ror 8/4/2/1, row_bcast 15/31), the two
// dependency chains interleaved: every DPP read is 2 wait states after the
// write of its source (the other chain's op + s_nop 0).
__device__ __forceinline__ void scan_reduce(int& x, int& r) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_bcast:31 row_mask:0xc bank_mask:0xf"
      : "+v"(x), "+v"(r));
}

// the row bound's period (extend_wave, extend_quad): every fourth row
#ifndef RB_MASK
#define RB_MASK 3
#endif

template <int CD, bool T5>
__device__ __forceinline__ ExtOut extend_wave(const DevOpt& o, int qlen, const uint8_t* __restrict__ qp, int qa,
                                              int qd, int tlen, const uint8_t* tb, int w, int end_bonus, int zdrop,
                                              int h0, Tally& tl) {
  const int r = (int)(threadIdx.x & 63);
  const int e_del = o.e_del, e_ins = o.e_ins, oe_del = o.oe_del, oe_ins = o.oe_ins;
  int hh[CD], ee[CD];
  uint32_t pf[CD];
  uint32_t pf4[T5 ? CD : 1];
  int Kc[CD], jEc[CD], Fc[CD], jc[CD];
#pragma unroll
  for (int c = 0; c < CD; ++c) {
    const int j = 64 * c + r;
    jc[c] = j;
    const int qb = j < qlen ? qp[qa + qd * j] : 0;
    pf[c] = qprof_word(o, qb);
    if (T5) pf4[c] = (uint32_t)(uint8_t)qprof4_val(o, qb);
    // row -1 of eh[] (ksw.c:392-395): H(-1,-1)=h0, then an insertion gap
    const int v = j == 0 ? h0 : max(h0 - oe_ins - (j - 1) * e_ins, 0);
    hh[c] = j <= qlen ? v : 0;
    ee[c] = 0;
    // F scan constants: u_j = t_j + j*e_ins, F_j = max_{k<j} u_k - (j-1)*e_ins
    jEc[c] = j * e_ins;
    Kc[c] = j * e_ins - oe_ins;    // u_j = max(M_j + Kc, jEc) in band, jEc outside
    Fc[c] = e_ins - j * e_ins;     // F_j = EX_j + Fc
  }
  {  // band clamp (ksw.c:399-407)
    const int mi = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_ins, e_ins);
    const int md = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_del, e_del);
    w = __builtin_amdgcn_readfirstlane(min(w, min(mi, md)));
  }
  // Row bookkeeping (band, left column, z-drop, maxima) is wave-uniform but
  // lives in VGPRs: a VALU op issues at ~2.5 SIMD cycles, an SALU op at ~4.3
  // (profiles/r01e_issue_costs.json), and VALU work of one wave overlaps the
  // SALU of another.  Only the two exits branch on scalars.
  int best = vgpr(h0), bi = vgpr(-1), bj = vgpr(-1), ei = vgpr(-1), esc = vgpr(-1), off = vgpr(0);
  int lo = vgpr(0), hi = vgpr(qlen);
  int iw = vgpr(-w), iw1 = vgpr(w + 1);  // i - w, i + w + 1
  int gl = vgpr(h0 - o.o_del - e_del);   // h0 - (o_del + e_del*(i+1))
  int vi = vgpr(0);                      // i
  int cells = vgpr(0);
  int rows = tlen;
  int tnext = tlen > 0 ? tb[0] : 0;
  // The row maximum of row i-1 is reduced while row i's F scan runs: the two
  // 6-step DPP chains interleave in one asm block (scan_reduce), and row i-1's
  // exit test moves to row i, whose results are dropped if row i-1 exits.
  int rkp = 0;  // row i-1's per-lane key (H << 10 | j)
  // row k's bookkeeping (ksw.c:454-465) from its reduced key; true = exit
  auto row_end = [&](int rkr, int vk) -> bool {
    const int mrow = rkr >> 10, mj = rkr & 1023;
    const bool up = mrow > best;
    const int di = vk - bi, dj = mj - bj;
    const int drop = best - mrow - max(__mul24(di - dj, e_del), __mul24(dj - di, e_ins));
    const bool brk = mrow == 0 || (!up && zdrop > 0 && drop > zdrop);
    off = up ? max(off, abs(mj - vk)) : off;
    best = up ? mrow : best;
    bi = up ? vk : bi;
    bj = up ? mj : bj;
    return __builtin_amdgcn_ballot_w64(brk) != 0;
  };
  for (int i = 0; i < tlen; ++i) {
    const int t = __builtin_amdgcn_readfirstlane(tnext);
    tnext = tb[i + 1];  // prefetch (the buffer is 2 rows longer than any call reads)
    lo = max(lo, iw);
    hi = min(min(hi, iw1), qlen);
    iw += 1;
    iw1 += 1;
    const int wd = usat32(hi, lo);  // hi > lo ? hi - lo : 0; in band: (unsigned)(j - lo) < wd
    const int left0 = lo == 0 ? max(gl, 0) : 0;
    gl -= e_del;
    const int sh = (t & 3) << 3;

    // pass 1 + segmented exclusive max-scan of u
    int M[CD], EX[CD];
    bool inb[CD];
    int carry = NEG;
#pragma unroll
    for (int c = 0; c < CD; ++c) {
      inb[c] = (unsigned)(jc[c] - lo) < (unsigned)wd;
      int sc;
      if (T5 && t == 4) sc = (int)(int8_t)(pf4[c] & 0xff);
      else sc = __builtin_amdgcn_sbfe((int)pf[c], sh, 8);
      const int m = hh[c] ? hh[c] + sc : 0;
      M[c] = m;
      const int u = inb[c] ? max(m + Kc[c], jEc[c]) : jEc[c];
      int x = c == 0 ? u : max(u, carry);
      if (c == 0) scan_reduce(x, rkp);
      else x = max_bc31(max_bc15(max_shr8(max_shr4(max_shr2(max_shr1(x))))));
      EX[c] = dpp<DPP_WAVE_SHR1>(carry, x);  // lane 0 takes the carry from the segments before
      if (c + 1 < CD) carry = __builtin_amdgcn_readlane(x, 63);
    }
    // pass 2: H, E, row-max key, next-row state; hsel = the register holding
    // column hi (H(i, hi-1) after the shift)
    int rk = 0, prev63 = 0, hsel = 0;
#pragma unroll
    for (int c = 0; c < CD; ++c) {
      const int f = EX[c] + Fc[c];
      const int h = max(max(M[c], ee[c]), f);
      const int en = max(max(ee[c] - e_del, M[c] - oe_del), 0);
      rk = max(rk, inb[c] ? (h << 10 | jc[c]) : 0);
      const int hs = dpp<DPP_WAVE_SHR1>(prev63, h);  // H(i, j-1)
      if (c + 1 < CD) prev63 = __builtin_amdgcn_readlane(h, 63);
      hsel = (c == 0 || (hi >> 6) == c) ? hs : hsel;
      hh[c] = inb[c] ? hs : hh[c];
      ee[c] = inb[c] ? en : ee[c];
    }
    const int hi_s = __builtin_amdgcn_readfirstlane(hi);
    // h1 = H(i, hi-1), or the first-column value when the band is empty
    const int h1r = __builtin_amdgcn_readlane(hsel, hi_s & 63);
    const int h1 = hi > lo ? h1r : left0;
    // eh[lo].h = first-column value (only when lo < hi), eh[hi] = {h1, 0}:
    // single-lane writes at uniform targets
    const int tlo = hi > lo ? lo : -1;
#pragma unroll
    for (int c = 0; c < CD; ++c) {
      hh[c] = jc[c] == tlo ? left0 : hh[c];
      const bool at_hi = jc[c] == hi;
      hh[c] = at_hi ? h1 : hh[c];
      ee[c] = at_hi ? 0 : ee[c];
    }
    // zero-trim of the band for the next row (ksw.c:466-469), computed ahead of
    // the row-max reduction (independent of it; applied only if no break):
    // first non-zero column in [lo,hi), last non-zero column in [lo,hi]
    int nlo, nhi;
    if constexpr (CD == 1) {
      // qlen < 64, so hi < 64: one mask per row, no segment loop
      const uint64_t nz = __builtin_amdgcn_ballot_w64((hh[0] | ee[0]) != 0);
      const uint64_t f = nz & __builtin_amdgcn_ballot_w64(inb[0]);
      const uint64_t l = f | (nz & (1ull << hi_s));
      nlo = f ? __builtin_ctzll(f) : hi_s;
      const int jl = l ? 63 - __builtin_clzll(l) : nlo - 1;
      nhi = min(jl + 2, qlen);
    } else {
      int jl = -1;
      nlo = hi_s;
#pragma unroll
      for (int c = CD - 1; c >= 0; --c) {
        const uint64_t nz = __builtin_amdgcn_ballot_w64((hh[c] | ee[c]) != 0);
        const uint64_t f = nz & __builtin_amdgcn_ballot_w64(inb[c]);
        const int hc = hi_s - 64 * c;
        const uint64_t l = f | (nz & ((unsigned)hc < 64u ? 1ull << hc : 0ull));
        nlo = f ? 64 * c + __builtin_ctzll(f) : nlo;  // descending c: the lowest segment wins
        jl = (jl < 0 && l) ? 64 * c + 63 - __builtin_clzll(l) : jl;
      }
      if (jl < 0) jl = nlo - 1;
      nhi = min(jl + 2, qlen);
    }
    if (i > 0 && row_end(__builtin_amdgcn_readlane(rkp, 63), vi - 1)) {
      rows = i;  // row i-1 was the last row: row i never ran
      break;
    }
    rkp = rk;
    cells += wd;
    {  // ksw.c:450-453
      const bool atend = max(lo, hi) == qlen;
      ei = (atend && !(esc > h1)) ? vi : ei;
      esc = atend ? max(esc, h1) : esc;
    }
    vi += 1;
    lo = nlo;
    hi = nhi;
    // the row bound of extend_quad, every fourth row: once no later cell can
    // reach gscore (<= max), row i's own bookkeeping is the last
    if (o.row_bound && (i & RB_MASK) == RB_MASK) {
      int bb = (lo == 0 && gl > 0) ? gl + qlen * o.max_mat : 0;
#pragma unroll
      for (int c = 0; c < CD; ++c) bb = max(bb, hh[c] > 0 ? hh[c] + __mul24(qlen - jc[c], o.max_mat) : 0);
      bb = max_bc31(max_bc15(max_ror1(max_ror2(max_ror4(max_ror8(bb))))));
      if (__builtin_amdgcn_readlane(bb, 63) < __builtin_amdgcn_readfirstlane(esc)) {
        const int rkr = max_bc31(max_bc15(max_ror1(max_ror2(max_ror4(max_ror8(rkp))))));
        (void)row_end(__builtin_amdgcn_readlane(rkr, 63), vi - 1);
        rows = i + 1;
        break;
      }
    }
  }
  if (rows == tlen && tlen > 0) {  // the last row's bookkeeping (its exit test is moot)
    int rkr = max_bc31(max_bc15(max_ror1(max_ror2(max_ror4(max_ror8(rkp))))));
    (void)row_end(__builtin_amdgcn_readlane(rkr, 63), vi - 1);
  }
  tl.cells += __builtin_amdgcn_readfirstlane(cells);
  tl.rows += rows;
  tl.calls += 1;
  auto u = [](int x) { return __builtin_amdgcn_readfirstlane(x); };
  return ExtOut{u(best), u(bj) + 1, u(bi) + 1, u(ei) + 1, u(esc), u(off)};
}

// CD is uniform per call (qlen is): one compiled body per segment count
// (blocked columns were measured slower: DESIGN.md §3)
template <int C, bool T5>
__device__ __forceinline__ ExtOut extend_wave_dispatch(const DevOpt& o, int qlen, const uint8_t* __restrict__ qp,
                                                    int qa, int qd, int tlen, const uint8_t* tb, int w,
                                                    int end_bonus, int zdrop, int h0, Tally& tl) {
  qlen = __builtin_amdgcn_readfirstlane(qlen);
  qa = __builtin_amdgcn_readfirstlane(qa);
  qd = __builtin_amdgcn_readfirstlane(qd);
  tlen = __builtin_amdgcn_readfirstlane(tlen);
  w = __builtin_amdgcn_readfirstlane(w);
  end_bonus = __builtin_amdgcn_readfirstlane(end_bonus);
  zdrop = __builtin_amdgcn_readfirstlane(zdrop);
  h0 = __builtin_amdgcn_readfirstlane(h0);
  const int cd = (qlen + 64) >> 6;  // ceil((qlen+1)/64)
#define EXT_SEG(n)                                                                                          \
  if (n <= C && cd == n) return extend_wave<(n <= C ? n : 1), T5>(o, qlen, qp, qa, qd, tlen, tb, w, end_bonus, zdrop, h0, tl);
  EXT_SEG(1) EXT_SEG(2) EXT_SEG(3) EXT_SEG(4) EXT_SEG(5) EXT_SEG(6) EXT_SEG(7) EXT_SEG(8)
  EXT_SEG(9) EXT_SEG(10) EXT_SEG(11) EXT_SEG(12) EXT_SEG(13) EXT_SEG(14) EXT_SEG(15) EXT_SEG(16)
#undef EXT_SEG
  return ExtOut{-1, 0, 0, 0, -1, 0};  // unreachable: cd <= C by construction
}

// ------------------------------------------------ ksw_extend2, two per wave
// TWO extensions per wave: lanes 0-31 run one ksw_extend2, lanes 32-63 another
// (the halves' rows run in lock step; a half whose call has ended is off in
// EXEC until the other's ends too).  Every per-row instruction of
// extend_wave_blk — the F scan, the row-max reduction, the band bookkeeping —
// then serves two extensions, and a 32-lane half covers a short extension
// (qlen < 32: most left/right extensions of a 150 bp read are below 64) with
// one column slot per lane.
//  * columns are BLOCKED over the half: lane r holds j = r*CPL + c, c < CPL;
//  * every per-call quantity (qlen, band, maxima, break state) is a per-lane
//    VGPR value that is uniform over the half: no readfirstlane, no ballot;
//  * the F scan is ONE inclusive max-scan over the half (row_shr 1/2/4/8 +
//    row_bcast:15 into rows 1/3, which never crosses the half boundary), the
//    row max a row_ror reduction finished by an exchange of
//    the half's two rows (v_permlane16_swap); the band trim (ksw.c:466-469)
//    a min and a max reduction of the same shape;
//  * the gscore/max_ie tracking (ksw.c:450-453) runs on the lane that owns
//    column qlen-1 (h1 = H(i, qlen-1) whenever the row ends at qlen) and is
//    read from it once per call.
// Half-wave all-reduce from per-row results: v_permlane16_swap (gfx950)
// exchanges rows 0<->1 and 2<->3 of two registers — a VALU op, so there is no
// LDS round trip (ds_swizzle) on the row's dependency chain.
__device__ __forceinline__ int half_max(int v) {  // v: its row's max in every lane -> the half's
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return max((int)r[0], (int)r[1]);
}
__device__ __forceinline__ int half_min(int v) {
  const auto r = __builtin_amdgcn_permlane16_swap((unsigned)v, (unsigned)v, false, false);
  return min((int)r[0], (int)r[1]);
}

// x <- inclusive max-scan over each 32-lane half; r <- its 16-lane row's max in
// every lane (finish with half_max(r)).  Interleaved like scan_reduce.
__device__ __forceinline__ void scan_reduce32(int& x, int& r) {
  asm volatile(
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_max_i32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 1\n\t"
      "v_max_i32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf"
      : "+v"(x), "+v"(r));
}

// lo <- 16-lane row min, hi <- row max, in every lane (two chains interleaved)
__device__ __forceinline__ void row_minmax(int& lo, int& hi) {
  asm volatile(
      "s_nop 1\n\t"
      "v_min_i32_dpp %0, %0, %0 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:8 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_min_i32_dpp %0, %0, %0 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:4 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_min_i32_dpp %0, %0, %0 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:2 row_mask:0xf bank_mask:0xf\n\t"
      "s_nop 0\n\t"
      "v_min_i32_dpp %0, %0, %0 row_ror:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_max_i32_dpp %1, %1, %1 row_ror:1 row_mask:0xf bank_mask:0xf"
      : "+v"(lo), "+v"(hi));
}

__device__ __forceinline__ int row_max32(int x) {
  return max_ror1(max_ror2(max_ror4(max_ror8(x))));
}

struct Tally32 {  // per-seed DP work (fits 32 bits: <= 1023 columns x a window's rows)
  int cells, rows, calls;
};

template <int CPL>
__device__ __forceinline__ ExtOut extend_pair(const DevOpt& o, int qlen, const uint8_t* __restrict__ qp, int qa,
                                              int qd, int tlen, const uint8_t* tb, int w, int end_bonus, int zdrop,
                                              int h0, Tally32& tl) {
  // the lane index is re-derived here behind an opaque move: otherwise the
  // compiler hoists every variant's lane constants (j0 + c, ...) to the kernel
  // entry, where they stay live across all of it (measured: 167 VGPRs)
  int r;
  asm volatile("v_and_b32 %0, 31, %1" : "=v"(r) : "v"((int)threadIdx.x));
  const int e_del = o.e_del, e_ins = o.e_ins, o_del = o.o_del, oe_ins = o.oe_ins;
  constexpr int KS = CPL <= 2 ? 1 : (CPL <= 4 ? 2 : (CPL <= 8 ? 3 : 4));  // in-lane column bits of the key
  static_assert(CPL >= 1 && CPL <= 16, "two extensions per wave: CPL <= 16");
  const int j0 = r * CPL;
  int hh[CPL], ee[CPL];
  uint32_t pf[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j = j0 + c;
    const int qv = qp[qa + qd * min(j, qlen - 1)];  // unconditional load (qlen >= 1)
    const int qb = j < qlen ? qv : 0;
    pf[c] = qprof_word(o, qb);
    const int v = j == 0 ? h0 : max(h0 - oe_ins - (j - 1) * e_ins, 0);  // ksw.c:392-395
    hh[c] = j <= qlen ? v : 0;
    ee[c] = 0;
  }
  {  // band clamp (ksw.c:399-407)
    const int mi = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_ins, e_ins);
    const int md = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_del, e_del);
    w = min(w, min(mi, md));
  }
  const int rE = e_ins * CPL * r;  // the lane's offset in the scan
  const int cq = qlen - 1 - j0;    // slot of column qlen-1 on its owner lane
  int best = h0, bi = -1, bj = -1, ei = -1, esc = -1, off = 0;
  int lo = 0, hi = qlen;
  int iw = -w, iw1 = w + 1;
  int gl = h0 - o.o_del - e_del;
  int vi = 0, cells = 0;
  int rows = tlen;
  int tnext = tlen > 0 ? tb[0] : 0;
  int rkp = 0;  // row i-1's per-lane key, reduced during row i's scan
  auto row_end = [&](int rkr, int vk) -> bool {  // ksw.c:454-465 of row vk
    const int mrow = rkr >> 10, mj = rkr & 1023;
    const bool up = mrow > best;
    const int di = vk - bi, dj = mj - bj;
    const int drop = best - mrow - max(__mul24(di - dj, e_del), __mul24(dj - di, e_ins));
    const bool brk = mrow == 0 || (!up && zdrop > 0 && drop > zdrop);
    off = up ? max(off, abs(mj - vk)) : off;
    best = up ? mrow : best;
    bi = up ? vk : bi;
    bj = up ? mj : bj;
    return brk;
  };
  // The halves run their rows in lock step; a half whose call ends leaves the
  // loop (EXEC) while the other finishes.  (A branch-free form — the ended half
  // kept in the loop with an empty band and select-guarded bookkeeping — was
  // measured 7 % slower: 0.97 vs 0.90 ms per spec_ext2_kernel<5> launch.)
  for (int i = 0; i < tlen; ++i) {
    const int t = tnext;
    tnext = tb[i + 1];  // prefetch (the buffer is 2 rows longer than any call reads)
    lo = max(lo, iw);
    hi = min(min(hi, iw1), qlen);
    iw += 1;
    iw1 += 1;
    const int wd = usat32(hi, lo);
    const int left0 = lo == 0 ? max(gl, 0) : 0;
    gl -= e_del;
    const int sh = (t & 3) << 3;
    const int x = j0 - lo;
    int M[CPL], A[CPL];
    int T = 0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const bool ib = (unsigned)(x + c) < (unsigned)wd;
      const int sc = __builtin_amdgcn_sbfe((int)pf[c], sh, 8);
      const int m = hh[c] ? hh[c] + sc : 0;
      M[c] = m;
      A[c] = (ib ? m : NEG) - oe_ins;
      T = max(T - e_ins, A[c]);
    }
    int sx = T + rE;
    scan_reduce32(sx, rkp);  // inclusive half scan of this row + row i-1's row maxima
    int EX = dpp<DPP_WAVE_SHR1>(NEG, sx);
    EX = r == 0 ? NEG : EX;  // lane 32 took lane 31's value
    int f = max(EX - rE + e_ins * CPL, 0);
    int hm[CPL];
    int lk = 0;
    const int hix = hi - j0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const unsigned d = (unsigned)(x + c);
      const bool ib = d < (unsigned)wd, ib2 = d <= (unsigned)wd;
      if (c > 0) f = max(max(f - e_ins, A[c - 1]), 0);
      const int h = max(max(M[c], ee[c]), f);
      hm[c] = ib ? h : 0;
      const int en = usat32(max(ee[c], M[c] - o_del), e_del);
      lk = max(lk, (hm[c] << KS) + c);
      ee[c] = ib ? en : (ib2 ? 0 : ee[c]);
      if (c > 0) hh[c] = ib2 ? hm[c - 1] : hh[c];
    }
    int hs0 = dpp<DPP_WAVE_SHR1>(0, hm[CPL - 1]);  // H(i, j0-1)
    hs0 = r == 0 ? left0 : hs0;                    // column 0: the first-column value
    hh[0] = (unsigned)x <= (unsigned)wd ? hs0 : hh[0];
    // h1 when the row ends at qlen: H(i, qlen-1) (0 when out of band), on its owner
    int h1q = 0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) h1q = cq == c ? hm[c] : h1q;
    // band trim for the next row (ksw.c:466-469): first non-zero column in
    // [lo, hi), last in [lo, hi]
    uint32_t nzm = 0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) nzm |= (uint32_t)((hh[c] | ee[c]) != 0) << c;
    const int lo_l = min(max(lo - j0, 0), 31), hi_l = min(max(hix, 0), 31);
    const uint32_t mf = nzm & ((1u << hi_l) - 1u) & ~((1u << lo_l) - 1u);   // [lo, hi)
    const uint32_t ml = mf | (nzm & ((unsigned)hix < (unsigned)CPL ? 1u << hix : 0u));  // + column hi
    int cl = mf ? j0 + (int)__builtin_ctz(mf) : 0x7fff;
    int ch = ml ? j0 + 31 - (int)__builtin_clz(ml) : -1;
    row_minmax(cl, ch);
    if (i > 0) {
      const int rkr = half_max(rkp);
      if (row_end(rkr, vi - 1)) {
        rows = i;  // row i-1 was the last row: row i never ran
        break;
      }
    }
    cl = half_min(cl);
    ch = half_max(ch);
    const int nlo = min(cl, hi);
    const int nhi = min(max(ch, nlo - 1) + 2, qlen);
    rkp = ((lk >> KS) << 10) | (j0 + (lk & ((1 << KS) - 1)));
    cells += wd;
    {  // ksw.c:450-453 (meaningful on the owner of column qlen-1)
      const bool atend = max(lo, hi) == qlen;
      ei = (atend && !(esc > h1q)) ? vi : ei;
      esc = atend ? max(esc, h1q) : esc;
    }
    vi += 1;
    lo = nlo;
    hi = nhi;
    // the row bound of extend_quad, every fourth row, per half (gscore lives on
    // the owner of column qlen-1 and is <= 0 on the half's other lanes)
    if (o.row_bound && (i & RB_MASK) == RB_MASK) {
      int bb = (lo == 0 && gl > 0) ? gl + qlen * o.max_mat : 0;
#pragma unroll
      for (int c = 0; c < CPL; ++c) bb = max(bb, hh[c] > 0 ? hh[c] + __mul24(qlen - j0 - c, o.max_mat) : 0);
      bb = half_max(row_max32(bb));
      if (bb < half_max(row_max32(esc))) {
        (void)row_end(half_max(row_max32(rkp)), vi - 1);
        rows = i + 1;
        break;
      }
    }
  }
  if (rows == tlen && tlen > 0) {  // the last row's bookkeeping (its exit test is moot)
    const int rkr = half_max(row_max32(rkp));
    (void)row_end(rkr, vi - 1);
  }
  // gscore / max_ie from the owner of column qlen-1 (qlen >= 1 for every call)
  const int own = (int)(threadIdx.x & 32) + (qlen - 1) / CPL;
  ei = __shfl(ei, own, 64);
  esc = __shfl(esc, own, 64);
  tl.cells += cells;
  tl.rows += rows;
  tl.calls += 1;
  return ExtOut{best, bj + 1, bi + 1, ei + 1, esc, off};
}

// The column count of the halves' current calls: CPL = ceil((qlen+1)/32) of
// the larger active half (both halves run one compiled body).
template <int PMAX>
__device__ __forceinline__ ExtOut extend_pair_dispatch(const DevOpt& o, int qlen, const uint8_t* __restrict__ qp,
                                                       int qa, int qd, int tlen, const uint8_t* tb, int w,
                                                       int end_bonus, int zdrop, int h0, Tally32& tl) {
  const unsigned long long ex = __builtin_amdgcn_read_exec();
  int qm = 0;
  if (ex & 1ull) qm = __builtin_amdgcn_readlane(qlen, 0);
  if ((ex >> 32) & 1ull) qm = max(qm, __builtin_amdgcn_readlane(qlen, 32));
  const int cpl = (qm + 32) >> 5;
#define EXT_PAIR(n) \
  if (n <= PMAX && cpl == n) return extend_pair<(n <= PMAX ? n : 1)>(o, qlen, qp, qa, qd, tlen, tb, w, end_bonus, zdrop, h0, tl);
  EXT_PAIR(1) EXT_PAIR(2) EXT_PAIR(3) EXT_PAIR(4) EXT_PAIR(5) EXT_PAIR(6) EXT_PAIR(7) EXT_PAIR(8)
#undef EXT_PAIR
  return ExtOut{-1, 0, 0, 0, -1, 0};  // unreachable: cpl <= PMAX by construction
}

// ------------------------------------------------ ksw_extend2, four per wave (packed 16-bit)
// FOUR extensions per wave: each 32-lane half runs two ksw_extend2 calls in
// lock step, call A in the low and call B in the high 16 bits of every DP
// register (v_pk_* ops: one instruction per column slot serves both).  Lane r
// of a half holds columns j = r*CPL + c of both calls, as in extend_pair.
// Every per-call quantity (band, maxima, break state) is uniform over its
// half; the band bounds, the E/H rows and the row maxima are packed, the
// row-end bookkeeping (ksw.c:454-465) runs per call in 32 bits.
// 16-bit ranges (quad_scores_ok on the host): H <= lq * max(mat) < 4096, so
// the row-max key H << KS | c and H * 2^sK + 128 (below) fit; no NEG sentinel
// is needed because every F contribution is clamped at 0 (a contribution <= 0
// never changes F = max(0, ...), ksw.c:446):
//  * M' = min(hh + S, hh * 2^sK), 2^sK > max(mat): hh + S where hh > 0, and
//    <= 0 where hh == 0 (ksw.c:430 sets M = 0 there; h = max(M, e, f) and the
//    E / F terms then see a value <= 0 either way).  S comes from v_perm_b32
//    on the two calls' profile words (bytes biased by 128) with a per-row
//    selector of the two target bases;
//  * F: A_c = min_u16(M - oe_ins, CAP_c) with CAP = 0xFFFF in band [lo, hi)
//    and 0 outside (cells right of the band only feed F of cells right of it);
//    the lane total T = max(sat(T - e_ins), A_c) >= 0, one inclusive max-scan
//    of T + (j0 + CPL) e_ins over the half (identity 0, two ops per DPP step),
//    F at the lane's first column = sat(EX - j0 e_ins);
//  * H stored for column j is H(i, j-1) within [lo, hi] (R = j <= hi), E in
//    band and 0 at column hi (ksw.c:449); columns left of lo become 0 (they are
//    never read again: lo only grows), columns right of hi keep their values;
//  * band trim (ksw.c:466-469): first non-zero column >= lo (a min over the
//    half) and last non-zero column <= hi (a max): a column left of lo is 0
//    here and one at or right of hi cannot move nlo = min(cl, hi);
//  * gscore / max_ie (ksw.c:450-453) on the lane owning column qlen-1.
// A call that ends (m == 0, z-drop, or its last target row) freezes with an
// empty band (lo = 0x7fff, hi = 0) while the others run on.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
namespace pk16 {
__device__ __forceinline__ s16x2 S(uint32_t x) { return __builtin_bit_cast(s16x2, x); }
__device__ __forceinline__ u16x2 U(uint32_t x) { return __builtin_bit_cast(u16x2, x); }
__device__ __forceinline__ uint32_t W(s16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t W(u16x2 x) { return __builtin_bit_cast(uint32_t, x); }
__device__ __forceinline__ uint32_t pk(int lo, int hi) { return __builtin_amdgcn_perm((uint32_t)hi, (uint32_t)lo, 0x05040100u); }
__device__ __forceinline__ int lo16(uint32_t x) { return (int)(int16_t)(x & 0xffffu); }
__device__ __forceinline__ int hi16(uint32_t x) { return (int)(int16_t)(x >> 16); }
__device__ __forceinline__ uint32_t add(uint32_t a, uint32_t b) { return W(U(a) + U(b)); }
__device__ __forceinline__ uint32_t sub(uint32_t a, uint32_t b) { return W(U(a) - U(b)); }
__device__ __forceinline__ uint32_t mad(uint32_t a, uint32_t b, uint32_t c) { return W(U(a) * U(b) + U(c)); }
__device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) { return W(U(a) * U(b)); }
__device__ __forceinline__ uint32_t smax(uint32_t a, uint32_t b) { return W(__builtin_elementwise_max(S(a), S(b))); }
__device__ __forceinline__ uint32_t smin(uint32_t a, uint32_t b) { return W(__builtin_elementwise_min(S(a), S(b))); }
__device__ __forceinline__ uint32_t umax(uint32_t a, uint32_t b) { return W(__builtin_elementwise_max(U(a), U(b))); }
__device__ __forceinline__ uint32_t umin(uint32_t a, uint32_t b) { return W(__builtin_elementwise_min(U(a), U(b))); }
__device__ __forceinline__ uint32_t usat(uint32_t a, uint32_t b) { return W(__builtin_elementwise_sub_sat(U(a), U(b))); }
__device__ __forceinline__ uint32_t ssat(uint32_t a, uint32_t b) { return W(__builtin_elementwise_sub_sat(S(a), S(b))); }
// the empty asm keeps a mask opaque: otherwise LLVM turns mask & a | ~mask & b
// back into per-half compares + v_cndmask + v_perm (5 ops for 1)
__device__ __forceinline__ uint32_t opq(uint32_t x) {
  asm("" : "+v"(x));
  return x;
}
__device__ __forceinline__ uint32_t neg15(uint32_t a) { return opq(W(S(a) >> (s16x2){15, 15})); }  // 0xffff where < 0
__device__ __forceinline__ uint32_t sel(uint32_t m, uint32_t a, uint32_t b) { return (m & a) | (~m & b); }

constexpr uint32_t ONE = 0x00010001u;
// DPP moves of whole registers (bound_ctrl: a lane without a source reads 0)
template <int CTRL>
__device__ __forceinline__ uint32_t mov0(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// inclusive max-scan over each G-lane group (G = 16: a DPP row, 32: a half)
// of packed values >= 0 (identity 0)
template <int G>
__device__ __forceinline__ uint32_t grp_scan_umax(uint32_t x) {
  x = umax(x, mov0<DPP_ROW_SHR(1)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(2)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(4)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(8)>(x));
  if constexpr (G == 16) return x;
  // rows 1 / 3 take the last lane of rows 0 / 2; rows 0 / 2 an identity 0
  const uint32_t t = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142 /* row_bcast:15 */, 0xA, 0xF, false);
  return umax(x, t);
}
// the whole half's min / max of packed values, in every lane of the half
__device__ __forceinline__ uint32_t half_umin(uint32_t x) {
  x = umin(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(8), 0xF, 0xF, false));
  x = umin(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(4), 0xF, 0xF, false));
  x = umin(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(2), 0xF, 0xF, false));
  x = umin(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(1), 0xF, 0xF, false));
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return umin((uint32_t)p[0], (uint32_t)p[1]);
}
// the group's umax of K, umin of L and smax of H at once: three independent
// chains step by step, so no DPP read waits on the write just before it
template <int G>
__device__ __forceinline__ void grp_red3(uint32_t& K, uint32_t& L, uint32_t& H) {
#define RED3_STEP(CTRL)                                                                  \
  {                                                                                      \
    const uint32_t k = (uint32_t)__builtin_amdgcn_mov_dpp((int)K, CTRL, 0xF, 0xF, false); \
    const uint32_t l = (uint32_t)__builtin_amdgcn_mov_dpp((int)L, CTRL, 0xF, 0xF, false); \
    const uint32_t h = (uint32_t)__builtin_amdgcn_mov_dpp((int)H, CTRL, 0xF, 0xF, false); \
    K = umax(K, k);                                                                      \
    L = umin(L, l);                                                                      \
    H = smax(H, h);                                                                      \
  }
  RED3_STEP(DPP_ROW_ROR(8))
  RED3_STEP(DPP_ROW_ROR(4))
  RED3_STEP(DPP_ROW_ROR(2))
  RED3_STEP(DPP_ROW_ROR(1))
#undef RED3_STEP
  if constexpr (G == 16) return;  // a DPP row: done
  const auto pk_ = __builtin_amdgcn_permlane16_swap(K, K, false, false);
  const auto pl = __builtin_amdgcn_permlane16_swap(L, L, false, false);
  const auto ph = __builtin_amdgcn_permlane16_swap(H, H, false, false);
  K = umax((uint32_t)pk_[0], (uint32_t)pk_[1]);
  L = umin((uint32_t)pl[0], (uint32_t)pl[1]);
  H = smax((uint32_t)ph[0], (uint32_t)ph[1]);
}
// the group's umax of U and smax of S at once (two independent chains)
template <int G>
__device__ __forceinline__ void grp_red2(uint32_t& U, uint32_t& S) {
#define RED2_STEP(CTRL)                                                                  \
  {                                                                                      \
    const uint32_t u = (uint32_t)__builtin_amdgcn_mov_dpp((int)U, CTRL, 0xF, 0xF, false); \
    const uint32_t s = (uint32_t)__builtin_amdgcn_mov_dpp((int)S, CTRL, 0xF, 0xF, false); \
    U = umax(U, u);                                                                      \
    S = smax(S, s);                                                                      \
  }
  RED2_STEP(DPP_ROW_ROR(8))
  RED2_STEP(DPP_ROW_ROR(4))
  RED2_STEP(DPP_ROW_ROR(2))
  RED2_STEP(DPP_ROW_ROR(1))
#undef RED2_STEP
  if constexpr (G == 16) return;
  const auto pu = __builtin_amdgcn_permlane16_swap(U, U, false, false);
  const auto ps = __builtin_amdgcn_permlane16_swap(S, S, false, false);
  U = umax((uint32_t)pu[0], (uint32_t)pu[1]);
  S = smax((uint32_t)ps[0], (uint32_t)ps[1]);
}
__device__ __forceinline__ uint32_t half_smax(uint32_t x) {
  x = smax(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(8), 0xF, 0xF, false));
  x = smax(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(4), 0xF, 0xF, false));
  x = smax(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(2), 0xF, 0xF, false));
  x = smax(x, (uint32_t)__builtin_amdgcn_mov_dpp((int)x, DPP_ROW_ROR(1), 0xF, 0xF, false));
  const auto p = __builtin_amdgcn_permlane16_swap(x, x, false, false);
  return smax((uint32_t)p[0], (uint32_t)p[1]);
}
}  // namespace pk16

// one ksw_extend2 call of a sub-slot (per lane, uniform over its half)
struct QCall {
  int qlen, qa, qd, tlen, w, eb, zdrop, h0;
  const uint8_t* q;   // query bytes: column j at q[qa + qd * j]
  const uint8_t* tb;  // target rows (LDS), at least tlen + 1 bytes
};

// a sub-slot without a task: no rows (its result is ignored)
__device__ __forceinline__ QCall quad_idle(const uint8_t* seq, const uint8_t* tb) {
  QCall q;
  q.qlen = 1;
  q.tlen = 0;
  q.qa = 0;
  q.qd = 1;
  q.eb = 0;
  q.h0 = 1;
  q.w = 1;
  q.zdrop = 0;
  q.q = seq;
  q.tb = tb;
  return q;
}

// K8: the row-max key is H << 8 | j, packed, one reduction for both calls
// (every H < 256: quad_key8_ok); else H << KS | c widened to H << 10 | j per call.
// G = the lanes of a group (two calls): 32 (four calls per wave) or 16 (eight
// calls per wave, K8 only: every scan and reduction stays inside a DPP row).
// SYM: o_del == o_ins, so E's and F's gap-open terms share one subtraction of
// the biased M per column.
template <int G, int CPL, bool K8, bool SYM>
__device__ __forceinline__ void extend_quad(const DevOpt& o, const QCall& A, const QCall& Bc, ExtOut& xa, ExtOut& xb,
                                            Tally32& ta, Tally32& tbl) {
  using namespace pk16;
  static_assert(G == 32 || G == 16, "four (G = 32) or eight (G = 16) calls per wave");
  int r;  // the lane index in its group, behind an opaque move (see extend_pair)
  if constexpr (G == 16) asm volatile("v_and_b32 %0, 15, %1" : "=v"(r) : "v"((int)threadIdx.x));
  else asm volatile("v_and_b32 %0, 31, %1" : "=v"(r) : "v"((int)threadIdx.x));
  constexpr int KS = CPL <= 2 ? 1 : (CPL <= 4 ? 2 : (CPL <= 8 ? 3 : 4));  // in-lane column bits of the key
  static_assert(CPL >= 1 && CPL * G <= 256, "columns per call: < 256 (16-bit j, 8-bit key)");
  const int e_del = o.e_del, e_ins = o.e_ins, oe_ins = o.oe_ins;
  const int j0 = r * CPL;
  const uint32_t J0 = pk(j0, j0);
  const uint32_t EI1 = pk(e_ins, e_ins), ED1 = pk(e_del, e_del);
  // F's gap open from the biased M (the e_ins of F(j+1) = max(F(j), M(j) - o_ins)
  // - e_ins is taken after the max), E's likewise with o_del
  const uint32_t MB_OI = pk(128 + o.o_ins, 128 + o.o_ins), OI1 = pk(o.o_ins, o.o_ins);
  const uint32_t MB_OD = SYM ? MB_OI : pk(128 + o.o_del, 128 + o.o_del);
  const int sk = 32 - __builtin_clz((unsigned)max(o.max_mat, 1));  // 2^sk > max(mat)
  const uint32_t KSH = pk(1 << sk, 1 << sk);
  const uint32_t RE = pk(e_ins * j0, e_ins * j0), RE2 = pk(e_ins * (j0 + CPL), e_ins * (j0 + CPL));
  // the key's multiplier kept opaque: a visible power of two makes LLVM split
  // the v_pk_mad_u16 into a shift and an add
  const uint32_t KMUL = opq(K8 ? pk(256, 256) : pk(1 << KS, 1 << KS));
  uint32_t hh[CPL], ee[CPL], pfa[CPL], pfb[CPL], qm[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    const int j = j0 + c;
    const int qva = A.q[A.qa + A.qd * min(j, A.qlen - 1)];  // unconditional loads (qlen >= 1)
    const int qvb = Bc.q[Bc.qa + Bc.qd * min(j, Bc.qlen - 1)];
    pfa[c] = qprof_word(o, j < A.qlen ? qva : 0) ^ 0x80808080u;  // bytes biased by 128
    pfb[c] = qprof_word(o, j < Bc.qlen ? qvb : 0) ^ 0x80808080u;
    const int va = j == 0 ? A.h0 : max(A.h0 - oe_ins - (j - 1) * e_ins, 0);  // ksw.c:392-395
    const int vb = j == 0 ? Bc.h0 : max(Bc.h0 - oe_ins - (j - 1) * e_ins, 0);
    hh[c] = pk(j <= A.qlen ? va : 0, j <= Bc.qlen ? vb : 0);
    ee[c] = 0;
    qm[c] = pk(j == A.qlen - 1 ? 0xffff : 0, j == Bc.qlen - 1 ? 0xffff : 0);
  }
  // band clamp (ksw.c:399-407)
  const int wa = min(A.w, min(band_cap_dev(A.qlen, o.max_mat, A.eb, o.o_ins, e_ins),
                              band_cap_dev(A.qlen, o.max_mat, A.eb, o.o_del, e_del)));
  const int wb = min(Bc.w, min(band_cap_dev(Bc.qlen, o.max_mat, Bc.eb, o.o_ins, e_ins),
                               band_cap_dev(Bc.qlen, o.max_mat, Bc.eb, o.o_del, e_del)));
  const uint32_t QL = pk(A.qlen, Bc.qlen);
  uint32_t LO = 0, HI = QL;
  uint32_t IW = pk(-wa, -wb), IW1 = pk(wa + 1, wb + 1);
  uint32_t GL = pk(A.h0 - o.o_del - e_del, Bc.h0 - o.o_del - e_del);  // h0 - (o_del + e_del (i+1))
  uint32_t EI = pk(-1, -1), ESC = pk(-1, -1);
  // the row-end state of both calls, packed (ksw.c:454-465): max, its cell,
  // max_off, the rows run, and DM = 0xffff once a call has ended
  uint32_t BEST = pk(A.h0, Bc.h0), BI = pk(-1, -1), BJ = pk(-1, -1), OFF = 0, I = 0;
  uint32_t ROWS = pk(max(A.tlen, 0), max(Bc.tlen, 0));
  uint32_t DM = pk(A.tlen <= 0 ? 0xffff : 0, Bc.tlen <= 0 ? 0xffff : 0);
  const uint32_t ZD = pk(min(A.zdrop, 32767), min(Bc.zdrop, 32767));
  const uint32_t ZDM = pk(A.zdrop > 0 ? 0xffff : 0, Bc.zdrop > 0 ? 0xffff : 0);
  const uint32_t TL2 = pk(A.tlen - 2, Bc.tlen - 2);  // i + 1 >= tlen <=> tlen - 2 - i < 0
  // row bound (below): (qlen - j) * max(mat) per column, and qlen * max(mat)
  uint32_t KQ[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) KQ[c] = pk((A.qlen - j0 - c) * o.max_mat, (Bc.qlen - j0 - c) * o.max_mat);
  const uint32_t QLA = pk(A.qlen * o.max_mat, Bc.qlen * o.max_mat);
  int cellsa = 0, cellsb = 0;
  int tna = A.tb[0], tnb = Bc.tb[0];
  // rows run while a call of the wave is live; the exit test is at the bottom
  // (bottom-tested: with the test at the top LLVM copied the loop-carried
  // state between registers on every row)
  int i = 0;
  if (__builtin_amdgcn_ballot_w64(DM != 0xffffffffu)) do {
    const int ta = tna, tbb = tnb;
    tna = A.tb[min(i + 1, max(A.tlen - 1, 0))];  // prefetch
    tnb = Bc.tb[min(i + 1, max(Bc.tlen - 1, 0))];
    // the band (ksw.c:415-419); an ended call: lo = 0x7fff, hi = 0
    LO = sel(DM, 0x7fff7fffu, smax(LO, IW));
    HI = sel(DM, 0u, smin(smin(HI, IW1), QL));
    IW = add(IW, ONE);
    IW1 = add(IW1, ONE);
    const uint32_t WD = usat(HI, LO);
    const uint32_t LEFT0 = neg15(sub(LO, ONE)) & smax(GL, 0u);  // the first-column value where lo == 0
    GL = ssat(GL, ED1);
    const uint32_t SEL = (uint32_t)ta | ((uint32_t)tbb << 16) | 0x0c040c00u;
    // XO: M' + 128 (M - o_ins with SYM, which E reads too); AA: M - o_ins in
    // the band, 0 out of it
    uint32_t XO[CPL], AA[CPL], CAP[CPL], R[CPL];
    uint32_t T = 0;
    // j <= hi  <=>  j - 1 < hi: column c's R is column c-1's "j < hi"
    R[0] = neg15(sub(add(J0, 0xffffffffu), HI));
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const uint32_t JC = add(J0, pk(c, c));
      const uint32_t ltlo = neg15(sub(JC, LO));  // j < lo
      const uint32_t lthi = neg15(sub(JC, HI));  // j < hi
      if (c + 1 < CPL) R[c + 1] = lthi;
      CAP[c] = lthi & ~ltlo;                     // lo <= j < hi
      const uint32_t sb = __builtin_amdgcn_perm(pfb[c], pfa[c], SEL);
      const uint32_t mb = smin(add(hh[c], sb), mad(hh[c], KSH, 0x00800080u));  // M' + 128
      const uint32_t xi = sub(mb, MB_OI);
      XO[c] = SYM ? xi : mb;
      AA[c] = umin(xi, CAP[c]);
      T = usat(smax(T, AA[c]), EI1);  // max(T - e_ins, M - oe_ins, 0)
    }
    const uint32_t sx = grp_scan_umax<G>(add(T, RE2));
    uint32_t EX;
    if constexpr (G == 16) {
      EX = mov0<DPP_ROW_SHR(1)>(sx);  // a row's lane 0 reads 0: no column to its left
    } else {
      EX = mov0<DPP_WAVE_SHR1>(sx);
      EX = r == 0 ? 0u : EX;  // lanes 0 and 32: no column to the left in the half
    }
    uint32_t f = usat(EX, RE);
    uint32_t LK = 0, H1Q = 0, hm[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (c > 0) f = usat(smax(f, AA[c - 1]), EI1);
      const uint32_t m = SYM ? add(XO[c], OI1) : sub(XO[c], 0x00800080u);  // M
      const uint32_t xd = SYM ? XO[c] : sub(XO[c], MB_OD);                   // M - o_del
      const uint32_t h = smax(smax(m, ee[c]), f);
      hm[c] = umin(h, CAP[c]);
      const uint32_t en = usat(smax(ee[c], xd), ED1);
      if constexpr (K8)
        LK = umax(LK, mad(hm[c], KMUL, add(J0, pk(c, c))));
      else
        LK = umax(LK, mad(hm[c], KMUL, pk(c, c)));
      ee[c] = sel(R[c], umin(en, CAP[c]), ee[c]);
      if (c > 0) hh[c] = sel(R[c], hm[c - 1], hh[c]);
      H1Q |= hm[c] & qm[c];
    }
    uint32_t hs0;  // H(i, j0 - 1); the group's first lane: the first-column value
    if constexpr (G == 16) {
      hs0 = (uint32_t)__builtin_amdgcn_update_dpp((int)LEFT0, (int)hm[CPL - 1], DPP_ROW_SHR(1), 0xF, 0xF, false);
    } else {
      hs0 = mov0<DPP_WAVE_SHR1>(hm[CPL - 1]);
      hs0 = r == 0 ? LEFT0 : hs0;
    }
    hh[0] = sel(R[0], hs0, hh[0]);
    // band trim candidates (ksw.c:466-469): the first and the last column j <=
    // hi whose stored H or E is non-zero (H, E >= 0).  No lower bound is
    // needed: every column left of lo was just written with H = E = 0 (out of
    // the band, j <= hi), and a live call has lo <= hi (else its row maximum is
    // 0 and it ends in this row).  CH carries last + 1 ("none": 0).
    uint32_t CL = 0x7fff7fffu, CH = 0;
#pragma unroll
    for (int c = CPL - 1; c >= 0; --c) {
      const uint32_t nz = neg15(sub(0u, hh[c] | ee[c]));  // 0xffff where H or E is non-zero
      CL = sel(nz, add(J0, pk(c, c)), CL);
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const uint32_t nz = neg15(sub(0u, hh[c] | ee[c]));
      CH = sel(nz & R[c], add(J0, pk(c + 1, c + 1)), CH);
    }
    // the row maxima (ksw.c:433: the LAST column of the maximum) and the trim,
    // reduced over the half: MROW = the row's max H, MJ = its column
    uint32_t MROW, MJ;
    if constexpr (K8) {
      uint32_t K = LK;
      grp_red3<G>(K, CL, CH);
      MROW = W(U(K) >> (u16x2){8, 8});
      MJ = K & 0x00ff00ffu;
    } else {
      const uint32_t lka = LK & 0xffffu, lkb = LK >> 16;
      int ka = (int)(((lka >> KS) << 10) | (uint32_t)(j0 + (int)(lka & ((1u << KS) - 1))));
      int kb = (int)(((lkb >> KS) << 10) | (uint32_t)(j0 + (int)(lkb & ((1u << KS) - 1))));
      if constexpr (G == 16) {  // every reduction inside the group's DPP row
#define RED4_STEP(CTRL)                                                                   \
  {                                                                                       \
    const int a_ = __builtin_amdgcn_mov_dpp(ka, CTRL, 0xF, 0xF, false);                   \
    const int b_ = __builtin_amdgcn_mov_dpp(kb, CTRL, 0xF, 0xF, false);                   \
    const uint32_t l_ = (uint32_t)__builtin_amdgcn_mov_dpp((int)CL, CTRL, 0xF, 0xF, false); \
    const uint32_t h_ = (uint32_t)__builtin_amdgcn_mov_dpp((int)CH, CTRL, 0xF, 0xF, false); \
    ka = max(ka, a_);                                                                     \
    kb = max(kb, b_);                                                                     \
    CL = umin(CL, l_);                                                                    \
    CH = smax(CH, h_);                                                                    \
  }
        RED4_STEP(DPP_ROW_ROR(8))
        RED4_STEP(DPP_ROW_ROR(4))
        RED4_STEP(DPP_ROW_ROR(2))
        RED4_STEP(DPP_ROW_ROR(1))
#undef RED4_STEP
      } else {
        ka = half_max(row_max32(ka));
        kb = half_max(row_max32(kb));
        CL = half_umin(CL);
        CH = half_smax(CH);
      }
      MROW = pk(ka >> 10, kb >> 10);
      MJ = pk(ka & 1023, kb & 1023);
    }
    // ksw.c:450-453 (meaningful on the owner of column qlen-1)
    {
      const uint32_t AT = neg15(sub(umin(sub(smax(LO, HI), QL), ONE), ONE));  // 0xffff where max(lo, hi) == qlen
      EI = sel(AT & ~neg15(sub(H1Q, ESC)), pk(i, i), EI);
      ESC = sel(AT, smax(ESC, H1Q), ESC);
    }
    cellsa += (int)(WD & 0xffffu);
    cellsb += (int)(WD >> 16);
    // ksw.c:454-465 on both calls at once (16-bit: quad_rows_ok); branch-free:
    // an ended call's row maximum is 0, which changes nothing but its break
    {
      const uint32_t UP = neg15(sub(BEST, MROW));  // m > max
      const uint32_t DD = sub(sub(I, BI), sub(MJ, BJ));
      const uint32_t DROP = sub(sub(BEST, MROW), smax(mul(DD, ED1), mul(sub(0u, DD), EI1)));
      const uint32_t BRK = neg15(sub(MROW, ONE)) | (~UP & ZDM & neg15(ssat(ZD, DROP)));  // m == 0 or a z-drop
      ROWS = sel(~DM & BRK, add(I, ONE), ROWS);
      OFF = sel(UP, smax(OFF, smax(sub(MJ, I), sub(I, MJ))), OFF);
      BEST = sel(UP, MROW, BEST);
      BI = sel(UP, I, BI);
      BJ = sel(UP, MJ, BJ);
      DM = DM | BRK | neg15(sub(TL2, I));  // a break, or its last target row
      I = add(I, ONE);
    }
    // the next row's band (ksw.c:466-469)
    const uint32_t NLO = smin(CL, HI);
    LO = NLO;
    HI = smin(add(smax(CH, NLO), ONE), QL);  // min(max(last, lo - 1) + 2, qlen)
    // Row bound, every fourth row: a cell of a later row is reached from a
    // stored diagonal value v = H(i, j-1) > 0 of column j (or from the first
    // column's h0 - o_del - e_del (i+2) while lo == 0) by at most qlen - j
    // matches, so no later cell exceeds B = max(v + (qlen - j) max(mat)).  (E
    // of column j is <= H(i, j) = the diagonal value of column j+1, and 0 at
    // and right of hi.)  Once B < gscore (<= max), no later row can move max,
    // its cell, max_off (ksw.c:454: m > max) or gscore / max_ie (ksw.c:450-453:
    // a tie moves max_ie), so the call ends with every output unchanged.
    if (o.row_bound && (i & RB_MASK) == RB_MASK) {
      uint32_t BB = neg15(sub(LO, ONE)) & neg15(sub(0u, GL)) & add(GL, QLA), SC = ESC;
#pragma unroll
      for (int c = 0; c < CPL; ++c) BB = umax(BB, neg15(sub(0u, hh[c])) & add(hh[c], KQ[c]));
      grp_red2<G>(BB, SC);
      const uint32_t STOP = neg15(sub(BB, SC)) & ~DM;  // B < gscore
      ROWS = sel(STOP, I, ROWS);
      DM |= STOP;
    }
    ++i;
    // the next row's target bases stay loaded in this row (else LLVM moves the
    // loads to the next row's top, in front of their only use)
    asm volatile("" : "+v"(tna), "+v"(tnb));
  } while (__builtin_amdgcn_ballot_w64(DM != 0xffffffffu));
  // gscore / max_ie from the owner of column qlen-1 of each call
  const int hb = (int)(threadIdx.x & (64 - G));  // the group's first lane
  const uint32_t ea = __shfl(pk(lo16(EI), lo16(ESC)), hb + (A.qlen - 1) / CPL, 64);
  const uint32_t eb = __shfl(pk(hi16(EI), hi16(ESC)), hb + (Bc.qlen - 1) / CPL, 64);
  xa = ExtOut{lo16(BEST), lo16(BJ) + 1, lo16(BI) + 1, lo16(ea) + 1, hi16(ea), lo16(OFF)};
  xb = ExtOut{hi16(BEST), hi16(BJ) + 1, hi16(BI) + 1, lo16(eb) + 1, hi16(eb), hi16(OFF)};
  ta.cells += cellsa;
  ta.rows += lo16(ROWS);
  ta.calls += 1;
  tbl.cells += cellsb;
  tbl.rows += hi16(ROWS);
  tbl.calls += 1;
}

// CPL = ceil((qlen+1)/G) of the wave's longest active call (all run one body)
template <int G, int PMAX, bool K8>
__device__ __forceinline__ void extend_quad_dispatch(const DevOpt& o, const QCall& A, const QCall& Bc, ExtOut& xa,
                                                     ExtOut& xb, Tally32& ta, Tally32& tbl) {
  int qm = 0;
#pragma unroll
  for (int g = 0; g < 64; g += G)
    qm = max(qm, max(__builtin_amdgcn_readlane(A.qlen, g), __builtin_amdgcn_readlane(Bc.qlen, g)));
  const int cpl = (qm + G) / G;
#ifndef BWAGPU_QUAD_SYM
#define BWAGPU_QUAD_SYM 1
#endif
  const bool sym = BWAGPU_QUAD_SYM && o.o_del == o.o_ins;  // bwa's defaults: 6 / 6
#define EXT_QUAD(n)                                                                            \
  if (n <= PMAX && cpl == n) {                                                                 \
    if (sym) return extend_quad<G, (n <= PMAX ? n : 1), K8, true>(o, A, Bc, xa, xb, ta, tbl);  \
    return extend_quad<G, (n <= PMAX ? n : 1), K8, false>(o, A, Bc, xa, xb, ta, tbl);          \
  }
  EXT_QUAD(1) EXT_QUAD(2) EXT_QUAD(3) EXT_QUAD(4) EXT_QUAD(5) EXT_QUAD(6) EXT_QUAD(7) EXT_QUAD(8) EXT_QUAD(9)
  EXT_QUAD(10) EXT_QUAD(11) EXT_QUAD(12) EXT_QUAD(13) EXT_QUAD(14) EXT_QUAD(15) EXT_QUAD(16)
#undef EXT_QUAD
}

// rows that extend_group can read for (qlen, w, end_bonus)
__device__ __forceinline__ int rows_needed(const DevOpt& o, int qlen, int tlen, int w, int end_bonus) {
  int mi = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_ins, o.e_ins);
  int md = band_cap_dev(qlen, o.max_mat, end_bonus, o.o_del, o.e_del);
  int we = min(w, min(mi, md));
  return min(tlen, qlen + we + 1);
}

// Gather the target rows of one extension into the group's LDS row buffer:
// row k is 2-strand coordinate x0 + dir*k.  Loop bounds are group-uniform and
// the body branch-free (tail lanes re-write row n-1), and eight loads per lane
// are issued before any is consumed: one HBM round trip per 8*G rows.
template <int G>
__device__ __forceinline__ void fill_target(uint8_t* tb, const DevRef& ref, int64_t x0, int dir, int n) {
  const int r = Grp<G>::lane();
  const int64_t two1 = (ref.l_pac << 1) - 1;
  for (int base = 0; base < n; base += 8 * G) {
    uint32_t raw[8];
    int sh[8];
    bool rev[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int kk = min(base + m * G + r, n - 1);
      const int64_t x = x0 + (int64_t)dir * kk;
      rev[m] = x >= ref.l_pac;
      const int64_t f = rev[m] ? two1 - x : x;
      raw[m] = ref.pac[f >> 2];
      sh[m] = (int)((~f & 3) << 1);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int kk = min(base + m * G + r, n - 1);
      const int b = (raw[m] >> sh[m]) & 3;
      tb[kk] = (uint8_t)(rev[m] ? 3 - b : b);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void mem_fence_group() {
  // the group (one wave or part of one) re-reads global data it wrote itself;
  // same-CU ordering: workgroup scope is sufficient (non-tgsplit mode)
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
}

template <int G>
__device__ void block_stats(const Tally& tl, int64_t* stats) {
  if (!stats) return;
  long long c = tl.cells, r = tl.rows, k = tl.calls;
  // only group leaders carry the read's tally; sum over the wave, then atomics
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o, 64);
    r += __shfl_xor(r, o, 64);
    k += __shfl_xor(k, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (c) atomicAdd((unsigned long long*)&stats[ST_CELLS], (unsigned long long)c);
    if (r) atomicAdd((unsigned long long*)&stats[ST_ROWS], (unsigned long long)r);
    if (k) atomicAdd((unsigned long long*)&stats[ST_CALLS], (unsigned long long)k);
  }
}

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)((uint64_t)hi << 32 | lo);
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)((uint64_t)hi << 32 | lo);
}

// resident workgroups of a kernel over the whole device (persistent grids).
// The answer depends on the kernel, its dynamic LDS bytes (which change per
// batch with the read lengths and options) and the device, so it is cached
// under exactly that key; GPU worker threads of several contexts call this
// concurrently.
template <typename K>
static int resident_blocks(K kernel, size_t lds, int block = kBlock) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 1024;
  struct Key {
    const void* k;
    size_t lds;
    int dev;
    bool operator<(const Key& o) const { return std::tie(k, lds, dev) < std::tie(o.k, o.lds, o.dev); }
  };
  static std::mutex mu;
  static std::map<Key, int> cache;
  const Key key{reinterpret_cast<const void*>(kernel), lds, dev};
  {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  int ncu = 0, per = 0;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 1024;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, block, lds) != hipSuccess || per < 1) per = 1;
  std::lock_guard<std::mutex> g(mu);
  return cache[key] = per * ncu;
}

// Both extensions' target rows of one seed in ONE HBM round trip: left rows
// x0l - k (k < nl) into tbl, right rows x0r + k (k < nr) into tbr.
__device__ __forceinline__ void fill_two(uint8_t* tbl, int64_t x0l, int nl, uint8_t* tbr, int64_t x0r, int nr,
                                         const DevRef& ref) {
  const int r = (int)(threadIdx.x & 63);
  const int64_t two1 = (ref.l_pac << 1) - 1;
  const int n = max(nl, nr);
  for (int base = 0; base < n; base += 256) {
    uint32_t raw[8];
    int sh[8], kk[8];
    bool rev[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const bool left = m < 4;
      const int nn = left ? nl : nr;
      const int k = min(base + (m & 3) * 64 + r, max(nn - 1, 0));
      kk[m] = k;
      const int64_t x = left ? x0l - k : x0r + k;
      rev[m] = x >= ref.l_pac;
      int64_t f = rev[m] ? two1 - x : x;
      f = f < 0 ? 0 : (f >= ref.l_pac ? ref.l_pac - 1 : f);  // only for an empty side (nn == 0)
      raw[m] = ref.pac[f >> 2];
      sh[m] = (int)((~f & 3) << 1);
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int bse = (raw[m] >> sh[m]) & 3;
      const uint8_t v = (uint8_t)(rev[m] ? 3 - bse : bse);
      if (m < 4) {
        if (nl > 0) tbl[kk[m]] = v;
      } else {
        if (nr > 0) tbr[kk[m]] = v;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ ReadDesc uniform_desc(const ReadDesc& d) {
  ReadDesc u;
  u.qoff = uni64(d.qoff);
  u.rd = uni(d.rd);
  u.lq = uni(d.lq);
  u.c0 = uni(d.c0);
  u.nch = uni(d.nch);
  u.s0 = uni(d.s0);
  u.ns = uni(d.ns);
  return u;
}

// wave-aggregated append: returns the slot of each predicated lane (-1 else)
__device__ __forceinline__ int wave_append(int32_t* cnt, bool p) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(p);
  if (m == 0) return -1;
  const int leader = __builtin_ctzll(m);
  int base = 0;
  if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(cnt, (int)__popcll(m));
  base = __shfl(base, leader, 64);
  const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  return p ? base + rank : -1;
}

// Dynamic queue with one head per XCD, each on its own 128-byte line
// (MI355X_MICROARCH.md "dequeue": one head word saturates at ~88 dequeues/us,
// and so do heads sharing a line): shard x holds list positions x, x + 8,
// ...; a wave claims K consecutive entries of a shard with one atomic, starting
// on its own XCD's shard and moving on when it runs dry.  Every position is
// taken exactly once by whichever waves exist; placement is never assumed.
struct ShardQ {
  int32_t* heads;
  int n, shard, tried;
  __device__ void init(int32_t* h, int n_) {
    heads = h;
    n = n_;
    shard = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7;  // HW_REG_XCC_ID
    tried = 0;
  }
  // -> first claimed entry index m0 of `shard` (positions shard + 8m, m < cap)
  __device__ bool claim(int K, int& m0, int& cap) {
    while (tried < 8) {
      cap = n > shard ? (n - shard + 7) >> 3 : 0;
      int32_t* h = heads + shard * kQHStride;
      // the wave's own shard is claimed from at once (one round trip); an
      // exhausted head only grows past cap.  Other shards are read first, so
      // that waves that have run dry do not hammer every head with atomics
      if (tried == 0 || __hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cap) {
        int v = 0;
        if ((threadIdx.x & 63) == 0) v = atomicAdd(h, K);
        v = __builtin_amdgcn_readfirstlane(__shfl(v, 0, 64));
        if (v < cap) {
          m0 = v;
          return true;
        }
      }
      shard = (shard + 1) & 7;
      ++tried;
    }
    return false;
  }
};

__device__ __forceinline__ int spec_bin(int lq) { return lq <= kSpecBinLen[0] ? 0 : (lq <= kSpecBinLen[1] ? 1 : 2); }

// the raw extent of a chain's seeds' reach (bwamem.c:650-657), min / max
__device__ __forceinline__ void seed_reach(const DevOpt& o, const bwagpu_seed_t& t, int lq, int64_t& wlo,
                                           int64_t& whi) {
  const int tail = lq - t.qbeg - t.len;
  wlo = min(wlo, t.rbeg - (int64_t)(t.qbeg + max_gap_len(o, t.qbeg)));
  whi = max(whi, t.rbeg + t.len + (int64_t)(tail + max_gap_len(o, tail)));
}

// the rest of the window (bwamem.c:658-668 + bns_fetch_seq's clipping,
// bntseq.c:421-446): clamp, one strand, the contig of the first seed; false
// when that seed is not in contig rid (where bwa asserts, bwamem.c:669)
__device__ __forceinline__ bool finish_window(const DevRef& ref, int rid, int64_t mid, int64_t& wlo, int64_t& whi) {
  const int64_t two = ref.l_pac << 1;
  wlo = max(wlo, (int64_t)0);
  whi = min(whi, two);
  if (wlo < ref.l_pac && ref.l_pac < whi) {
    if (mid < ref.l_pac) whi = ref.l_pac;
    else wlo = ref.l_pac;
  }
  bool ok = rid >= 0 && rid < ref.n_seqs;
  if (ok) {
    const int64_t fpos = mid >= ref.l_pac ? two - 1 - mid : mid;
    int64_t cb = ref.ann_offset[rid], ce = cb + ref.ann_len[rid];
    ok = fpos >= cb && fpos < ce;
    if (mid >= ref.l_pac) {
      const int64_t t0 = cb;
      cb = two - ce;
      ce = two - t0;
    }
    wlo = max(wlo, cb);
    whi = min(whi, ce);
  }
  return ok;
}

// One seed's extension (bwamem.c:717-792) by one wave: both target windows
// gathered in one round trip, left ksw_extend2 (reversed query prefix and
// window) with the MAX_BAND_TRY retry, right ksw_extend2 from the left score,
// the local vs to-end choice of each side.  s, lq, cw are wave-uniform.
template <int C>
__device__ __forceinline__ SeedExt extend_seed(const DevOpt& o, const DevRef& ref, const bwagpu_seed_t& s, int lq,
                               const uint8_t* q, const ChainWin& cw, uint8_t* tbl, uint8_t* tbr) {
  Tally tl{0, 0, 0};
  const int qlenL = s.qbeg, qlenR = lq - (s.qbeg + s.len);
  const int64_t x0L = s.rbeg - 1, x0R = s.rbeg + s.len;
  const int tlenL = (int)(s.rbeg - cw.lo), tlenR = (int)(cw.hi - x0R);
  fill_two(tbl, x0L, qlenL ? rows_needed(o, qlenL, tlenL, o.w << 1, o.pen_clip5) : 0, tbr, x0R,
           qlenR ? rows_needed(o, qlenR, tlenR, o.w << 1, o.pen_clip3) : 0, ref);
  int score = -1, truesc = -1, qb = 0, qe = lq, sc0 = 0;
  int aw0 = o.w, aw1 = o.w;
  int64_t rb = s.rbeg, re = s.rbeg + s.len;
#pragma nounroll
  for (int side = 0; side < 2; ++side) {
    const bool left = side == 0;
    if (left && s.qbeg == 0) {  // bwamem.c:753
      score = truesc = s.len * o.a;
      continue;
    }
    if (!left && qlenR == 0) continue;  // bwamem.c:781
    const int qlen = left ? qlenL : qlenR;
    const int64_t x0 = left ? x0L : x0R;
    const int tlen = left ? tlenL : tlenR;
    const int qa = left ? s.qbeg - 1 : s.qbeg + s.len;
    const int eb = left ? o.pen_clip5 : o.pen_clip3;
    const int h0 = left ? s.len * o.a : score;
    uint8_t* const tb = left ? tbl : tbr;
    sc0 = score;
    ExtOut x{};
    for (int t = 0; t < 2; ++t) {  // MAX_BAND_TRY (bwamem.c:639)
      const int prev = score;
      const int aw = o.w << t;
      aw0 = left ? aw : aw0;
      aw1 = left ? aw1 : aw;
      x = extend_wave_dispatch<C, false>(o, qlen, q, qa, left ? -1 : 1, tlen, tb, aw, eb, o.zdrop, h0, tl);
      score = x.score;
      if (score == prev || x.max_off < (aw >> 1) + (aw >> 2)) break;
    }
    const bool local = x.gscore <= 0 || x.gscore <= score - eb;
    if (left) {
      qb = local ? s.qbeg - x.qle : 0;
      rb = s.rbeg - (local ? x.tle : x.gtle);
      truesc = local ? score : x.gscore;
    } else {
      qe = local ? qa + x.qle : lq;
      re = x0 + (local ? x.tle : x.gtle);
      truesc += (local ? score : x.gscore) - sc0;
    }
  }
  SeedExt e;
  e.rb = rb;
  e.re = re;
  e.qb = qb;
  e.qe = qe;
  e.score = score;
  e.truesc = truesc;
  e.w = aw0 > aw1 ? aw0 : aw1;
  e.cells = (int32_t)tl.cells;
  e.rows = (int32_t)tl.rows;
  e.calls = (int32_t)tl.calls + 1;  // + 1: a computed slot is never all-zero
  return e;
}


__device__ __forceinline__ void store_ext(SeedExt* dst, const SeedExt& e) {
  const int d = (int)(threadIdx.x & 63);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&e);
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) v = d == k ? w[k] : v;
  if (d < 12) reinterpret_cast<uint32_t*>(dst)[d] = v;
}

__device__ __forceinline__ bwagpu_seed_t uni_seed(const bwagpu_seed_t& s) {
  bwagpu_seed_t u;
  u.rbeg = uni64(s.rbeg);
  u.qbeg = uni(s.qbeg);
  u.len = uni(s.len);
  u.score = uni(s.score);
  u.pad_ = uni(s.pad_);
  return u;
}

}  // namespace bwagpu
