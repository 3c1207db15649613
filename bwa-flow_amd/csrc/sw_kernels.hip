// sw_kernels.hip — MI355X (gfx950) seed-extension kernels.
//
// The hot path of bwa-flow's ChainsToRegions stage (src/Pipeline.cpp:503-544):
// for every read, every chain goes through mem_chain2aln (bwa/bwamem.c:641-795),
// whose inner loop is the banded affine-gap extension ksw_extend2
// (bwa/ksw.c:380-479).  Integer DP, VALU-bound, no MFMA.
//
// Mapping to CDNA4:
//  * one GROUP of G lanes (G = 16/32/64, a divisor of the 64-wide wave) owns one
//    read for the whole of mem_chain2aln: window, seed order, containment test,
//    left/right extensions with band retries, seedcov, region output.  The
//    read's intra-chain sequential dependencies (containment of later seeds in
//    earlier regions, left->right h0 chaining) stay inside the group, so the
//    whole stage is one launch with no host replay.
//  * ksw_extend2 runs row by row over the target with the query columns spread
//    over the group's lanes in contiguous blocks of Cd = ceil((qlen+1)/G)
//    columns.  Everything the reference keeps in eh[] (H of the previous row
//    shifted by one column, E) lives in registers; the within-row horizontal
//    gap F, a left-to-right recurrence in the reference, is turned into a
//    max-plus prefix scan:  F(i,j) = max(0, max_{k<j} (t_k - (j-1-k)*e_ins)),
//    t_k = max(M_k - oe_ins, 0), computed as a lane-local scan + one
//    group-exclusive scan of u_k = t_k + k*e_ins.
//  * row max + LAST argmax in one reduction of the key (H << 10 | j).
//  * band trimming (ksw.c:466-469) by min/max reductions of the non-zero columns.
//  * target rows are gathered once per task from the HBM-resident 2-bit pac
//    (bntseq.c:225 bit order; reverse strand = complement of mirrored forward,
//    bntseq.c:405-411) into a per-group LDS row buffer.
//
// Every value that steers control flow (band, maxima, breaks) is identical in
// all lanes of a group, so groups of one wave diverge only from each other.
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>
#include <map>
#include <atomic>
#include <mutex>
#include <tuple>

#include "engine.h"
#include "wave_ops.h"

namespace bwagpu {

const Variant kVariants[kNumVariants] = {{64, 3, VK_FAST}, {64, 4, VK_FAST}, {64, 16, VK_GENERIC}};
const Variant kExtVariants[kNumExtVariants] = {{64, 3, VK_FAST}, {64, 4, VK_FAST}, {64, 16, VK_GENERIC}};

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

// Optional per-read trace (bwagpu_debug_set_trace): 8 words per read index:
// start/end s_memrealtime (100 MHz), DP rows, DP cells, HW_ID, XCC_ID.
__device__ uint32_t* g_trace = nullptr;

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
// inclusive max-scan over each 32-lane half of packed values >= 0 (identity 0)
__device__ __forceinline__ uint32_t half_scan_umax(uint32_t x) {
  x = umax(x, mov0<DPP_ROW_SHR(1)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(2)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(4)>(x));
  x = umax(x, mov0<DPP_ROW_SHR(8)>(x));
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

template <int CPL>
__device__ __forceinline__ void extend_quad(const DevOpt& o, const QCall& A, const QCall& Bc, ExtOut& xa, ExtOut& xb,
                                            Tally32& ta, Tally32& tbl) {
  using namespace pk16;
  int r;  // the lane index behind an opaque move (see extend_pair)
  asm volatile("v_and_b32 %0, 31, %1" : "=v"(r) : "v"((int)threadIdx.x));
  constexpr int KS = CPL <= 2 ? 1 : (CPL <= 4 ? 2 : (CPL <= 8 ? 3 : 4));  // in-lane column bits of the key
  static_assert(CPL >= 1 && CPL <= 8, "four extensions per wave: CPL <= 8");
  const int e_del = o.e_del, e_ins = o.e_ins, oe_ins = o.oe_ins;
  const int j0 = r * CPL;
  const uint32_t J0 = pk(j0, j0);
  const uint32_t EI1 = pk(e_ins, e_ins), ED1 = pk(e_del, e_del);
  const uint32_t MB_OE = pk(128 + oe_ins, 128 + oe_ins), MB_OD = pk(128 + o.o_del, 128 + o.o_del);
  const int sk = 32 - __builtin_clz((unsigned)max(o.max_mat, 1));  // 2^sk > max(mat)
  const uint32_t KSH = pk(1 << sk, 1 << sk);
  const uint32_t RE = pk(e_ins * j0, e_ins * j0), RE2 = pk(e_ins * (j0 + CPL), e_ins * (j0 + CPL));
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
  int cellsa = 0, cellsb = 0;
  int tna = A.tb[0], tnb = Bc.tb[0];
  // rows run while a call of the wave is live; the exit test is at the bottom
  for (int i = 0; __builtin_amdgcn_ballot_w64(DM != 0xffffffffu); ++i) {
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
    const uint32_t HI1 = add(HI, ONE);
    uint32_t MB[CPL], AA[CPL], CAP[CPL], R[CPL], GEL[CPL];
    uint32_t T = 0;
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const uint32_t JC = add(J0, pk(c, c));
      const uint32_t ltlo = neg15(sub(JC, LO));  // j < lo
      R[c] = neg15(sub(JC, HI1));                // j <= hi
      GEL[c] = ~ltlo;
      CAP[c] = neg15(sub(JC, HI)) & ~ltlo;       // lo <= j < hi
      const uint32_t sb = __builtin_amdgcn_perm(pfb[c], pfa[c], SEL);
      const uint32_t mb = smin(add(hh[c], sb), mad(hh[c], KSH, 0x00800080u));  // M' + 128
      MB[c] = mb;
      AA[c] = umin(sub(mb, MB_OE), CAP[c]);
      T = smax(usat(T, EI1), AA[c]);
    }
    const uint32_t sx = half_scan_umax(add(T, RE2));
    uint32_t EX = mov0<DPP_WAVE_SHR1>(sx);
    EX = r == 0 ? 0u : EX;  // lanes 0 and 32: no column to the left in the half
    uint32_t f = usat(EX, RE);
    uint32_t LK = 0, H1Q = 0, hm[CPL];
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      if (c > 0) f = smax(usat(f, EI1), AA[c - 1]);
      const uint32_t h = smax(smax(sub(MB[c], 0x00800080u), ee[c]), f);
      hm[c] = umin(h, CAP[c]);
      const uint32_t en = usat(smax(ee[c], sub(MB[c], MB_OD)), ED1);
      LK = umax(LK, mad(hm[c], pk(1 << KS, 1 << KS), pk(c, c)));
      ee[c] = sel(R[c], umin(en, CAP[c]), ee[c]);
      if (c > 0) hh[c] = sel(R[c], hm[c - 1], hh[c]);
      H1Q |= hm[c] & qm[c];
    }
    uint32_t hs0 = mov0<DPP_WAVE_SHR1>(hm[CPL - 1]);  // H(i, j0 - 1)
    hs0 = r == 0 ? LEFT0 : hs0;
    hh[0] = sel(R[0], hs0, hh[0]);
    // band trim candidates: first non-zero column >= lo, last non-zero <= hi
    uint32_t CL = 0x7fff7fffu, CH = 0xffffffffu;
#pragma unroll
    for (int c = CPL - 1; c >= 0; --c) {
      const uint32_t nz = neg15(sub(0u, hh[c] | ee[c]));  // 0xffff where H or E is non-zero (both >= 0)
      CL = sel(nz & GEL[c], add(J0, pk(c, c)), CL);
    }
#pragma unroll
    for (int c = 0; c < CPL; ++c) {
      const uint32_t nz = neg15(sub(0u, hh[c] | ee[c]));
      CH = sel(nz & R[c], add(J0, pk(c, c)), CH);
    }
    // the row maxima (key H << 10 | j, ksw.c:433) and the trim, reduced over the half
    const uint32_t lka = LK & 0xffffu, lkb = LK >> 16;
    int ka = (int)(((lka >> KS) << 10) | (uint32_t)(j0 + (int)(lka & ((1u << KS) - 1))));
    int kb = (int)(((lkb >> KS) << 10) | (uint32_t)(j0 + (int)(lkb & ((1u << KS) - 1))));
    CL = half_umin(CL);
    CH = half_smax(CH);
    ka = half_max(row_max32(ka));
    kb = half_max(row_max32(kb));
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
      const uint32_t MROW = pk(ka >> 10, kb >> 10), MJ = pk(ka & 1023, kb & 1023);
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
    HI = smin(add(smax(CH, sub(NLO, ONE)), pk(2, 2)), QL);
  }
  // gscore / max_ie from the owner of column qlen-1 of each call
  const int hb = (int)(threadIdx.x & 32);
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

// CPL = ceil((qlen+1)/32) of the wave's longest active call (all four run one body)
template <int PMAX>
__device__ __forceinline__ void extend_quad_dispatch(const DevOpt& o, const QCall& A, const QCall& Bc, ExtOut& xa,
                                                     ExtOut& xb, Tally32& ta, Tally32& tbl) {
  const int qm = max(max(__builtin_amdgcn_readlane(A.qlen, 0), __builtin_amdgcn_readlane(Bc.qlen, 0)),
                     max(__builtin_amdgcn_readlane(A.qlen, 32), __builtin_amdgcn_readlane(Bc.qlen, 32)));
  const int cpl = (qm + 32) >> 5;
#define EXT_QUAD(n) \
  if (n <= PMAX && cpl == n) return extend_quad<(n <= PMAX ? n : 1)>(o, A, Bc, xa, xb, ta, tbl);
  EXT_QUAD(1) EXT_QUAD(2) EXT_QUAD(3) EXT_QUAD(4) EXT_QUAD(5) EXT_QUAD(6) EXT_QUAD(7) EXT_QUAD(8)
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

// ------------------------------------------------------------ chain prep
// One lane per chain: the window [rmax0, rmax1) of mem_chain2aln
// (bwamem.c:648-668, with bns_fetch_seq's contig clipping) and the seed order
// (srt[] = score<<32|i ascending, bwamem.c:671-674).
__global__ void __launch_bounds__(256) chain_prep_kernel(DevOpt o, DevRef ref, DevBatch b, ChainWin* win,
                                                         uint64_t* srt, bwagpu_seed_t* prog, int64_t* stats) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= b.n_chains) return;
  const int s0 = b.chain_seed_off[c], s1 = b.chain_seed_off[c + 1], ns = s1 - s0;
  if (ns <= 0) {
    win[c] = ChainWin{0, 0};
    return;
  }
  // which read owns this chain: binary search over read_chain_off
  int lo_r = 0, hi_r = b.n_reads - 1;
  while (lo_r < hi_r) {
    int mid = (lo_r + hi_r + 1) >> 1;
    if (b.read_chain_off[mid] <= c) lo_r = mid;
    else hi_r = mid - 1;
  }
  const int lq = (int)(b.seq_off[lo_r + 1] - b.seq_off[lo_r]);
  const int64_t two = ref.l_pac << 1;
  int64_t wlo = two, whi = 0;
  for (int i = 0; i < ns; ++i) {
    const bwagpu_seed_t t = b.seeds[s0 + i];
    const int tail = lq - t.qbeg - t.len;
    wlo = min(wlo, t.rbeg - (int64_t)(t.qbeg + max_gap_len(o, t.qbeg)));
    whi = max(whi, t.rbeg + t.len + (int64_t)(tail + max_gap_len(o, tail)));
  }
  wlo = max(wlo, (int64_t)0);
  whi = min(whi, two);
  const int64_t mid = b.seeds[s0].rbeg;
  if (wlo < ref.l_pac && ref.l_pac < whi) {
    if (mid < ref.l_pac) whi = ref.l_pac;
    else wlo = ref.l_pac;
  }
  const int rid = b.chain_rid[c];
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
  if (!ok) {
    atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_RID);
    win[c] = ChainWin{0, -1};
  } else {
    win[c] = ChainWin{wlo, whi};
  }
  // heap sort of the keys, ascending, in place in srt[s0..s1)
  uint64_t* a = srt + s0;
  for (int i = 0; i < ns; ++i) a[i] = (uint64_t)(uint32_t)b.seeds[s0 + i].score << 32 | (uint32_t)i;
  auto sift = [&](int root, int n) {
    uint64_t v = a[root];
    for (;;) {
      int ch = 2 * root + 1;
      if (ch >= n) break;
      if (ch + 1 < n && a[ch + 1] > a[ch]) ++ch;
      if (a[ch] <= v) break;
      a[root] = a[ch];
      root = ch;
    }
    a[root] = v;
  };
  for (int i = ns / 2 - 1; i >= 0; --i) sift(i, ns);
  for (int n = ns - 1; n > 0; --n) {
    uint64_t t = a[0];
    a[0] = a[n];
    a[n] = t;
    sift(0, n);
  }
  // the seeds in processing order (descending key, bwamem.c:676); pad_ flags
  // the key that is 0 from the start, which the overlap test skips like a
  // marked seed (bwamem.c:700)
  for (int t = 0; t < ns; ++t) {
    const uint64_t k = a[ns - 1 - t];
    bwagpu_seed_t v = b.seeds[s0 + (uint32_t)k];
    v.pad_ = k == 0 ? 1 : 0;
    prog[s0 + t] = v;
  }
}

// ------------------------------------------------------------ read order
// Reads are dealt to the wave kernels in order [variant | cost, descending]:
// grouped by kernel variant (read length -> columns per lane; seed/chain
// counts -> fast or generic kernel), and within a variant longest-first
// (LPT), so the static deal of chain2aln_fast_kernel ends with short reads.
// The cost estimate uses the first chain's top seed (the first extension
// mem_chain2aln performs): rows ~ qlen + 16 per side, each row costing
// ~1 + qlen/64 wave-wide segments.  The order is a counting sort over
// kNumVariants x kCostBins bins (histogram -> scan -> scatter), which also
// writes each read's descriptor in its slot.
constexpr int kCostBins = 256;
constexpr int kBins = kNumVariants * kCostBins;

__device__ __forceinline__ int read_variant(const DevBatch& b, int rd, int lq) {
  const int c0 = b.read_chain_off[rd], c1 = b.read_chain_off[rd + 1];
  const int s0 = b.chain_seed_off[c0], s1 = b.chain_seed_off[c1];
  const bool small = s1 - s0 <= kFastMaxSeeds && c1 - c0 <= kFastMaxChains;
  for (int k = 0; k < kNumVariants; ++k)
    if (lq <= kVariants[k].max_len() && (small || kVariants[k].kind != VK_FAST)) return k;
  return -1;
}

__global__ void __launch_bounds__(256) read_bins_kernel(DevBatch b, int32_t* bins, int32_t* hist, int32_t* counts,
                                                        int64_t* stats) {
  __shared__ int h[kBins];
  for (int k = threadIdx.x; k < kBins; k += blockDim.x) h[k] = 0;
  __syncthreads();
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  int v = -1;
  if (rd < b.n_reads) {
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    v = read_variant(b, rd, lq);
    const int c0 = b.read_chain_off[rd], c1 = b.read_chain_off[rd + 1];
    uint32_t cost = 0;
    int nseed = 0;
    for (int c = c0; c < c1; ++c) {
      const int s0 = b.chain_seed_off[c], s1 = b.chain_seed_off[c + 1];
      nseed += s1 - s0;
      if (s1 == s0 || cost) continue;
      int best = s0;
      for (int k = s0 + 1; k < s1; ++k)
        if (b.seeds[k].score >= b.seeds[best].score) best = k;
      const bwagpu_seed_t t = b.seeds[best];
      const int left = t.qbeg, right = lq - t.qbeg - t.len;
      cost = (uint32_t)((left ? (left + 16) * (1 + left / 64) : 0) + (right ? (right + 16) * (1 + right / 64) : 0) + 8);
    }
    cost += (uint32_t)(c1 - c0) * 8 + (uint32_t)nseed;
    if (v < 0) {
      atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_LEN);
      v = kNumVariants - 1;
    }
    const int bin = v * kCostBins + (kCostBins - 1 - (int)min(cost >> 2, (uint32_t)(kCostBins - 1)));
    bins[rd] = bin;
    atomicAdd(&h[bin], 1);
  }
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kNumVariants; ++k) {
    const unsigned long long m = __ballot(v == k);
    if (m != 0 && lane == __ffsll((long long)m) - 1) atomicAdd(&counts[k], __popcll(m));
  }
  __syncthreads();
  for (int k = threadIdx.x; k < kBins; k += blockDim.x)
    if (h[k]) atomicAdd(&hist[k], h[k]);
}

// exclusive scan of the kBins bin counts, in place (one block)
__global__ void __launch_bounds__(256) bin_scan_kernel(int32_t* hist) {
  __shared__ int part[256];
  constexpr int per = (kBins + 255) / 256;
  const int t = threadIdx.x;
  int v[per], sum = 0;
#pragma unroll
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    v[k] = i < kBins ? hist[i] : 0;
    sum += v[k];
  }
  part[t] = sum;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int x = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  int run = part[t] - sum;
#pragma unroll
  for (int k = 0; k < per; ++k) {
    const int i = t * per + k;
    if (i < kBins) hist[i] = run;
    run += v[k];
  }
}

__global__ void __launch_bounds__(256) read_scatter_kernel(DevBatch b, const int32_t* __restrict__ bins,
                                                           int32_t* offs, ReadDesc* desc, int32_t* list) {
  // ranks within the block from an LDS histogram, one global reservation per
  // (block, bin): hot bins see a few hundred global atomics, not one per read
  __shared__ int lh[kBins];
  __shared__ int lbase[kBins];
  for (int k = threadIdx.x; k < kBins; k += blockDim.x) lh[k] = 0;
  __syncthreads();
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  const int bin = rd < b.n_reads ? bins[rd] : 0;
  const int rank = rd < b.n_reads ? atomicAdd(&lh[bin], 1) : 0;
  __syncthreads();
  for (int k = threadIdx.x; k < kBins; k += blockDim.x)
    if (lh[k]) lbase[k] = atomicAdd(&offs[k], lh[k]);
  __syncthreads();
  if (rd >= b.n_reads) return;
  const int p = lbase[bin] + rank;
  ReadDesc d;
  d.qoff = b.seq_off[rd];
  d.rd = rd;
  d.lq = (int)(b.seq_off[rd + 1] - d.qoff);
  d.c0 = b.read_chain_off[rd];
  d.nch = b.read_chain_off[rd + 1] - d.c0;
  d.s0 = b.chain_seed_off[d.c0];
  d.ns = b.chain_seed_off[d.c0 + d.nch] - d.s0;
  desc[p] = d;
  list[p] = rd;
}

hipError_t launch_read_order(const DevBatch& b, int32_t* bins, int32_t* hist, int32_t* counts, ReadDesc* desc,
                             int32_t* list, int64_t* stats, hipStream_t st) {
  if (b.n_reads == 0) return hipSuccess;
  const int nb = (b.n_reads + 255) / 256;
  hipLaunchKernelGGL(read_bins_kernel, dim3(nb), dim3(256), 0, st, b, bins, hist, counts, stats);
  hipLaunchKernelGGL(bin_scan_kernel, dim3(1), dim3(256), 0, st, hist);
  hipLaunchKernelGGL(read_scatter_kernel, dim3(nb), dim3(256), 0, st, b, bins, hist, desc, list);
  return hipGetLastError();
}

// ------------------------------------------------------------ diagnostics


hipError_t set_trace(void* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &p, sizeof(p)); }

// ------------------------------------------------------------ chain2aln
template <int G, int C>
__global__ void __launch_bounds__(kBlock) chain2aln_kernel(DevOpt o, DevRef ref, DevBatch b,
                                                           const int32_t* __restrict__ read_list,
                                                           const int32_t* __restrict__ counts, int variant, int tb_bytes,
                                                           const ChainWin* __restrict__ win,
                                                           uint64_t* srt, bwagpu_alnreg_t* out,
                                                           int32_t* out_n, int64_t* stats) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  using GR = Grp<G>;
  const int gib = guni<G>(threadIdx.x / G);
  const int r = GR::lane();
  int base = 0;
  for (int v = 0; v < variant; ++v) base += counts[v];
  const int n_list = counts[variant];
  Tally tl{0, 0, 0};
  uint8_t* tb = lds + gib * tb_bytes;
  // Dynamic work queue, one head per XCD (counts[16 + 8*variant + shard]):
  // shard x holds list positions x, x+8, x+16, ... (costliest first).  A wave
  // starts on its own XCD's shard, so each head sees ~1/8 of the dequeues
  // (MI355X_MICROARCH.md, "dequeue"), and moves on to the other shards when
  // it runs dry — placement is never assumed, every position is taken exactly
  // once by whichever waves exist.  A relaxed load skips exhausted heads.
  const int xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20) & 7;  // HW_REG_XCC_ID
  int32_t* heads = const_cast<int32_t*>(counts) + 16 + 8 * variant;
  int shard = xcc, tried = 0;
  const int leader = (gib * G) & 63;

  for (;;) {
    int li = -1;
    while (tried < 8) {
      int32_t* h = heads + shard;
      if ((__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) / G) * 8 + shard < n_list) {
        // every lane of the group adds 1: the compiler folds this into ONE
        // wave-level atomic of the active-lane count (Guideline 12), so a
        // group's increment is exactly G and its lane 0 sees the old value
        const int slot = atomicAdd(h, 1);
        li = (guni<G>(__shfl(slot, leader, 64)) / G) * 8 + shard;
        if (li < n_list) break;
      }
      li = -1;
      shard = (shard + 1) & 7;
      ++tried;
    }
    if (li < 0) break;
    const int rd = guni<G>(read_list[base + li]);
    uint32_t* const trace = g_trace;
    const uint64_t t_start = trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const long long tr_cells = tl.cells, tr_rows = tl.rows;
    const int64_t qoff = guni64<G>(b.seq_off[rd]);
    const int lq = guni<G>((int)(b.seq_off[rd + 1] - qoff));
    const uint8_t* q = b.seq + qoff;
    const int c0 = guni<G>(b.read_chain_off[rd]), c1 = guni<G>(b.read_chain_off[rd + 1]);
    bwagpu_alnreg_t* av = out + b.chain_seed_off[c0];
    int nreg = 0;
    for (int c = c0; c < c1; ++c) {
      const int s0 = guni<G>(b.chain_seed_off[c]), ns = guni<G>(b.chain_seed_off[c + 1]) - s0;
      if (ns == 0) continue;
      ChainWin cw = win[c];
      cw.lo = guni64<G>(cw.lo);
      cw.hi = guni64<G>(cw.hi);
      if (cw.hi < cw.lo) continue;  // flagged by prep (reference would assert)
      const int rid = guni<G>(b.chain_rid[c]);
      const float frac_rep = b.chain_frac_rep[c];
      uint64_t* key = srt + s0;
      const bwagpu_seed_t* sd = b.seeds + s0;
      for (int k = ns - 1; k >= 0; --k) {
        mem_fence_group();
        const uint64_t kk = __hip_atomic_load(&key[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        bwagpu_seed_t s = sd[guni<G>((int)(uint32_t)kk)];
        s.rbeg = guni64<G>(s.rbeg);
        s.qbeg = guni<G>(s.qbeg);
        s.len = guni<G>(s.len);
        // containment test against the read's regions so far (bwamem.c:678-697).
        // Lanes test regions in parallel; loop bounds are uniform and bodies
        // branch-free so the read's control flow stays scalar.
        int hit = INT_MAX;
        for (int base = 0; base < nreg; base += G) {
          const int i = base + r;
          const bwagpu_alnreg_t* pr = &av[min(i, nreg - 1)];
          const int64_t prb = __hip_atomic_load(&pr->rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int64_t pre = __hip_atomic_load(&pr->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int pqb = __hip_atomic_load(&pr->qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int pqe = __hip_atomic_load(&pr->qe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int pw = __hip_atomic_load(&pr->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const int psl = __hip_atomic_load(&pr->seedlen0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          const bool inside = !(s.rbeg < prb || s.rbeg + s.len > pre || s.qbeg < pqb || s.qbeg + s.len > pqe) &&
                              !(s.len - psl > .1 * lq);
          // ahead of the seed ...
          const int qd1 = s.qbeg - pqb;
          const int64_t rd1 = s.rbeg - prb;
          const int g1 = max_gap_len(o, qd1 < rd1 ? qd1 : (int)rd1);
          const int bw1 = g1 < pw ? g1 : pw;
          // ... and behind it
          const int qd2 = pqe - (s.qbeg + s.len);
          const int64_t rd2 = pre - (s.rbeg + s.len);
          const int g2 = max_gap_len(o, qd2 < rd2 ? qd2 : (int)rd2);
          const int bw2 = g2 < pw ? g2 : pw;
          const bool near = (qd1 - rd1 < bw1 && rd1 - qd1 < bw1) || (qd2 - rd2 < bw2 && rd2 - qd2 < bw2);
          hit = guni<G>(GR::gmin(i < nreg && inside && near ? i : INT_MAX));
          if (hit != INT_MAX) break;
        }
        if (hit != INT_MAX) {
          // overlapping-seed check among seeds already visited (bwamem.c:698-707)
          int ov = INT_MAX;
          for (int base = k + 1; base < ns; base += G) {
            const int i = base + r;
            const uint64_t ki = __hip_atomic_load(&key[min(i, ns - 1)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const bwagpu_seed_t t = sd[(uint32_t)ki];
            const bool a = s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                           (int64_t)(t.qbeg - s.qbeg) != t.rbeg - s.rbeg;
            const bool b2 = t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                            (int64_t)(s.qbeg - t.qbeg) != s.rbeg - t.rbeg;
            const bool p = i < ns && ki != 0 && !(t.len < s.len * .95) && (a || b2);
            ov = guni<G>(GR::gmin(p ? i : INT_MAX));
            if (ov != INT_MAX) break;
          }
          if (ov == INT_MAX) {  // skip; mark like srt[k] = 0 (bwamem.c:709)
            // every lane stores the same word: no lane-divergent branch in the read's control flow
            __hip_atomic_store(&key[k], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            mem_fence_group();
            continue;
          }
        }

        // ---- extend this seed (bwamem.c:717-792): side 0 = left, 1 = right.
        // One call site for ksw_extend2 so the DP body is instantiated once.
        int score = -1, truesc = -1, qb = 0, qe = lq, sc0 = 0;
        int aw[2] = {o.w, o.w};
        int64_t rb = s.rbeg, re = s.rbeg + s.len;
#pragma nounroll
        for (int side = 0; side < 2; ++side) {
          const bool left = side == 0;
          if (left && s.qbeg == 0) {  // bwamem.c:753
            score = truesc = s.len * o.a;
            continue;
          }
          if (!left && s.qbeg + s.len == lq) continue;  // bwamem.c:781
          const int qlen = left ? s.qbeg : lq - (s.qbeg + s.len);
          const int64_t x0 = left ? s.rbeg - 1 : s.rbeg + s.len;
          const int dir = left ? -1 : 1;
          const int tlen = left ? (int)(s.rbeg - cw.lo) : (int)(cw.hi - x0);
          const int qa = left ? s.qbeg - 1 : s.qbeg + s.len;
          const int eb = left ? o.pen_clip5 : o.pen_clip3;
          const int h0 = left ? s.len * o.a : score;
          sc0 = score;
          ExtOut x{};
          for (int t = 0; t < 2; ++t) {  // MAX_BAND_TRY (bwamem.c:639)
            const int prev = score;
            aw[side] = o.w << t;
            const int nr = rows_needed(o, qlen, tlen, aw[side], eb);
            fill_target<G>(tb, ref, x0, dir, nr);
            x = extend_wave_dispatch<C, false>(o, qlen, q, qa, dir, tlen, tb, aw[side], eb, o.zdrop, h0, tl);
            score = x.score;
            if (score == prev || x.max_off < (aw[side] >> 1) + (aw[side] >> 2)) break;
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
        const int aw0 = aw[0], aw1 = aw[1];
        // seedcov (bwamem.c:784-788)
        long long cov = 0;
        for (int base = 0; base < ns; base += G) {
          const int i = base + r;
          const bwagpu_seed_t t = sd[min(i, ns - 1)];
          const bool in = i < ns && t.qbeg >= qb && t.qbeg + t.len <= qe && t.rbeg >= rb && t.rbeg + t.len <= re;
          cov += in ? t.len : 0;
        }
        cov = grp_sum64(cov, G);
        {  // the 88-byte mem_alnreg_t as 22 dwords, lane d writes dword d (lanes >= 21 repeat the last)
          const int d = r % G < 21 ? r % G : 21;
          uint32_t v = 0;
          v = d == 0 ? (uint32_t)rb : v;
          v = d == 1 ? (uint32_t)((uint64_t)rb >> 32) : v;
          v = d == 2 ? (uint32_t)re : v;
          v = d == 3 ? (uint32_t)((uint64_t)re >> 32) : v;
          v = d == 4 ? (uint32_t)qb : v;
          v = d == 5 ? (uint32_t)qe : v;
          v = d == 6 ? (uint32_t)rid : v;
          v = d == 7 ? (uint32_t)score : v;
          v = d == 8 ? (uint32_t)truesc : v;
          v = d == 13 ? (uint32_t)(aw0 > aw1 ? aw0 : aw1) : v;
          v = d == 14 ? (uint32_t)cov : v;
          v = d == 17 ? (uint32_t)s.len : v;
          v = d == 19 ? __float_as_uint(frac_rep) : v;
          reinterpret_cast<uint32_t*>(&av[nreg])[d] = v;
        }
        ++nreg;
        mem_fence_group();
      }
    }
    out_n[rd] = nreg;  // same value from every lane
    if (trace) {
      const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
      const int d = r % G < 7 ? r % G : 7;
      uint32_t v = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
      v = d == 0 ? (uint32_t)t_start : v;
      v = d == 1 ? (uint32_t)(t_start >> 32) : v;
      v = d == 2 ? (uint32_t)t_end : v;
      v = d == 3 ? (uint32_t)(t_end >> 32) : v;
      v = d == 4 ? (uint32_t)(tl.rows - tr_rows) : v;
      v = d == 5 ? (uint32_t)(tl.cells - tr_cells) : v;
      v = d == 6 ? __builtin_amdgcn_s_getreg((31 << 11) | 4) : v;  // HW_REG_HW_ID
      trace[(size_t)rd * 8 + d] = v;
    }
  }
  if (r != 0) tl = Tally{0, 0, 0};
  block_stats<G>(tl, stats);
}

// ------------------------------------------------------------ chain2aln, fast
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

__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)((uint64_t)hi << 32 | lo);
}

// mem_chain2aln for reads of <= 256 bp with <= 32 seeds and chains: one read
// per wave, the read's data in a per-wave LDS table, not in registers:
//   table    the read's seeds in processing order (prog, written by
//            chain_prep_kernel: chains in order, seeds by descending key), its
//            chains' seed ranges / windows / rid / frac_rep, and its bases (the
//            query of both extensions) — filled by global_load_lds DMA;
//   regions  the read's mem_alnreg_t records so far (88 B each);
//   tbl/tbr  the target rows of the current seed's left / right extension.
// Containment (bwamem.c:678-697), the overlap test (698-707) and seedcov
// (784-788) are lane-parallel tests (lane i: region i or seed i) + a ballot or
// a reduction.
// Scheduling is static: reads are cost-sorted (read_bins_kernel) and dealt to
// the resident waves in zig-zag rounds, so a wave knows its next read and DMAs
// that read's table (double-buffered) while the current read's DP runs; the
// DMA goes out after the current read's first target fill, so no fill waits
// on it.  No queue atomics and no dependent load chain on the critical path.
constexpr int kTabLanes = kFastMaxSeeds;  // seeds / chains per read (<= 64)
struct LaneTab {                          // byte offsets inside one table, [field][lane]
  static constexpr int RBL = 0;                      // prog: rbeg low / high dword, qbeg, len, pad_
  static constexpr int RBH = RBL + 4 * kTabLanes;
  static constexpr int QB = RBH + 4 * kTabLanes;
  static constexpr int LEN = QB + 4 * kTabLanes;
  static constexpr int FLAG = LEN + 4 * kTabLanes;
  static constexpr int CS0 = FLAG + 4 * kTabLanes;   // chain_seed_off[c]
  static constexpr int CS1 = CS0 + 4 * kTabLanes;    // chain_seed_off[c + 1]
  static constexpr int WIN = CS1 + 4 * kTabLanes;    // ChainWin (16 B / lane)
  static constexpr int RID = WIN + 16 * kTabLanes;
  static constexpr int FRAC = RID + 4 * kTabLanes;
  static constexpr int SEQ = FRAC + 4 * kTabLanes;   // the read's bases from dword (qoff & ~3): 128 dwords
  static constexpr int BYTES = SEQ + 2 * kSeqLds;
};
static_assert(LaneTab::WIN % 16 == 0 && LaneTab::BYTES % 16 == 0, "table alignment");

#define BWAGPU_GLDS(gptr, lptr, SIZE)                                                                   \
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(gptr),            \
                                   (void __attribute__((address_space(3)))*)(lptr), SIZE, 0, 0)

// DMA read d's table (d uniform, d.ns > 0) into tab
__device__ __forceinline__ void fetch_table(uint8_t* tab, const DevBatch& b, const C2AArgs& a, const ReadDesc& d,
                                            int r) {
  if (r < kTabLanes) {
    const uint32_t* pg = reinterpret_cast<const uint32_t*>(a.prog + d.s0 + min(r, d.ns - 1));
    BWAGPU_GLDS(pg + 0, tab + LaneTab::RBL, 4);
    BWAGPU_GLDS(pg + 1, tab + LaneTab::RBH, 4);
    BWAGPU_GLDS(pg + 2, tab + LaneTab::QB, 4);
    BWAGPU_GLDS(pg + 3, tab + LaneTab::LEN, 4);
    BWAGPU_GLDS(pg + 5, tab + LaneTab::FLAG, 4);
    const int cc = d.c0 + min(r, d.nch - 1);
    BWAGPU_GLDS(b.chain_seed_off + cc, tab + LaneTab::CS0, 4);
    BWAGPU_GLDS(b.chain_seed_off + cc + 1, tab + LaneTab::CS1, 4);
    BWAGPU_GLDS(a.win + cc, tab + LaneTab::WIN, 16);
    BWAGPU_GLDS(b.chain_rid + cc, tab + LaneTab::RID, 4);
    BWAGPU_GLDS(b.chain_frac_rep + cc, tab + LaneTab::FRAC, 4);
  }
  // bases by aligned dwords (a 1-byte LDS DMA writes a whole dword per lane):
  // the read starts at byte (qoff & 3) of the SEQ area; the last dword read is
  // the one holding the read's last base
  const uint32_t* q = reinterpret_cast<const uint32_t*>(b.seq) + (d.qoff >> 2);
  const int last = (int)(((d.qoff & 3) + d.lq - 1) >> 2);
  BWAGPU_GLDS(q + min(r, last), tab + LaneTab::SEQ, 4);
  BWAGPU_GLDS(q + min(64 + r, last), tab + LaneTab::SEQ + 256, 4);
}

__device__ __forceinline__ void wait_dma() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ int lds_i32(const uint8_t* p) { return *reinterpret_cast<const int*>(p); }
__device__ __forceinline__ int64_t lds_i64(const uint8_t* p) {
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(p), hi = *reinterpret_cast<const uint32_t*>(p + 4);
  return (int64_t)((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ int64_t tab_rb(const uint8_t* tab, int i) {
  const uint32_t lo = *reinterpret_cast<const uint32_t*>(tab + LaneTab::RBL + 4 * i);
  const uint32_t hi = *reinterpret_cast<const uint32_t*>(tab + LaneTab::RBH + 4 * i);
  return (int64_t)((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)((uint64_t)hi << 32 | lo);
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

constexpr int kRegBytes = 88 * kFastMaxSeeds;  // LDS region records per wave
constexpr int kFastWaveLds(int tb) { return 2 * LaneTab::BYTES + kRegBytes + 2 * tb; }

template <int C>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) chain2aln_fast_kernel(DevOpt o, DevRef ref, DevBatch b, C2AArgs a,
                                                                int variant, int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int r = (int)(threadIdx.x & 63);
  const int wib = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint8_t* const wl = lds + wib * kFastWaveLds(tb_bytes);
  uint8_t* const tabs = wl;  // two tables
  uint32_t* const regs = reinterpret_cast<uint32_t*>(wl + 2 * LaneTab::BYTES);  // region k: dwords [22k, 22k+22)
  uint8_t* const tbl = wl + 2 * LaneTab::BYTES + kRegBytes;
  uint8_t* const tbr = tbl + tb_bytes;
  int base = 0;
  for (int v = 0; v < variant; ++v) base += a.counts[v];
  const int n_list = a.counts[variant];
  Tally tl{0, 0, 0};
  // static zig-zag deal over the resident waves (cost-sorted list: LPT-like)
  const int NW = (int)gridDim.x * (kBlock / 64), W = (int)blockIdx.x * (kBlock / 64) + wib;
  auto pos = [&](int round) { return round * NW + ((round & 1) ? NW - 1 - W : W); };
  int round = 0;
  if (pos(0) < n_list) {
    ReadDesc d = uniform_desc(a.desc[base + pos(0)]);
    if (d.ns > 0) fetch_table(tabs, b, a, d, r);
    for (;;) {
      uint8_t* const tab = tabs + (round & 1) * LaneTab::BYTES;
      uint8_t* const ntab = tabs + ((round + 1) & 1) * LaneTab::BYTES;
      const bool has_next = pos(round + 1) < n_list;
      ReadDesc dn{};
      if (has_next) dn = uniform_desc(a.desc[base + pos(round + 1)]);
      bool fetched = !has_next || dn.ns == 0;
      const int rd = d.rd, lq = d.lq, nch = d.nch, ns = d.ns, s0 = d.s0;
      int nreg = 0;
      if (ns > 0) {
        wait_dma();  // this read's table has landed
        const uint8_t* const sq = tab + LaneTab::SEQ + (d.qoff & 3);
        uint64_t skipped = 0;  // srt[k] = 0 marks (bwamem.c:709), by program position
        for (int c = 0; c < nch; ++c) {
          const int cs0 = uni(lds_i32(tab + LaneTab::CS0 + 4 * c)) - s0;
          const int cs1 = uni(lds_i32(tab + LaneTab::CS1 + 4 * c)) - s0;
          if (cs1 == cs0) continue;
          const int64_t clo = uni64(lds_i64(tab + LaneTab::WIN + 16 * c));
          const int64_t chi = uni64(lds_i64(tab + LaneTab::WIN + 16 * c + 8));
          if (chi < clo) continue;  // flagged by prep (the reference would assert)
          const int rid = uni(lds_i32(tab + LaneTab::RID + 4 * c));
          const float frac = __int_as_float(uni(lds_i32(tab + LaneTab::FRAC + 4 * c)));
          for (int e = cs0; e < cs1; ++e) {
            const int64_t srb = uni64(tab_rb(tab, e));
            const int sqb = uni(lds_i32(tab + LaneTab::QB + 4 * e));
            const int slen = uni(lds_i32(tab + LaneTab::LEN + 4 * e));
            if (nreg > 0) {
              // containment in an existing region (bwamem.c:678-697), one region per lane
              const uint32_t* g = regs + 22 * min(r, nreg - 1);
              const int64_t R_rb = (int64_t)((uint64_t)g[1] << 32 | g[0]);
              const int64_t R_re = (int64_t)((uint64_t)g[3] << 32 | g[2]);
              const int R_qb = (int)g[4], R_qe = (int)g[5], R_w = (int)g[13], R_sl = (int)g[17];
              const bool inside = !(srb < R_rb || srb + slen > R_re || sqb < R_qb || sqb + slen > R_qe) &&
                                  !(slen - R_sl > .1 * lq);
              const int qd1 = sqb - R_qb;
              const int64_t rd1 = srb - R_rb;
              const int g1 = max_gap_len(o, qd1 < rd1 ? qd1 : (int)rd1);
              const int bw1 = g1 < R_w ? g1 : R_w;
              const int qd2 = R_qe - (sqb + slen);
              const int64_t rd2 = R_re - (srb + slen);
              const int g2 = max_gap_len(o, qd2 < rd2 ? qd2 : (int)rd2);
              const int bw2 = g2 < R_w ? g2 : R_w;
              const bool near = (qd1 - rd1 < bw1 && rd1 - qd1 < bw1) || (qd2 - rd2 < bw2 && rd2 - qd2 < bw2);
              if (__builtin_amdgcn_ballot_w64(r < nreg && inside && near) != 0) {
                // an overlapping seed among those already visited (bwamem.c:698-707), seed per lane
                const int rr = min(r, kTabLanes - 1);
                const int64_t p_rb = tab_rb(tab, rr);
                const int p_qb = lds_i32(tab + LaneTab::QB + 4 * rr);
                const int p_len = lds_i32(tab + LaneTab::LEN + 4 * rr);
                const int p_flag = lds_i32(tab + LaneTab::FLAG + 4 * rr);
                const bool a1 = sqb <= p_qb && sqb + slen - p_qb >= slen >> 2 && (int64_t)(p_qb - sqb) != p_rb - srb;
                const bool b1 = p_qb <= sqb && p_qb + p_len - sqb >= slen >> 2 && (int64_t)(sqb - p_qb) != srb - p_rb;
                const bool live = r >= cs0 && r < e && !((skipped >> r) & 1ull) && p_flag == 0;
                if (__builtin_amdgcn_ballot_w64(live && !(p_len < slen * .95) && (a1 || b1)) == 0) {
                  skipped |= 1ull << e;
                  continue;
                }
              }
            }
            // ---- extend (bwamem.c:717-792); both target windows in one round trip
            const int qlenL = sqb, qlenR = lq - (sqb + slen);
            const int64_t x0L = srb - 1, x0R = srb + slen;
            const int tlenL = (int)(srb - clo), tlenR = (int)(chi - x0R);
            fill_two(tbl, x0L, qlenL ? rows_needed(o, qlenL, tlenL, o.w << 1, o.pen_clip5) : 0, tbr, x0R,
                     qlenR ? rows_needed(o, qlenR, tlenR, o.w << 1, o.pen_clip3) : 0, ref);
            if (!fetched) {  // the next read's table, in flight during this seed's DP
              fetch_table(ntab, b, a, dn, r);
              fetched = true;
            }
            int score = -1, truesc = -1, qb = 0, qe = lq, sc0 = 0;
            int aw0 = o.w, aw1 = o.w;  // the band of each side (scalars: an indexed pair would live in scratch)
            int64_t rb = srb, re = srb + slen;
#pragma nounroll
            for (int side = 0; side < 2; ++side) {
              const bool left = side == 0;
              if (left && sqb == 0) {  // bwamem.c:753
                score = truesc = slen * o.a;
                continue;
              }
              if (!left && qlenR == 0) continue;  // bwamem.c:781
              const int qlen = left ? qlenL : qlenR;
              const int64_t x0 = left ? x0L : x0R;
              const int tlen = left ? tlenL : tlenR;
              const int qa = left ? sqb - 1 : sqb + slen;
              const int eb = left ? o.pen_clip5 : o.pen_clip3;
              const int h0 = left ? slen * o.a : score;
              uint8_t* const tb = left ? tbl : tbr;
              sc0 = score;
              ExtOut x{};
              for (int t = 0; t < 2; ++t) {  // MAX_BAND_TRY (bwamem.c:639)
                const int prev = score;
                const int aw = o.w << t;
                aw0 = left ? aw : aw0;
                aw1 = left ? aw1 : aw;
                x = extend_wave_dispatch<C, false>(o, qlen, sq, qa, left ? -1 : 1, tlen, tb, aw, eb, o.zdrop, h0,
                                                   tl);
                score = x.score;
                if (score == prev || x.max_off < (aw >> 1) + (aw >> 2)) break;
              }
              const bool local = x.gscore <= 0 || x.gscore <= score - eb;
              if (left) {
                qb = local ? sqb - x.qle : 0;
                rb = srb - (local ? x.tle : x.gtle);
                truesc = local ? score : x.gscore;
              } else {
                qe = local ? qa + x.qle : lq;
                re = x0 + (local ? x.tle : x.gtle);
                truesc += (local ? score : x.gscore) - sc0;
              }
            }
            // seedcov over the chain's seeds (bwamem.c:784-788), seed per lane
            long long cov;
            {
              const int rr = min(r, kTabLanes - 1);
              const int64_t p_rb = tab_rb(tab, rr);
              const int p_qb = lds_i32(tab + LaneTab::QB + 4 * rr);
              const int p_len = lds_i32(tab + LaneTab::LEN + 4 * rr);
              const bool in =
                  r >= cs0 && r < cs1 && p_qb >= qb && p_qb + p_len <= qe && p_rb >= rb && p_rb + p_len <= re;
              cov = grp_sum64(in ? p_len : 0, 64);
            }
            // region nreg as its 88-byte record (rest zero: bwamem.c:718), lane d writes dword d
            {
              const int dw = r < 21 ? r : 21;
              uint32_t v = 0;
              v = dw == 0 ? (uint32_t)rb : v;
              v = dw == 1 ? (uint32_t)((uint64_t)rb >> 32) : v;
              v = dw == 2 ? (uint32_t)re : v;
              v = dw == 3 ? (uint32_t)((uint64_t)re >> 32) : v;
              v = dw == 4 ? (uint32_t)qb : v;
              v = dw == 5 ? (uint32_t)qe : v;
              v = dw == 6 ? (uint32_t)rid : v;
              v = dw == 7 ? (uint32_t)score : v;
              v = dw == 8 ? (uint32_t)truesc : v;
              v = dw == 13 ? (uint32_t)(aw0 > aw1 ? aw0 : aw1) : v;
              v = dw == 14 ? (uint32_t)cov : v;
              v = dw == 17 ? (uint32_t)slen : v;
              v = dw == 19 ? __float_as_uint(frac) : v;
              regs[22 * nreg + dw] = v;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            ++nreg;
          }
        }
        // ---- the read's mem_alnreg_v: LDS records -> global, dword-parallel
        uint32_t* const dst = reinterpret_cast<uint32_t*>(a.out + s0);
        for (int k = r; k < 22 * nreg; k += 64) dst[k] = regs[k];
      }
      a.out_n[rd] = nreg;  // same value from every lane
      if (!has_next) break;
      if (!fetched) fetch_table(ntab, b, a, dn, r);
      d = dn;
      ++round;
    }
  }
  if (r != 0) tl = Tally{0, 0, 0};
  block_stats<64>(tl, a.stats);
}

// ------------------------------------------------------------ extend batch
template <int G, int C, bool T5>
__global__ void __launch_bounds__(kBlock) extend_kernel(DevOpt o, const bwagpu_ext_task_t* __restrict__ tasks,
                                                        const int32_t* __restrict__ task_list, int32_t n_list,
                                                        const uint8_t* __restrict__ qpool,
                                                        const uint8_t* __restrict__ tpool, int tb_bytes,
                                                        bwagpu_ext_result_t* res, int64_t* stats) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  using GR = Grp<G>;
  constexpr int GPB = kBlock / G;
  const int gib = threadIdx.x / G;
  const int r = GR::lane();
  const int li = blockIdx.x * GPB + gib;
  Tally tl{0, 0, 0};
  uint8_t* tb = lds + gib * tb_bytes;
  if (li < n_list) {
    const int k = task_list[li];
    const bwagpu_ext_task_t t = tasks[k];
    const uint8_t* q = qpool + t.qoff;
    const uint8_t* tp = tpool + t.toff;
    ExtOut x;
    if (t.h0 <= 0) {
      x = ExtOut{-1, 0, 0, 0, -1, 0};  // reference asserts h0 > 0 (ksw.c:385)
    } else {
      const int nr = rows_needed(o, t.qlen, t.tlen, t.w, t.end_bonus);
      for (int base = 0; base < nr; base += G) {
        const int i = min(base + r, nr - 1);
        tb[i] = tp[i];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      x = extend_wave_dispatch<C, T5>(o, t.qlen, q, 0, 1, t.tlen, tb, t.w, t.end_bonus, t.zdrop, t.h0, tl);
    }
    if (r == 0) res[k] = bwagpu_ext_result_t{x.score, x.qle, x.tle, x.gtle, x.gscore, x.max_off};
    if (r != 0) tl = Tally{0, 0, 0};
  }
  block_stats<G>(tl, stats);
}

// ------------------------------------------------------------ launchers
hipError_t launch_chain_prep(const DevOpt& o, const DevRef& ref, const DevBatch& b, ChainWin* win, uint64_t* srt,
                             bwagpu_seed_t* prog, int64_t* stats, hipStream_t st) {
  if (b.n_chains == 0) return hipSuccess;
  const int nb = (b.n_chains + 255) / 256;
  hipLaunchKernelGGL(chain_prep_kernel, dim3(nb), dim3(256), 0, st, o, ref, b, win, srt, prog, stats);
  return hipGetLastError();
}

// resident workgroups of a kernel over the whole device (persistent grids).
// The answer depends on the kernel, its dynamic LDS bytes (which change per
// batch with the read lengths and options) and the device, so it is cached
// under exactly that key; GPU worker threads of several contexts call this
// concurrently.
template <typename K>
static int resident_blocks(K kernel, size_t lds) {
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
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, kBlock, lds) != hipSuccess || per < 1) per = 1;
  std::lock_guard<std::mutex> g(mu);
  return cache[key] = per * ncu;
}

size_t fast_wave_lds(int tb) { return (size_t)kFastWaveLds(tb); }

template <int C>
static hipError_t launch_c2a_fast(const DevOpt& o, const DevRef& ref, const DevBatch& b, int variant, int32_t n,
                                  int tb, const C2AArgs& a, hipStream_t st) {
  const size_t lds = (size_t)(kBlock / 64) * kFastWaveLds(tb);
  const int cap = resident_blocks(chain2aln_fast_kernel<C>, lds);
  const int nb = std::min((n + 3) / 4, cap);
  hipLaunchKernelGGL((chain2aln_fast_kernel<C>), dim3(nb), dim3(kBlock), lds, st, o, ref, b, a, variant, tb);
  return hipGetLastError();
}

template <int G, int C>
static hipError_t launch_c2a_t(const DevOpt& o, const DevRef& ref, const DevBatch& b, int variant, int32_t n, int tb,
                               const C2AArgs& a, hipStream_t st) {
  constexpr int GPB = kBlock / G;
  // persistent-style grid: the waves pull reads from the device-side queue
  const int nb = std::min((n + GPB - 1) / GPB, 2048);
  hipLaunchKernelGGL((chain2aln_kernel<G, C>), dim3(nb), dim3(kBlock), (size_t)GPB * tb, st, o, ref, b, a.read_list,
                     a.counts, variant, tb, a.win, a.srt, a.out, a.out_n, a.stats);
  return hipGetLastError();
}

hipError_t launch_chain2aln(int variant, const DevOpt& o, const DevRef& ref, const DevBatch& b, int32_t max_list,
                            int tb_bytes, const C2AArgs& a, hipStream_t st) {
  if (max_list == 0) return hipSuccess;
  switch (variant) {
    case 0: return launch_c2a_fast<3>(o, ref, b, 0, max_list, tb_bytes, a, st);
    case 1: return launch_c2a_fast<4>(o, ref, b, 1, max_list, tb_bytes, a, st);
    case 2: return launch_c2a_t<64, 16>(o, ref, b, 2, max_list, tb_bytes, a, st);
  }
  return hipErrorInvalidValue;
}

template <int G, int C, bool T5>
static hipError_t launch_ext_t(const DevOpt& o, const bwagpu_ext_task_t* tasks, const int32_t* list, int32_t n,
                               const uint8_t* qp, const uint8_t* tp, int tb, bwagpu_ext_result_t* res,
                               int64_t* stats, hipStream_t st) {
  constexpr int GPB = kBlock / G;
  const int nb = (n + GPB - 1) / GPB;
  hipLaunchKernelGGL((extend_kernel<G, C, T5>), dim3(nb), dim3(kBlock), (size_t)GPB * tb, st, o, tasks, list, n,
                     qp, tp, tb, res, stats);
  return hipGetLastError();
}

hipError_t launch_extend(int variant, bool t5, const DevOpt& o, int32_t, const bwagpu_ext_task_t* tasks,
                         const int32_t* task_list, int32_t n_list, const uint8_t* qpool, const uint8_t* tpool,
                         int tb_bytes, bwagpu_ext_result_t* res, int64_t* stats, hipStream_t st) {
  if (n_list == 0) return hipSuccess;
#define EXT_CASE(v, G, C)                                                                              \
  case v:                                                                                              \
    return t5 ? launch_ext_t<G, C, true>(o, tasks, task_list, n_list, qpool, tpool, tb_bytes, res, stats, st) \
              : launch_ext_t<G, C, false>(o, tasks, task_list, n_list, qpool, tpool, tb_bytes, res, stats, st);
  switch (variant) {
    EXT_CASE(0, 64, 3)
    EXT_CASE(1, 64, 4)
    EXT_CASE(2, 64, 16)
  }
#undef EXT_CASE
  return hipErrorInvalidValue;
}

// bare task list, four per wave (extend_quad): sub-slot s of the grid takes
// tasks s, s + NS, ... of the list; all four sub-slots of a wave run their
// current calls together, and one whose call ended takes its next task at the
// call boundary.  Every task has h0 > 0, no N in its target rows and
// qlen + 1 <= 32 * PMAX (the host routes the rest to extend_kernel).
template <int PMAX>
__global__ void __launch_bounds__(kBlock) extend4_kernel(DevOpt o, const bwagpu_ext_task_t* __restrict__ tasks,
                                                         const int32_t* __restrict__ task_list, int32_t n_list,
                                                         const uint8_t* __restrict__ qpool,
                                                         const uint8_t* __restrict__ tpool, int tb_bytes,
                                                         bwagpu_ext_result_t* res, int64_t* stats) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int r = (int)(threadIdx.x & 31);
  const int half = (int)(blockIdx.x * (kBlock / 32) + (threadIdx.x >> 5));  // global half index
  const int NS = (int)gridDim.x * (kBlock / 32) * 2;                         // sub-slots in the grid
  uint8_t* const tba = lds + (size_t)(threadIdx.x >> 5) * 2 * tb_bytes;
  uint8_t* const tbb = tba + tb_bytes;
  int la = 2 * half, lb = 2 * half + 1;  // list positions of the sub-slots' tasks
  int ka = -1, kb = -1;                 // their task indices, -1: none
  long long cells = 0, rows = 0, calls = 0;
  QCall ca = quad_idle(qpool, tba), cb = quad_idle(qpool, tbb);
  auto take = [&](int& li, int& k, QCall& c, uint8_t* tb) {
    k = -1;
    c = quad_idle(qpool, tb);
    if (li >= n_list) return;
    k = task_list[li];
    li += NS;
    const bwagpu_ext_task_t t = tasks[k];
    const int nr = rows_needed(o, t.qlen, t.tlen, t.w, t.end_bonus);
    for (int base = 0; base < nr; base += 32) tb[min(base + r, nr - 1)] = tpool[t.toff + min(base + r, nr - 1)];
    c.qlen = t.qlen;
    c.qa = 0;
    c.qd = 1;
    c.tlen = t.tlen;
    c.w = t.w;
    c.eb = t.end_bonus;
    c.zdrop = t.zdrop;
    c.h0 = t.h0;
    c.q = qpool + t.qoff;
    c.tb = tb;
  };
  take(la, ka, ca, tba);
  take(lb, kb, cb, tbb);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  while (__builtin_amdgcn_ballot_w64(ka >= 0 || kb >= 0)) {
    ExtOut xa, xb;
    Tally32 ta{0, 0, 0}, tb{0, 0, 0};
    extend_quad_dispatch<PMAX>(o, ca, cb, xa, xb, ta, tb);
    if (ka >= 0) {
      if (r == 0) res[ka] = bwagpu_ext_result_t{xa.score, xa.qle, xa.tle, xa.gtle, xa.gscore, xa.max_off};
      cells += ta.cells;
      rows += ta.rows;
      calls += ta.calls;
    }
    if (kb >= 0) {
      if (r == 0) res[kb] = bwagpu_ext_result_t{xb.score, xb.qle, xb.tle, xb.gtle, xb.gscore, xb.max_off};
      cells += tb.cells;
      rows += tb.rows;
      calls += tb.calls;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (ka >= 0) take(la, ka, ca, tba);
    if (kb >= 0) take(lb, kb, cb, tbb);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  Tally tl{r == 0 ? cells : 0, r == 0 ? rows : 0, r == 0 ? calls : 0};
  block_stats<64>(tl, stats);
}

hipError_t launch_extend4(const DevOpt& o, const bwagpu_ext_task_t* tasks, const int32_t* task_list, int32_t n_list,
                          const uint8_t* qpool, const uint8_t* tpool, int tb_bytes, bwagpu_ext_result_t* res,
                          int64_t* stats, hipStream_t st) {
  if (n_list == 0) return hipSuccess;
  const size_t lds = (size_t)(kBlock / 32) * 2 * tb_bytes;
  const int nb = std::min((n_list + 15) / 16, std::max(1, resident_blocks(extend4_kernel<8>, lds) / 2));
  hipLaunchKernelGGL(extend4_kernel<8>, dim3(nb), dim3(kBlock), lds, st, o, tasks, task_list, n_list, qpool, tpool,
                     tb_bytes, res, stats);
  return hipGetLastError();
}

// ============================================================ speculative chain2aln
// mem_chain2aln (bwamem.c:641-795) restructured for load balance on
// reference-seeded batches, where a few reads (tandem repeats: hundreds of
// seeds, one region each) carry more DP than thousands of ordinary reads and,
// run serially by one wave, set the stage's critical path.
//
// The one sequential dependency of mem_chain2aln is the decision whether a
// seed is extended at all: the containment test against the read's regions so
// far (bwamem.c:678-697) and the overlapping-seed test (698-707).  The
// extension itself (717-792: left ksw_extend2 with the band retry, right
// ksw_extend2 from the left score, local vs to-end choice) depends only on the
// seed, the read and its chain's window.  So:
//   round A   extend the first seed (processing order) of every chain — it is
//             almost always extended; one wave per task, dynamic queue;
//   emulate   replay the sequential logic per read with the round-A regions:
//             every seed that would be extended and has no result yet becomes
//             a round-B task (its region unknown, so later seeds of the read
//             are tested against fewer regions: a superset is predicted);
//   round B   extend those;
//   final     replay the sequential logic exactly, with every result it needs
//             precomputed except rare mispredictions, which it computes inline.
// Output = the reference's regions, byte for byte; the stats count only the DP
// of extensions mem_chain2aln performs (spec work is a separate diagnostic).

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
      if (__hip_atomic_load(h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cap) {
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

// lane per chain: window (bwamem.c:648-668 + bns_fetch_seq's clipping), the
// round-A task (the chain's first seed in processing order) and, for chains
// of up to kOrderLane seeds, the processing order; longer chains are listed
// for spec_order_kernel, which does their window and order one workgroup
// each (a lane looping over ~170 seeds was this kernel's tail).  chain_read
// comes from spec_reads_kernel.
__global__ void __launch_bounds__(256) spec_chain_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  bool task = false, longc = false;
  int bin = 0, s0 = 0;
  if (c < b.n_chains) {
    const int rd = a.chain_read[c];
    s0 = b.chain_seed_off[c];
    const int ns = b.chain_seed_off[c + 1] - s0;
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    if (ns <= 0) {
      a.win[c] = ChainWin{0, 0};
    } else {
      int64_t wlo = ref.l_pac << 1, whi = 0;
      longc = ns > kOrderLane;
      if (!longc) {
        // the processing order (descending key score<<32|i, bwamem.c:671-676),
        // ranked in registers
        uint64_t key[kOrderLane];
#pragma unroll
        for (int t = 0; t < kOrderLane; ++t) {
          key[t] = ~0ull;
          if (t < ns) {
            const bwagpu_seed_t v = b.seeds[s0 + t];
            key[t] = (uint64_t)(uint32_t)v.score << 32 | (uint32_t)t;
            seed_reach(o, v, lq, wlo, whi);
          }
        }
#pragma unroll
        for (int t = 0; t < kOrderLane; ++t) {
          if (t < ns) {
            int rank = 0;
#pragma unroll
            for (int u = 0; u < kOrderLane; ++u) rank += key[u] < key[t];
            bwagpu_seed_t v = b.seeds[s0 + t];
            v.pad_ = key[t] == 0 ? 1 : 0;
            a.prog[s0 + ns - 1 - rank] = v;
            a.seedchain[s0 + ns - 1 - rank] = c;
          }
        }
      }
      const bool ok = finish_window(ref, b.chain_rid[c], b.seeds[s0].rbeg, wlo, whi);
      if (!ok) {
        atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_RID);
        a.win[c] = ChainWin{0, -1};
      } else {
        if (!longc) a.win[c] = ChainWin{wlo, whi};
        task = lq <= BWAGPU_MAX_READ_LEN;
        bin = spec_bin(lq);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < kSpecBins; ++k) {
    const int p = wave_append(&a.ctr[SPC_CNT + k], task && bin == k);
    if (p >= 0) a.tasks[(size_t)k * b.n_chains + p] = make_int2(s0, c);
  }
  const int p = wave_append(&a.ctr[SPC_LONG_N], longc);
  if (p >= 0) a.longc[p] = c;
}

// rows are triangular: row k holds words w < ceil(k / 64) (only seeds j < k
// count); tri_off(k) = sum over i < k of ceil(i / 64)
__host__ __device__ inline int64_t tri_off(int k) {
  if (k <= 1) return 0;
  const int64_t q = (k - 1) >> 6;
  return 32 * q * (q + 1) + (int64_t)(k - 1 - 64 * q) * (q + 1);
}

// lane per read: length check, and the list of heavy reads (selected first)
__global__ void __launch_bounds__(256) spec_reads_kernel(DevBatch b, SpecArgs a) {
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  bool heavy = false;
  int ns = 0;
  if (rd < b.n_reads) {
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    if (lq > BWAGPU_MAX_READ_LEN) atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_LEN);
    ReadDesc d;
    d.qoff = b.seq_off[rd];
    d.rd = rd;
    d.lq = lq;
    d.c0 = b.read_chain_off[rd];
    d.nch = b.read_chain_off[rd + 1] - d.c0;
    d.s0 = b.chain_seed_off[d.c0];
    d.ns = b.chain_seed_off[d.c0 + d.nch] - d.s0;
    a.rdesc[rd] = d;
    for (int c = d.c0; c < d.c0 + d.nch; ++c) a.chain_read[c] = rd;
    heavy = d.ns > kSelLight || d.nch > kSelLight;
    ns = d.ns;
  }
  const int p = wave_append(&a.ctr[SPC_HEAVY_N], heavy);
  if (p >= 0) {
    a.heavy[p] = rd;
    // the read's pair matrices (kSelMatMaxSeeds seeds at most, and room left)
    const long long words = 2 * tri_off(ns);
    int woff = -1, col = 0;
    if (ns <= kSelMatMaxSeeds) {
      const long long o = (long long)atomicAdd(reinterpret_cast<unsigned long long*>(&a.ctr[SPC_MATW64]),
                                               (unsigned long long)words);
      if (o + words <= a.mat_words) {
        woff = (int)o;
        col = atomicAdd(&a.ctr[SPC_HCOLS], ns);
        for (int i = 0; i < ns; ++i) a.colent[col + i] = p;
      }
    }
    a.hinfo[p] = make_int4(rd, woff, col, ns);
  }
}

// The processing order (descending key score<<32|i, bwamem.c:671-676) of
// the chains spec_chain_kernel listed (more than kOrderLane seeds), by
// ranking: keys are unique, so rank = the number of smaller keys.  One
// workgroup per chain with the keys staged in LDS (a lane looping over global
// keys made the longest chain, ~170 seeds, a 250 us tail).  pad_ = 1 flags
// the key that is 0 from the start (skipped by the overlap test like a
// marked seed, bwamem.c:700).
constexpr int kOrderBlocks = 1024;
constexpr int kOrderLds = 4096;  // longer chains rank against global memory
__device__ __forceinline__ uint64_t order_key(const bwagpu_seed_t* sd, int i) {
  return (uint64_t)(uint32_t)sd[i].score << 32 | (uint32_t)i;
}
__global__ void __launch_bounds__(256) spec_order_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a) {
  __shared__ uint64_t keys[kOrderLds];
  __shared__ int64_t wred[2][4];
  const int tid = (int)threadIdx.x;
  const int n_long = __hip_atomic_load(&a.ctr[SPC_LONG_N], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (int gi = (int)blockIdx.x; gi < n_long; gi += (int)gridDim.x) {
    const int g = a.longc[gi];
    const int s0 = b.chain_seed_off[g], ns = b.chain_seed_off[g + 1] - s0;
    const bwagpu_seed_t* sd = b.seeds + s0;
    const bool in_lds = ns <= kOrderLds;
    const int rd = a.chain_read[g];
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    int64_t wlo = ref.l_pac << 1, whi = 0;
    for (int i = tid; i < ns; i += 256) {
      const bwagpu_seed_t v = sd[i];
      if (in_lds) keys[i] = (uint64_t)(uint32_t)v.score << 32 | (uint32_t)i;
      seed_reach(o, v, lq, wlo, whi);
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
      wlo = min(wlo, (int64_t)__shfl_xor((long long)wlo, m, 64));
      whi = max(whi, (int64_t)__shfl_xor((long long)whi, m, 64));
    }
    if ((tid & 63) == 0) {
      wred[0][tid >> 6] = wlo;
      wred[1][tid >> 6] = whi;
    }
    __syncthreads();
    if (tid == 0) {
      wlo = min(min(wred[0][0], wred[0][1]), min(wred[0][2], wred[0][3]));
      whi = max(max(wred[1][0], wred[1][1]), max(wred[1][2], wred[1][3]));
      if (finish_window(ref, b.chain_rid[g], sd[0].rbeg, wlo, whi)) a.win[g] = ChainWin{wlo, whi};
    }
    for (int i = tid; i < ns; i += 256) {
      bwagpu_seed_t v = sd[i];
      const uint64_t ki = (uint64_t)(uint32_t)v.score << 32 | (uint32_t)i;
      int rank = 0;
      if (in_lds)
        for (int j = 0; j < ns; ++j) rank += keys[j] < ki;
      else
        for (int j = 0; j < ns; ++j) rank += order_key(sd, j) < ki;
      v.pad_ = ki == 0 ? 1 : 0;
      a.prog[s0 + ns - 1 - rank] = v;
      a.seedchain[s0 + ns - 1 - rank] = g;
    }
    __syncthreads();
  }
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

// Extension tasks of one list (round * kSpecBins + bin): one wave per task,
// claimed one at a time from the sharded queue (a wave holding a second task
// while others idle at the end of the list cost more: DESIGN.md §5).
template <int C>
__global__ void __launch_bounds__(kBlock) spec_ext_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                          int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int wib = uni((int)(threadIdx.x >> 6));
  uint8_t* const tbl = lds + wib * 2 * tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  const int n = uni(__hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int2* tl = a.tasks + spec_list_off(list, b.n_chains, b.n_seeds);
  ShardQ qq;
  qq.init(a.qh + 8 * kQHStride * list, n);
  long long spec_cells = 0;
  int m0, cap;
  while (qq.claim(1, m0, cap)) {
    for (int m = m0; m < m0 + 1 && m < cap; ++m) {
      const int2 tk = tl[qq.shard + 8 * m];
      const int pos = uni(tk.x), c = uni(tk.y);
      const int rd = uni(a.chain_read[c]);
      const int64_t qoff = uni64(b.seq_off[rd]);
      const int lq = uni((int)(b.seq_off[rd + 1] - qoff));
      const bwagpu_seed_t s = uni_seed(a.prog[pos]);
      ChainWin cw = a.win[c];
      cw.lo = uni64(cw.lo);
      cw.hi = uni64(cw.hi);
      const SeedExt e = extend_seed<C>(o, ref, s, lq, b.seq + qoff, cw, tbl, tbr);
      store_ext(a.ext + pos, e);
      spec_cells += e.cells;
    }
  }
  if ((threadIdx.x & 63) == 0 && spec_cells)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
}

// ---------------------------------------------------- two seeds per wave
// The same extension tasks with one seed per 32-lane half (extend_pair).
// Everything below is per lane and uniform over a half; the halves diverge
// only through EXEC (a half without a left side, a retry or a task waits for
// the other).
//
// Both target windows of the half's seed into its LDS rows (fill_two on 32
// lanes: 4 loads per side per lane in flight, 128 rows per side per pass).
__device__ __forceinline__ void fill_two_half(uint8_t* tbl, int64_t x0l, int nl, uint8_t* tbr, int64_t x0r, int nr,
                                              const DevRef& ref) {
  const int r = (int)(threadIdx.x & 31);
  const int64_t two1 = (ref.l_pac << 1) - 1;
  const int n = max(nl, nr);
  for (int base = 0; base < n; base += 128) {
    uint32_t raw[8];
    int sh[8], kk[8];
    bool rev[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const bool left = m < 4;
      const int nn = left ? nl : nr;
      const int k = min(base + (m & 3) * 32 + r, max(nn - 1, 0));
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

// One half's task and the state of its extension, in LDS for the whole task:
// re-read (volatile, LDS address space) around every call, so that none of it
// occupies VGPRs across the DP loop.
struct PairCtx {
  int64_t rbeg, lo, hi, qoff;  // the seed, its chain's window, its read
  int32_t qbeg, len, lq, phase;
  int64_t rb, re;              // the region so far
  int32_t score, truesc, qb, qe, sc0, aw0, aw1, cells, rows, calls, pad_[2];
};
static_assert(sizeof(PairCtx) == 112, "PairCtx layout");
typedef volatile __attribute__((address_space(3))) PairCtx LdsCtx;

// extend_seed (bwamem.c:717-792) for the half's seed, as a state machine with
// ONE extend_pair call site: phase 0/1 = left side try 0/1 (MAX_BAND_TRY,
// bwamem.c:639), 2/3 = right side, 4 = done; a half whose phases are over
// leaves the loop (EXEC) while the other finishes.
template <int PMAX>
__device__ __forceinline__ SeedExt extend_seed2(const DevOpt& o, const DevRef& ref, LdsCtx* cx, const uint8_t* seq,
                                                uint8_t* tbl, uint8_t* tbr) {
  {
    const int64_t rbeg = cx->rbeg, lo = cx->lo, hi = cx->hi;
    const int qbeg = cx->qbeg, len = cx->len, lq = cx->lq;
    const int qlenL = qbeg, qlenR = lq - (qbeg + len);
    const int64_t x0R = rbeg + len;
    fill_two_half(tbl, rbeg - 1, qlenL ? rows_needed(o, qlenL, (int)(rbeg - lo), o.w << 1, o.pen_clip5) : 0, tbr, x0R,
                  qlenR ? rows_needed(o, qlenR, (int)(hi - x0R), o.w << 1, o.pen_clip3) : 0, ref);
    cx->phase = qbeg != 0 ? 0 : (qlenR != 0 ? 2 : 4);
    const int sc = qbeg != 0 ? -1 : len * o.a;  // bwamem.c:753
    cx->score = sc;
    cx->truesc = sc;
    cx->qb = 0;
    cx->qe = lq;
    cx->sc0 = 0;
    cx->aw0 = o.w;
    cx->aw1 = o.w;
    cx->rb = rbeg;
    cx->re = rbeg + len;
    cx->cells = 0;
    cx->rows = 0;
    cx->calls = 0;
  }
  for (;;) {
    const int phase = cx->phase;
    if (phase >= 4) break;
    const int64_t rbeg = cx->rbeg;
    const int qbeg = cx->qbeg, len = cx->len, lq = cx->lq;
    const bool left = phase < 2;
    const int t = phase & 1;
    const int qlenR = lq - (qbeg + len);
    const int qlen = left ? qbeg : qlenR;
    const int64_t x0 = left ? rbeg - 1 : rbeg + len;
    const int tlen = left ? (int)(rbeg - cx->lo) : (int)(cx->hi - x0);
    const int qa = left ? qbeg - 1 : qbeg + len;
    const int eb = left ? o.pen_clip5 : o.pen_clip3;
    if (t == 0) cx->sc0 = cx->score;
    const int h0 = left ? len * o.a : cx->sc0;
    const int aw = o.w << t;
    if (left) cx->aw0 = aw;
    else cx->aw1 = aw;
    Tally32 tl{0, 0, 0};
    const ExtOut x = extend_pair_dispatch<PMAX>(o, qlen, seq + cx->qoff, qa, left ? -1 : 1, tlen, left ? tbl : tbr, aw,
                                             eb, o.zdrop, h0, tl);
    cx->cells = cx->cells + tl.cells;
    cx->rows = cx->rows + tl.rows;
    cx->calls = cx->calls + tl.calls;
    const int prev = cx->score;
    const int score = x.score;
    cx->score = score;
    if (t == 0 && !(score == prev || x.max_off < (aw >> 1) + (aw >> 2))) {
      cx->phase = phase + 1;  // the band retry
      continue;
    }
    const bool local = x.gscore <= 0 || x.gscore <= score - eb;
    if (left) {
      cx->qb = local ? qbeg - x.qle : 0;
      cx->rb = rbeg - (local ? x.tle : x.gtle);
      cx->truesc = local ? score : x.gscore;
      cx->phase = qlenR != 0 ? 2 : 4;
    } else {
      cx->qe = local ? qa + x.qle : lq;
      cx->re = x0 + (local ? x.tle : x.gtle);
      cx->truesc = cx->truesc + (local ? score : x.gscore) - cx->sc0;
      cx->phase = 4;
    }
  }
  SeedExt e;
  e.rb = cx->rb;
  e.re = cx->re;
  e.qb = cx->qb;
  e.qe = cx->qe;
  e.score = cx->score;
  e.truesc = cx->truesc;
  const int aw0 = cx->aw0, aw1 = cx->aw1;
  e.w = aw0 > aw1 ? aw0 : aw1;
  e.cells = cx->cells;
  e.rows = cx->rows;
  e.calls = cx->calls + 1;  // + 1: a computed slot is never all-zero
  return e;
}

__device__ __forceinline__ void store_ext_half(SeedExt* dst, const SeedExt& e) {
  const int d = (int)(threadIdx.x & 31);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(&e);
  uint32_t v = 0;
#pragma unroll
  for (int k = 0; k < 12; ++k) v = d == k ? w[k] : v;
  if (d < 12) reinterpret_cast<uint32_t*>(dst)[d] = v;
}

// Extension tasks of one list, two per wave: a wave claims two consecutive
// entries of a shard (one atomic), lanes 0-31 take the first, 32-63 the second.
// PMAX = the bin's largest CPL: ceil(read length / 32) (qlen + 1 <= read length)
template <int PMAX>
__global__ void __launch_bounds__(kBlock) spec_ext2_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                           int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int hf = (int)(threadIdx.x >> 5) & 1;
  // per half: left rows, right rows, the task context
  uint8_t* const tbl = lds + (size_t)(threadIdx.x >> 5) * (2 * tb_bytes + sizeof(PairCtx));
  uint8_t* const tbr = tbl + tb_bytes;
  LdsCtx* const cx = (LdsCtx*)(tbr + tb_bytes);
  const int n = uni(__hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int2* tl = a.stasks + spec_list_off(list, b.n_chains, b.n_seeds);  // in pair order (spec_sort_*)
  ShardQ qq;
  qq.init(a.qh + 8 * kQHStride * list, n);
  long long spec_cells = 0;
  int m0, cap;
  while (qq.claim(2, m0, cap)) {
    const int m = m0 + hf;
    if (m < cap) {
      const int2 tk = tl[qq.shard + 8 * m];
      const int pos = tk.x, c = tk.y;
      if ((threadIdx.x & 31) == 0) {
        const int rd = a.chain_read[c];
        const bwagpu_seed_t s = a.prog[pos];
        const ChainWin cw = a.win[c];
        const int64_t qoff = b.seq_off[rd];
        cx->rbeg = s.rbeg;
        cx->lo = cw.lo;
        cx->hi = cw.hi;
        cx->qoff = qoff;
        cx->qbeg = s.qbeg;
        cx->len = s.len;
        cx->lq = (int)(b.seq_off[rd + 1] - qoff);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      const SeedExt e = extend_seed2<PMAX>(o, ref, cx, b.seq, tbl, tbr);
      store_ext_half(a.ext + pos, e);
      spec_cells += e.cells;
    }
  }
  if ((threadIdx.x & 31) == 0 && spec_cells)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
}

// LDS bytes of a spec_ext2_kernel workgroup
static size_t ext2_lds(int tb_bytes) { return (size_t)(kBlock / 32) * (2 * (size_t)tb_bytes + sizeof(PairCtx)); }

// ---------------------------------------------------- four seeds per wave
// The same extension tasks with two seeds per 32-lane half, packed in the
// 16-bit halves of the DP registers (extend_quad).  Each sub-slot (half x
// low/high) walks its own seed through extend_seed's state machine
// (bwamem.c:717-792: left side with the band retry, right side from the left
// score, local vs to-end), held in registers; the four sub-slots call
// extend_quad together, and a sub-slot whose seed is done takes the next task
// of the list at once (one claim per call boundary for all the sub-slots that
// need one), so a wave idles only inside a call whose four rows counts differ.
struct QTask {
  int64_t rbeg, wlo, whi, qoff, rb, re;
  int pos, qbeg, len, lq, phase, score, truesc, qb, qe, sc0, aw0, aw1, cells, rows, calls;
};

// the task's seed, window and read; both target windows into the sub-slot's LDS rows
__device__ __forceinline__ void qtask_start(QTask& t, const DevOpt& o, const DevRef& ref, const DevBatch& b,
                                            const SpecArgs& a, int2 tk, uint8_t* tl, uint8_t* tr) {
  const int rd = a.chain_read[tk.y];
  const bwagpu_seed_t s = a.prog[tk.x];
  const ChainWin cw = a.win[tk.y];
  t.pos = tk.x;
  t.rbeg = s.rbeg;
  t.wlo = cw.lo;
  t.whi = cw.hi;
  t.qoff = b.seq_off[rd];
  t.lq = (int)(b.seq_off[rd + 1] - t.qoff);
  t.qbeg = s.qbeg;
  t.len = s.len;
  const int qlenL = t.qbeg, qlenR = t.lq - (t.qbeg + t.len);
  const int64_t x0R = t.rbeg + t.len;
  fill_two_half(tl, t.rbeg - 1, qlenL ? rows_needed(o, qlenL, (int)(t.rbeg - t.wlo), o.w << 1, o.pen_clip5) : 0, tr,
                x0R, qlenR ? rows_needed(o, qlenR, (int)(t.whi - x0R), o.w << 1, o.pen_clip3) : 0, ref);
  t.phase = qlenL != 0 ? 0 : (qlenR != 0 ? 2 : 4);
  const int sc = qlenL != 0 ? -1 : t.len * o.a;  // bwamem.c:753
  t.score = sc;
  t.truesc = sc;
  t.qb = 0;
  t.qe = t.lq;
  t.sc0 = 0;
  t.aw0 = o.w;
  t.aw1 = o.w;
  t.rb = t.rbeg;
  t.re = t.rbeg + t.len;
  t.cells = t.rows = t.calls = 0;
}

// the ksw_extend2 call of the task's phase (0/1: left try 0/1, 2/3: right)
__device__ __forceinline__ QCall qtask_call(QTask& t, const DevOpt& o, const uint8_t* seq, const uint8_t* tl,
                                            const uint8_t* tr) {
  const bool left = t.phase < 2;
  const int tt = t.phase & 1;
  const int qlenR = t.lq - (t.qbeg + t.len);
  const int64_t x0 = left ? t.rbeg - 1 : t.rbeg + t.len;
  QCall q;
  q.qlen = left ? t.qbeg : qlenR;
  q.tlen = left ? (int)(t.rbeg - t.wlo) : (int)(t.whi - x0);
  q.qa = left ? t.qbeg - 1 : t.qbeg + t.len;
  q.qd = left ? -1 : 1;
  q.eb = left ? o.pen_clip5 : o.pen_clip3;
  if (tt == 0) t.sc0 = t.score;
  q.h0 = left ? t.len * o.a : t.sc0;
  q.w = o.w << tt;
  if (left) t.aw0 = q.w;
  else t.aw1 = q.w;
  q.zdrop = o.zdrop;
  q.q = seq + t.qoff;
  q.tb = left ? tl : tr;
  return q;
}

// the call's result into the task (bwamem.c:737-792); true = the seed is done
__device__ __forceinline__ bool qtask_advance(QTask& t, const DevOpt& o, const ExtOut& x, const Tally32& tl) {
  const bool left = t.phase < 2;
  const int tt = t.phase & 1;
  t.cells += tl.cells;
  t.rows += tl.rows;
  t.calls += tl.calls;
  const int prev = t.score;
  t.score = x.score;
  const int aw = o.w << tt;
  if (tt == 0 && !(x.score == prev || x.max_off < (aw >> 1) + (aw >> 2))) {  // the band retry (MAX_BAND_TRY)
    t.phase += 1;
    return false;
  }
  const int eb = left ? o.pen_clip5 : o.pen_clip3;
  const bool local = x.gscore <= 0 || x.gscore <= x.score - eb;
  if (left) {
    t.qb = local ? t.qbeg - x.qle : 0;
    t.rb = t.rbeg - (local ? x.tle : x.gtle);
    t.truesc = local ? x.score : x.gscore;
    t.phase = t.lq - (t.qbeg + t.len) != 0 ? 2 : 4;
  } else {
    t.qe = local ? t.qbeg + t.len + x.qle : t.lq;
    t.re = t.rbeg + t.len + (local ? x.tle : x.gtle);
    t.truesc += (local ? x.score : x.gscore) - t.sc0;
    t.phase = 4;
  }
  return t.phase >= 4;
}

__device__ __forceinline__ SeedExt qtask_ext(const QTask& t) {
  SeedExt e;
  e.rb = t.rb;
  e.re = t.re;
  e.qb = t.qb;
  e.qe = t.qe;
  e.score = t.score;
  e.truesc = t.truesc;
  e.w = t.aw0 > t.aw1 ? t.aw0 : t.aw1;
  e.cells = t.cells;
  e.rows = t.rows;
  e.calls = t.calls + 1;  // + 1: a computed slot is never all-zero
  return e;
}

// The sub-slots' task states wait in LDS while a call runs (loaded before and
// stored after it): kept in registers across extend_quad they cost ~50 VGPRs,
// which at 2 waves per SIMD left the other caller stream's selection kernels
// no room on the SIMD.
static_assert(sizeof(QTask) <= 112, "QTask layout");
constexpr int kQTaskLds = 112;
typedef volatile __attribute__((address_space(3))) QTask LdsQ;
__device__ __forceinline__ void qpark(LdsQ* p, const QTask& t) {
  p->rbeg = t.rbeg;
  p->wlo = t.wlo;
  p->whi = t.whi;
  p->qoff = t.qoff;
  p->rb = t.rb;
  p->re = t.re;
  p->pos = t.pos;
  p->qbeg = t.qbeg;
  p->len = t.len;
  p->lq = t.lq;
  p->phase = t.phase;
  p->score = t.score;
  p->truesc = t.truesc;
  p->qb = t.qb;
  p->qe = t.qe;
  p->sc0 = t.sc0;
  p->aw0 = t.aw0;
  p->aw1 = t.aw1;
  p->cells = t.cells;
  p->rows = t.rows;
  p->calls = t.calls;
}
__device__ __forceinline__ QTask qload(LdsQ* p) {
  QTask t;
  t.rbeg = p->rbeg;
  t.wlo = p->wlo;
  t.whi = p->whi;
  t.qoff = p->qoff;
  t.rb = p->rb;
  t.re = p->re;
  t.pos = p->pos;
  t.qbeg = p->qbeg;
  t.len = p->len;
  t.lq = p->lq;
  t.phase = p->phase;
  t.score = p->score;
  t.truesc = p->truesc;
  t.qb = p->qb;
  t.qe = p->qe;
  t.sc0 = p->sc0;
  t.aw0 = p->aw0;
  t.aw1 = p->aw1;
  t.cells = p->cells;
  t.rows = p->rows;
  t.calls = p->calls;
  return t;
}

// Extension tasks of one list (in pair order, spec_sort_*), four per wave.
// PMAX = the bin's largest CPL: ceil(read length / 32).
template <int PMAX>
__global__ void __launch_bounds__(kBlock) spec_ext4_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                           int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int hf = (int)(threadIdx.x >> 5) & 1;
  // per half: A left, A right, B left, B right target rows, then A's and B's task states
  uint8_t* const tal = lds + (size_t)(threadIdx.x >> 5) * (4 * (size_t)tb_bytes + 2 * kQTaskLds);
  uint8_t* const tar = tal + tb_bytes;
  uint8_t* const tbl = tar + tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  LdsQ* const qa = (LdsQ*)(tbr + tb_bytes);
  LdsQ* const qb = (LdsQ*)(tbr + tb_bytes + kQTaskLds);
  const int n = uni(__hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int2* tl = a.stasks + spec_list_off(list, b.n_chains, b.n_seeds);
  ShardQ qq;
  qq.init(a.qh + 8 * kQHStride * list, n);
  bool ha = false, hb = false, more = n > 0;
  long long spec_cells = 0;
  for (;;) {
    if (more) {  // every sub-slot without a seed takes the next entry: one claim for the wave
      const uint64_t na = __builtin_amdgcn_ballot_w64(!ha), nb = __builtin_amdgcn_ballot_w64(!hb);
      const int n0 = (int)(na & 1) + (int)(nb & 1), n1 = (int)((na >> 32) & 1) + (int)((nb >> 32) & 1);
      if (n0 + n1 > 0) {
        int m0, cap;
        if (qq.claim(n0 + n1, m0, cap)) {
          const int ia = m0 + (hf ? n0 : 0), ib = ia + (ha ? 0 : 1);
          if (!ha && ia < cap) {
            QTask t;
            qtask_start(t, o, ref, b, a, tl[qq.shard + 8 * ia], tal, tar);
            if (t.phase >= 4) store_ext_half(a.ext + t.pos, qtask_ext(t));  // a whole-read seed (bwamem.c:753, 781)
            else qpark(qa, t);
            ha = t.phase < 4;
          }
          if (!hb && ib < cap) {
            QTask t;
            qtask_start(t, o, ref, b, a, tl[qq.shard + 8 * ib], tbl, tbr);
            if (t.phase >= 4) store_ext_half(a.ext + t.pos, qtask_ext(t));
            else qpark(qb, t);
            hb = t.phase < 4;
          }
        } else {
          more = false;
        }
      }
    }
    if (!__builtin_amdgcn_ballot_w64(ha || hb)) {
      if (!more) break;
      continue;
    }
    QCall ca = quad_idle(b.seq, tal), cb = quad_idle(b.seq, tbl);
    if (ha) {
      QTask t = qload(qa);
      ca = qtask_call(t, o, b.seq, tal, tar);
      qpark(qa, t);
    }
    if (hb) {
      QTask t = qload(qb);
      cb = qtask_call(t, o, b.seq, tbl, tbr);
      qpark(qb, t);
    }
    ExtOut xa, xb;
    Tally32 ta{0, 0, 0}, tb{0, 0, 0};
    extend_quad_dispatch<PMAX>(o, ca, cb, xa, xb, ta, tb);
    if (ha) {
      QTask t = qload(qa);
      if (qtask_advance(t, o, xa, ta)) {
        store_ext_half(a.ext + t.pos, qtask_ext(t));
        spec_cells += t.cells;
        ha = false;
      } else {
        qpark(qa, t);
      }
    }
    if (hb) {
      QTask t = qload(qb);
      if (qtask_advance(t, o, xb, tb)) {
        store_ext_half(a.ext + t.pos, qtask_ext(t));
        spec_cells += t.cells;
        hb = false;
      } else {
        qpark(qb, t);
      }
    }
  }
  if ((threadIdx.x & 31) == 0 && spec_cells)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
}

// LDS bytes of a spec_ext4_kernel workgroup
static size_t ext4_lds(int tb_bytes) { return (size_t)(kBlock / 32) * (4 * (size_t)tb_bytes + 2 * kQTaskLds); }


// Task order for the pair kernel: the two seeds a wave takes should need the
// same phases for about as long — a half whose seed has no left side, or a
// much shorter one, idles while the other runs (EXEC).  A counting sort of
// the C = 3 / 4 lists of a round by key = (left qlen / 8, right qlen / 8):
// count (per-block LDS histograms, one global atomic per block and key),
// scan (one block per list), scatter (per-block LDS ranks, one global atomic
// per block and key to reserve the block's range).  Claims then take entries
// 8 apart in the sorted list (the sharded queue), which have about the same
// key.  The order changes nothing but which seeds share a wave.
__device__ __forceinline__ int pair_key(const DevBatch& b, const SpecArgs& a, int2 tk) {
  const bwagpu_seed_t s = a.prog[tk.x];
  const int rd = a.chain_read[tk.y];
  const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
  const int ql = min(s.qbeg, 255), qr = min(max(lq - s.qbeg - s.len, 0), 255);
  return (ql >> 3) << 5 | (qr >> 3);
}

__global__ void __launch_bounds__(256) spec_sort_count(DevBatch b, SpecArgs a, int round) {
  __shared__ int hist[kSortKeys];
  const int list = round * kSpecBins + (int)blockIdx.y;
  int32_t* gh = a.sorth + (round * 2 + (int)blockIdx.y) * kSortKeys;
  for (int k = threadIdx.x; k < kSortKeys; k += 256) hist[k] = 0;
  __syncthreads();
  const int n = __hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int2* tl = a.tasks + spec_list_off(list, b.n_chains, b.n_seeds);
  const int chunk = (n + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (int i = i0 + (int)threadIdx.x; i < i1; i += 256) atomicAdd(&hist[pair_key(b, a, tl[i])], 1);
  __syncthreads();
  for (int k = threadIdx.x; k < kSortKeys; k += 256)
    if (hist[k]) atomicAdd(&gh[k], hist[k]);
}

__global__ void __launch_bounds__(256) spec_sort_scan(SpecArgs a, int round) {
  __shared__ int part[256];
  int32_t* gh = a.sorth + (round * 2 + (int)blockIdx.x) * kSortKeys;
  const int t = (int)threadIdx.x;  // 4 keys per thread
  int v[4], s = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = gh[4 * t + k];
    s += v[k];
  }
  part[t] = s;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {  // inclusive scan of the per-thread sums
    const int x = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  int base = part[t] - s;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    gh[4 * t + k] = base;  // the key's first position (a cursor from here on)
    base += v[k];
  }
}

__global__ void __launch_bounds__(256) spec_sort_scatter(DevBatch b, SpecArgs a, int round) {
  __shared__ int cnt[kSortKeys];
  const int list = round * kSpecBins + (int)blockIdx.y;
  int32_t* gh = a.sorth + (round * 2 + (int)blockIdx.y) * kSortKeys;
  for (int k = threadIdx.x; k < kSortKeys; k += 256) cnt[k] = 0;
  __syncthreads();
  const int n = __hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const size_t off = spec_list_off(list, b.n_chains, b.n_seeds);
  const int2* tl = a.tasks + off;
  int2* out = a.stasks + off;
  const int chunk = (n + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  constexpr int kPer = 16;  // entries per thread held across the barrier
  int keys[kPer], rank[kPer];
  int2 tk[kPer];
  for (int base = i0; base < i1; base += 256 * kPer) {
#pragma unroll
    for (int m = 0; m < kPer; ++m) {
      const int i = base + m * 256 + (int)threadIdx.x;
      keys[m] = -1;
      if (i < i1) {
        tk[m] = tl[i];
        keys[m] = pair_key(b, a, tk[m]);
        rank[m] = atomicAdd(&cnt[keys[m]], 1);
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < kSortKeys; k += 256) {
      const int c = cnt[k];
      cnt[k] = c ? atomicAdd(&gh[k], c) : 0;  // this pass's range of key k
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kPer; ++m)
      if (keys[m] >= 0) out[cnt[keys[m]] + rank[m]] = tk[m];
    __syncthreads();
    for (int k = threadIdx.x; k < kSortKeys; k += 256) cnt[k] = 0;
    __syncthreads();
  }
}

// The pair kernel's grid: its waves pull tasks from the queue, so the grid
// only sets its occupancy.  2 workgroups per CU (8 waves per CU, 2 per SIMD)
// instead of the resident capacity (5 per SIMD): the batch on the other caller
// stream (the bench's ping-pong) and this batch's selection kernels keep the
// rest, and an even count per CU beats an uneven one.  Same-box sweep
// (DESIGN.md §3): capacity 19.87, 60 % 20.74, 50 % 20.66, 2/CU (40 %) 21.74,
// 30 % 20.16, 1/CU 19.72 Mreads/s.  BWAGPU_EXT2_BLOCKS_PER_CU overrides.
static int ext2_grid(int nb) {
  static const int per_cu = [] {
    const char* e = getenv("BWAGPU_EXT2_BLOCKS_PER_CU");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : v;
  }();
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    return nb;
  return std::max(1, std::min(nb, per_cu * ncu));
}

// ============================================================ FPGA wire format
// bwagpu_sw_stream (include/bwagpu.h).  Lane per read record: the record's
// bases unpacked to bytes (4-bit words, first base in the high nibble,
// FPGAPipeline.cpp:262-276), then every chain's window and every task checked
// and written to tasks[task index], binned by read length like the spec
// lists.  Anything that does not parse sets a flag and is not queued.
__device__ __forceinline__ int64_t stream64(const int32_t* b, int64_t at) {
  return (int64_t)((uint64_t)(uint32_t)b[at] | (uint64_t)(uint32_t)b[at + 1] << 32);
}

__global__ void __launch_bounds__(256) stream_decode_kernel(StreamArgs a) {
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  if (rd >= a.n_reads) return;
  const int32_t* __restrict__ in = a.buf;
  const int64_t p = a.rstart[rd];
  const int64_t end = in[p];  // the host walk checked p + 2 < end <= words
  const int lq = in[p + 1];   // and 0 <= lq <= BWAGPU_MAX_READ_LEN
  const int nw = (lq + 7) >> 3;
  int err = 0;
  if (p + 3 + nw > end) err |= STR_ERR_RECORD;
  int64_t c = p + 2 + nw;
  if (!err) {
    uint8_t* q = a.qpool + 8 * p;
    for (int k = 0; k < nw; ++k) {
      const uint32_t w = (uint32_t)in[p + 2 + k];
      uint32_t lo4 = 0, hi4 = 0;
      int bad = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t v = w >> (28 - 4 * j) & 15;
        bad |= 8 * k + j < lq && v > 4;
        if (j < 4) lo4 |= v << (8 * j);
        else hi4 |= v << (8 * (j - 4));
      }
      if (bad) err |= STR_ERR_BASE;
      reinterpret_cast<uint2*>(q)[k] = make_uint2(lo4, hi4);  // qpool is 8-byte aligned per word
    }
    const int nch = in[c++];
    for (int ch = 0; ch < nch && !err; ++ch) {
      if (c + 5 > end) {
        err |= STR_ERR_RECORD;
        break;
      }
      const int64_t lo = stream64(in, c), hi = stream64(in, c + 2);
      const int ns = in[c + 4];
      c += 5;
      if (ns < 0 || c + 5 * (int64_t)ns > end) {
        err |= STR_ERR_RECORD;
        break;
      }
      if (ns && (lo < 0 || hi > 2 * a.l_pac || lo > hi || (lo < a.l_pac && a.l_pac < hi))) {
        err |= STR_ERR_SEED;
        break;
      }
      for (int k = 0; k < ns; ++k, c += 5) {
        const int t = in[c];
        StreamTask T;
        T.s.rbeg = stream64(in, c + 1);
        T.s.qbeg = in[c + 3];
        T.s.len = in[c + 4];
        T.s.score = 0;
        T.s.pad_ = 0;
        if (t < 0 || t >= a.cap) {
          err |= STR_ERR_TASK;
          break;
        }
        if (T.s.qbeg < 0 || T.s.len <= 0 || T.s.qbeg + T.s.len > lq || T.s.rbeg < lo || T.s.rbeg + T.s.len > hi) {
          err |= STR_ERR_SEED;
          break;
        }
        if (atomicAdd(&a.seen[t], 1) != 0) {
          err |= STR_ERR_DUP;
          break;
        }
        T.lo = lo;
        T.hi = hi;
        T.qoff = 8 * p;
        T.lq = lq;
        T.pad_ = 0;
        a.tasks[t] = T;
        const int bin = spec_bin(lq);
        a.lists[(size_t)bin * a.cap + atomicAdd(&a.ctr[bin], 1)] = t;
        atomicAdd(&a.ctr[kStrDecoded], 1);
        atomicMax(&a.ctr[kStrMax], t + 1);
      }
    }
    if (!err && c != end) err |= STR_ERR_RECORD;
  }
  if (err) atomicOr(&a.ctr[kStrErr], err);
}

// one wave per task from the bin's sharded queue; the record (5 words of two
// int16 each, little-endian like the FPGA's short[]): t, qb | dqe, drb | dre,
// score | truesc, w
template <int C>
__global__ void __launch_bounds__(kBlock) stream_ext_kernel(DevOpt o, DevRef ref, StreamArgs a, int bin,
                                                            int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int wib = uni((int)(threadIdx.x >> 6));
  uint8_t* const tbl = lds + wib * 2 * tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  const int n = uni(__hip_atomic_load(&a.ctr[bin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int32_t* L = a.lists + (size_t)bin * a.cap;
  ShardQ qq;
  qq.init(a.ctr + kStrHeads + 8 * kQHStride * bin, n);
  int m0, cap;
  while (qq.claim(1, m0, cap)) {
    for (int m = m0; m < m0 + 1 && m < cap; ++m) {
      const int t = uni(L[qq.shard + 8 * m]);
      const StreamTask& T = a.tasks[t];
      const bwagpu_seed_t s = uni_seed(T.s);
      const int lq = uni(T.lq);
      ChainWin cw;
      cw.lo = uni64(T.lo);
      cw.hi = uni64(T.hi);
      const SeedExt e = extend_seed<C>(o, ref, s, lq, a.qpool + uni64(T.qoff), cw, tbl, tbr);
      const int d = (int)(threadIdx.x & 63);
      const uint32_t dqe = (uint16_t)(e.qe - (s.qbeg + s.len)), drb = (uint16_t)(e.rb - s.rbeg),
                     dre = (uint16_t)(e.re - (s.rbeg + s.len));
      uint32_t v = (uint32_t)t;
      v = d == 1 ? (uint16_t)e.qb | dqe << 16 : v;
      v = d == 2 ? drb | dre << 16 : v;
      v = d == 3 ? (uint16_t)e.score | (uint32_t)(uint16_t)e.truesc << 16 : v;
      v = d == 4 ? (uint32_t)(uint16_t)e.w : v;
      if (d < 5) a.out[(size_t)5 * t + d] = (int32_t)v;
    }
  }
}

hipError_t launch_sw_stream(const DevOpt& o, const DevRef& ref, const StreamArgs& a, int tb_bytes, hipStream_t st) {
  if (a.n_reads == 0) return hipSuccess;
  hipLaunchKernelGGL(stream_decode_kernel, dim3((a.n_reads + 255) / 256), dim3(256), 0, st, a);
  const size_t lds = (size_t)(kBlock / 64) * 2 * tb_bytes;
  hipLaunchKernelGGL(stream_ext_kernel<3>, dim3(resident_blocks(stream_ext_kernel<3>, lds)), dim3(kBlock), lds, st,
                     o, ref, a, 0, tb_bytes);
  hipLaunchKernelGGL(stream_ext_kernel<4>, dim3(resident_blocks(stream_ext_kernel<4>, lds)), dim3(kBlock), lds, st,
                     o, ref, a, 1, tb_bytes);
  hipLaunchKernelGGL(stream_ext_kernel<16>, dim3(resident_blocks(stream_ext_kernel<16>, lds)), dim3(kBlock), lds,
                     st, o, ref, a, 2, tb_bytes);
  return hipGetLastError();
}

// The sequential logic of mem_chain2aln over one read's chains, by one wave.
// A seed that is extended but has no result yet:
//   SEL_EMULATE  becomes a round-B task (its region stays unknown in this pass);
//   SEL_FINAL    becomes a round-C task and the read goes to the redo list
//                (its later decisions depend on that region);
//   SEL_REDO     (the redo list only) is computed inline — the pass that
//                guarantees every read completes.
// SEL_FINAL and SEL_REDO write the read's mem_alnreg_v.
// Two shapes: LIGHT reads (<= kSelLight seeds, so every chain and the region
// list fit one lane slot) four waves per workgroup, 2 KB of LDS each; HEAVY
// reads one wave per workgroup with up to 64 KB of LDS region records (beyond
// that: the region's seed slot in regpos[] and its SeedExt, re-read with
// workgroup-scope atomics), chains of <= 256 seeds in four VGPR slots (longer:
// prog[] and skip flags in skipf[]).  The two shapes run concurrently on two
// streams.
enum { SEL_EMULATE = 0, SEL_FINAL = 1, SEL_REDO = 2 };
struct RegRec {  // a region's containment fields (bwamem.c:682-696)
  int64_t rb, re;
  int32_t qb, qe, w, seedlen0;
};
constexpr int kSelHeavyLds = 64 * 1024;
constexpr int kSelExtCache = 256;  // a heavy chain's SeedExt records staged in LDS
__host__ __device__ constexpr int sel_light_wave_lds() { return kSelLight * (int)sizeof(RegRec); }
__host__ __device__ constexpr int sel_heavy_cap(int mode, int tb) {
  return (kSelHeavyLds - 4 * (BWAGPU_MAX_READ_LEN + 1) - kSelExtCache * (int)(sizeof(SeedExt) + sizeof(bwagpu_seed_t)) -
          (mode == SEL_REDO ? 2 * tb : 0)) / (int)sizeof(RegRec);
}

// max_gap_len (cal_max_gap, bwamem.c:630-637) of every length a containment
// test can ask for (min(qd, rd) of a region holding the seed: 0..lq-1),
// tabulated in LDS per workgroup instead of two divisions per lane and region
constexpr int kMglN = BWAGPU_MAX_READ_LEN + 1;

// near(s, p): the two gap tests of bwamem.c:688-696 for a region p that holds s
__device__ __forceinline__ bool seed_near(const int32_t* MG, const bwagpu_seed_t& s, const RegRec& p) {
  const int qd1 = s.qbeg - p.qb;
  const int64_t rd1 = s.rbeg - p.rb;
  const int g1 = MG[min(max(qd1 < rd1 ? qd1 : (int)rd1, 0), kMglN - 1)];
  const int bw1 = g1 < p.w ? g1 : p.w;
  const int qd2 = p.qe - (s.qbeg + s.len);
  const int64_t rd2 = p.re - (s.rbeg + s.len);
  const int g2 = MG[min(max(qd2 < rd2 ? qd2 : (int)rd2, 0), kMglN - 1)];
  const int bw2 = g2 < p.w ? g2 : p.w;
  return (qd1 - rd1 < bw1 && rd1 - qd1 < bw1) || (qd2 - rd2 < bw2 && rd2 - qd2 < bw2);
}

// the 88-byte mem_alnreg_t (rest zero: bwamem.c:718); lane d writes dword d
__device__ __forceinline__ void write_region(bwagpu_alnreg_t* dst, const SeedExt& e, int rid, int cov, int slen,
                                             float frac) {
  const int r = (int)(threadIdx.x & 63);
  const int dw = r < 21 ? r : 21;
  uint32_t v = 0;
  v = dw == 0 ? (uint32_t)e.rb : v;
  v = dw == 1 ? (uint32_t)((uint64_t)e.rb >> 32) : v;
  v = dw == 2 ? (uint32_t)e.re : v;
  v = dw == 3 ? (uint32_t)((uint64_t)e.re >> 32) : v;
  v = dw == 4 ? (uint32_t)e.qb : v;
  v = dw == 5 ? (uint32_t)e.qe : v;
  v = dw == 6 ? (uint32_t)rid : v;
  v = dw == 7 ? (uint32_t)e.score : v;
  v = dw == 8 ? (uint32_t)e.truesc : v;
  v = dw == 13 ? (uint32_t)e.w : v;
  v = dw == 14 ? (uint32_t)cov : v;
  v = dw == 17 ? (uint32_t)slen : v;
  v = dw == 19 ? __float_as_uint(frac) : v;
  reinterpret_cast<uint32_t*>(dst)[dw] = v;
}

// a region's containment record into LDS (lanes 0-7 one field each)
__device__ __forceinline__ void put_regrec(RegRec* dst, const SeedExt& e, int slen) {
  const int r = (int)(threadIdx.x & 63);
  const int f = r < 8 ? r : 7;
  int32_t v = 0;
  v = f == 0 ? (int32_t)(uint32_t)e.rb : v;
  v = f == 1 ? (int32_t)((uint64_t)e.rb >> 32) : v;
  v = f == 2 ? (int32_t)(uint32_t)e.re : v;
  v = f == 3 ? (int32_t)((uint64_t)e.re >> 32) : v;
  v = f == 4 ? e.qb : v;
  v = f == 5 ? e.qe : v;
  v = f == 6 ? e.w : v;
  v = f == 7 ? slen : v;
  if (r < 8) reinterpret_cast<int32_t*>(dst)[f] = v;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// diagnostics (bwagpu_debug_set_trace): per read and selection pass, 8 words
// at g_trace[(pass * n_reads + rd) * 8]: start / end s_memrealtime (100 MHz),
// seeds, regions, XCC id, shape (1 light, 2 heavy)
__device__ __forceinline__ void trace_read(int pass, int n_reads, int rd, uint64_t t0, int ns, int nreg, int shape) {
  uint32_t* const tr = g_trace;
  if (!tr) return;
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  const int r = (int)(threadIdx.x & 63);
  const int d = r < 7 ? r : 7;
  uint32_t v = (uint32_t)shape;
  v = d == 0 ? (uint32_t)t0 : v;
  v = d == 1 ? (uint32_t)(t0 >> 32) : v;
  v = d == 2 ? (uint32_t)t1 : v;
  v = d == 3 ? (uint32_t)(t1 >> 32) : v;
  v = d == 4 ? (uint32_t)ns : v;
  v = d == 5 ? (uint32_t)nreg : v;
  v = d == 6 ? __builtin_amdgcn_s_getreg((31 << 11) | 20) : v;
  if (r < 8) tr[((size_t)pass * n_reads + rd) * 8 + d] = v;
}

template <int MODE, bool HEAVY>
__global__ void __launch_bounds__(64) spec_select_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int tb_bytes) {
  static_assert(HEAVY, "one-wave heavy shape only");
  constexpr bool WRITE = MODE != SEL_EMULATE;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int r = (int)(threadIdx.x & 63);
  // LDS: max_gap_len table | chain seeds (pad_ = skip flag | 2 * pending) |
  // their SeedExt records | region records | (redo) target rows
  int32_t* const MG = reinterpret_cast<int32_t*>(lds);
  bwagpu_seed_t* const SC = reinterpret_cast<bwagpu_seed_t*>(lds + 4 * kMglN);
  SeedExt* const EC = reinterpret_cast<SeedExt*>(SC + kSelExtCache);
  RegRec* const R = reinterpret_cast<RegRec*>(EC + kSelExtCache);
  const int cap_reg = sel_heavy_cap(MODE, tb_bytes);
  uint8_t* const tbl = reinterpret_cast<uint8_t*>(R + cap_reg);
  uint8_t* const tbr = tbl + tb_bytes;
  for (int x = r; x < kMglN; x += 64) MG[x] = max_gap_len(o, x);
  Tally tl{0, 0, 0};
  const int n_list = uni(__hip_atomic_load(&a.ctr[MODE == SEL_REDO ? SPC_REDO_N : SPC_HEAVY_N], __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
  const int32_t* const hlist = MODE == SEL_REDO ? a.redo : a.heavy;
  for (;;) {
    int t = 0;
    if (r == 0) t = atomicAdd(&a.ctr[SPC_SEL_CUR + MODE], 1);
    t = uni(__shfl(t, 0, 64));
    if (t >= n_list) break;
    if (MODE != SEL_REDO && uni(a.hinfo[t].y) >= 0) continue;  // the pair-matrix kernels' read
    const int rd = uni(hlist[t]);
    const uint64_t t_start = g_trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const ReadDesc d = uniform_desc(a.rdesc[rd]);
    if (d.lq > BWAGPU_MAX_READ_LEN) continue;  // flagged by spec_reads_kernel
    const uint8_t* const q = b.seq + d.qoff;
    const int rep_lim = (int)floor(.1 * d.lq) + 1;  // s->len - p->seedlen0 > .1 * l_query, bwamem.c:685
    bool redo = false;
    Tally rt{0, 0, 0};
    int nreg = 0;
    for (int c = d.c0; c < d.c0 + d.nch && !redo; ++c) {
      const int s0 = uni(b.chain_seed_off[c]), ns = uni(b.chain_seed_off[c + 1]) - s0;
      if (ns == 0) continue;
      ChainWin cw = a.win[c];
      cw.lo = uni64(cw.lo);
      cw.hi = uni64(cw.hi);
      if (cw.hi < cw.lo) continue;  // flagged by spec_chain_kernel (the reference would assert)
      const int rid = uni(b.chain_rid[c]);
      const float frac = __int_as_float(uni(__float_as_int(b.chain_frac_rep[c])));
      // the chain's seeds (processing order) and their extension results, staged
      // in LDS (chains of more than kSelExtCache seeds: prog[] / ext[] / skipf[])
      const bool big = ns > kSelExtCache;
      for (int i = r; i < min(ns, kSelExtCache); i += 64) {
        bwagpu_seed_t v = a.prog[s0 + i];
        v.pad_ = v.pad_ != 0 ? 1 : 0;
        SC[i] = v;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(a.ext + s0 + i);
        uint32_t* dst = reinterpret_cast<uint32_t*>(EC + i);
#pragma unroll
        for (int w = 0; w < 12; ++w) dst[w] = __hip_atomic_load(src + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (big)
        for (int i = r; i < ns; i += 64)
          __hip_atomic_store(&a.skipf[s0 + i], a.prog[s0 + i].pad_ != 0 ? 1 : 0, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      mem_fence_group();
      auto seed_at = [&](int i) -> bwagpu_seed_t { return i < kSelExtCache ? SC[i] : a.prog[s0 + i]; };
      auto flag_at = [&](int i) -> int {
        return i < kSelExtCache ? SC[i].pad_
                                : __hip_atomic_load(&a.skipf[s0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      };
      auto set_flag = [&](int i, int f) {
        if (r == 0) {
          if (i < kSelExtCache) SC[i].pad_ |= f;
          else __hip_atomic_store(&a.skipf[s0 + i], f | 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        mem_fence_group();
      };
      for (int k = 0; k < ns; ++k) {
        const bwagpu_seed_t s = uni_seed(seed_at(k));
        // containment in a region so far (bwamem.c:678-697), one region per lane
        bool hit = false;
        for (int base = 0; base < nreg && !hit; base += 64) {
          const int i = min(base + r, nreg - 1);
          RegRec p;
          if (i < cap_reg) {
            p = R[i];
          } else {
            const int pp = __hip_atomic_load(&a.regpos[d.s0 + i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const SeedExt* pe = a.ext + pp;
            p.rb = __hip_atomic_load(&pe->rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p.re = __hip_atomic_load(&pe->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p.qb = __hip_atomic_load(&pe->qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p.qe = __hip_atomic_load(&pe->qe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p.w = __hip_atomic_load(&pe->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            p.seedlen0 = a.prog[pp].len;
          }
          const bool inside = base + r < nreg &&
                              !(s.rbeg < p.rb || s.rbeg + s.len > p.re || s.qbeg < p.qb || s.qbeg + s.len > p.qe) &&
                              !(s.len - p.seedlen0 >= rep_lim);
          if (__builtin_amdgcn_ballot_w64(inside) == 0) continue;
          hit = __builtin_amdgcn_ballot_w64(inside && seed_near(MG, s, p)) != 0;
        }
        if (hit) {
          // a long overlapping seed of this chain already visited (bwamem.c:698-707)
          const int len95 = uni((int)ceil(s.len * .95));  // t->len < s->len * .95 <=> t->len < ceil(...)
          bool ov = false;
          for (int base = 0; base < k && !ov; base += 64) {
            const int i = min(base + r, k - 1);
            const bwagpu_seed_t t = seed_at(i);
            const bool tsk = (flag_at(i) & 1) != 0;
            const bool a1 = s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 && (int64_t)(t.qbeg - s.qbeg) != t.rbeg - s.rbeg;
            const bool b1 = t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 && (int64_t)(s.qbeg - t.qbeg) != s.rbeg - t.rbeg;
            ov = __builtin_amdgcn_ballot_w64(base + r < k && !tsk && t.len >= len95 && (a1 || b1)) != 0;
          }
          if (!ov) {  // skipped: srt[k] = 0 (bwamem.c:709)
            set_flag(k, 1);
            continue;
          }
        }
        // ---- this seed is extended (bwamem.c:717-792)
        const int pos = s0 + k;
        const SeedExt* const pe = k < kSelExtCache ? EC + k : a.ext + pos;
        SeedExt e;
        e.calls = uni(__hip_atomic_load(&pe->calls, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        if (e.calls == 0) {  // no result yet
          if constexpr (MODE == SEL_REDO) {
            e = extend_seed<16>(o, ref, s, d.lq, q, cw, tbl, tbr);
            store_ext(a.ext + pos, e);
            mem_fence_group();
            if (r == 0) atomicAdd(&a.ctr[SPC_MISS], 1);
          } else if constexpr (MODE == SEL_EMULATE) {
            set_flag(k, 2);  // pending: collected per chain below
            continue;        // its region stays unknown in this pass
          } else {
            const int list = 2 * kSpecBins + spec_bin(d.lq);
            if (r == 0) {
              const int p = atomicAdd(&a.ctr[SPC_CNT + list], 1);
              a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(pos, c);
              a.redo[atomicAdd(&a.ctr[SPC_REDO_N], 1)] = rd;
            }
            redo = true;  // the rest of this read waits for the redo pass
            break;
          }
        } else {
          e.rb = uni64(__hip_atomic_load(&pe->rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.re = uni64(__hip_atomic_load(&pe->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.qb = uni(__hip_atomic_load(&pe->qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.qe = uni(__hip_atomic_load(&pe->qe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.score = uni(__hip_atomic_load(&pe->score, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.truesc = uni(__hip_atomic_load(&pe->truesc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.w = uni(__hip_atomic_load(&pe->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.cells = uni(__hip_atomic_load(&pe->cells, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          e.rows = uni(__hip_atomic_load(&pe->rows, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
        }
        if constexpr (WRITE) {
          // seedcov over the chain's seeds (bwamem.c:784-788)
          long long cov = 0;
          for (int base = 0; base < ns; base += 64) {
            const int i = base + r;
            const bwagpu_seed_t t = seed_at(min(i, ns - 1));
            const bool in = i < ns && t.qbeg >= e.qb && t.qbeg + t.len <= e.qe && t.rbeg >= e.rb && t.rbeg + t.len <= e.re;
            cov += in ? t.len : 0;
          }
          cov = grp_sum64(cov, 64);
          write_region(a.out + d.s0 + nreg, e, rid, (int)cov, s.len, frac);
          rt.cells += e.cells;
          rt.rows += e.rows;
          rt.calls += e.calls - 1;
        }
        if (nreg < cap_reg) {
          put_regrec(R + nreg, e, s.len);
        } else {
          if (r == 0) __hip_atomic_store(&a.regpos[d.s0 + nreg], pos, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          mem_fence_group();
        }
        ++nreg;
      }
      if constexpr (MODE == SEL_EMULATE) {  // this chain's round-B tasks
        const int list = kSpecBins + spec_bin(d.lq);
        for (int base = 0; base < ns; base += 64) {
          const int i = base + r;
          const bool pnd = i < ns && (flag_at(min(i, ns - 1)) & 2) != 0;
          const int p = wave_append(&a.ctr[SPC_CNT + list], pnd);
          if (p >= 0) a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(s0 + i, c);
        }
      }
    }
    if (MODE != SEL_REDO) trace_read(MODE, b.n_reads, rd, t_start, d.ns, nreg, 2);
    if constexpr (WRITE) {
      if (!redo) {
        a.out_n[rd] = nreg;
        tl.cells += rt.cells;
        tl.rows += rt.rows;
        tl.calls += rt.calls;
      }
    }
  }
  if constexpr (WRITE) {
    if (r != 0) tl = Tally{0, 0, 0};
    block_stats<64>(tl, a.stats);
  }
}

// LIGHT reads (<= kSelLight seeds and chains): the whole read in registers,
// lane i = seed i of the read in processing order (chain-major, as prog[]
// stores them) with its SeedExt; lane c = chain c.  mem_chain2aln's
// sequential decisions depend on each other only through two bit sets — the
// seeds extended so far (their regions) and the seeds skipped so far — so:
//   1. pairs: for every seed k, the 64-bit masks of earlier seeds j whose
//      region would hold it (bwamem.c:678-697: C) and of earlier seeds of its
//      chain that overlap it (698-707, before the skip filter: O), and its
//      seedcov if extended (784-788) — lane-parallel, no loop-carried state;
//   2. scan: the sequential logic on scalar masks only:
//        hit = C[k] & extended;  skipped = hit && !(O[k] & ~skipped);
//   3. output: every extended seed's record lane-parallel at its rank.
// A seed that must be extended but has no result: SEL_EMULATE marks it a
// round-B task (pending: neither extended nor skipped, as in the per-seed
// form); SEL_FINAL sends the read to the redo pass.
// A misprediction in the final pass of a light read (a seed the replay must
// extend has no result: ~10-20 per C2 batch) is extended inline, which takes
// the kernel to 129 VGPRs (3 waves per SIMD).  Sending it to round C + the
// redo pass like one of a longer read instead (82 VGPRs) is bit-exact, but
// measured 19.8-19.9 vs 21.6-21.7 Mreads/s on C2.
template <int MODE>
__global__ void __launch_bounds__(kBlock) spec_select_light(DevOpt o, DevRef ref, DevBatch b, SpecArgs a,
                                                            int tb_bytes) {
  constexpr bool WRITE = MODE != SEL_EMULATE;
  __shared__ int32_t MG[kMglN];
  extern __shared__ __attribute__((aligned(16))) uint8_t lrows[];  // per wave: target rows of an inline extension
  uint8_t* const tbl = lrows + (threadIdx.x >> 6) * 2 * tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  for (int x = threadIdx.x; x < kMglN; x += kBlock) MG[x] = max_gap_len(o, x);
  __syncthreads();
  const int r = (int)(threadIdx.x & 63);
  const uint64_t lt_mask = r ? (~0ull >> (64 - r)) : 0ull;  // lanes below r
  Tally tl{0, 0, 0};
  // static deal: wave w takes reads w, w + NW, ... (light reads cost about the
  // same; no queue atomics), the next read's descriptor in flight meanwhile
  const int NW = (int)gridDim.x * (kBlock / 64);
  int rd = (int)blockIdx.x * (kBlock / 64) + uni((int)(threadIdx.x >> 6));
  ReadDesc dn{};
  if (rd < b.n_reads) dn = a.rdesc[rd];
  for (; rd < b.n_reads; rd += NW) {
    const uint64_t t_start = g_trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const ReadDesc d = uniform_desc(dn);
    if (rd + NW < b.n_reads) dn = a.rdesc[rd + NW];
    if (d.ns > kSelLight || d.nch > kSelLight) continue;  // the heavy kernel's read
    if (d.lq > BWAGPU_MAX_READ_LEN) continue;             // flagged by spec_reads_kernel
    if (d.ns == 0) {
      if (WRITE) a.out_n[rd] = 0;
      continue;
    }
    // a miss of the final pass is computed inline and the read starts over
    // with it (a region changes only later decisions; light reads are cheap)
    for (;;) {
    // everything of the read, one round trip
    const int ci = min(r, max(d.nch - 1, 0)), si = min(r, d.ns - 1);
    const int cs_l = b.chain_seed_off[d.c0 + ci] - d.s0, ce_l = b.chain_seed_off[d.c0 + ci + 1] - d.s0;
    const ChainWin cw_l = a.win[d.c0 + ci];
    const int rid_l = b.chain_rid[d.c0 + ci];
    const float fr_l = b.chain_frac_rep[d.c0 + ci];
    const bwagpu_seed_t sd = a.prog[d.s0 + si];
    const SeedExt x = a.ext[d.s0 + si];  // earlier launches, or this wave's inline extension
    // this seed's chain (a chain with a flagged window is never processed)
    int cid = 0, rid = 0;
    float frac = 0.f;
    bool vchain = false;
    for (int c = 0; c < d.nch; ++c) {
      const int cs = __builtin_amdgcn_readlane(cs_l, c), ce = __builtin_amdgcn_readlane(ce_l, c);
      const bool in = r >= cs && r < ce;
      const bool ok = readlane64(cw_l.hi, c) >= readlane64(cw_l.lo, c);
      cid = in ? c : cid;
      vchain = in ? ok : vchain;
      rid = in ? __builtin_amdgcn_readlane(rid_l, c) : rid;
      frac = in ? __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fr_l), c)) : frac;
    }
    const bool present = r < d.ns && vchain;
    const bool computed = present && x.calls != 0;
    const uint64_t present_m = __builtin_amdgcn_ballot_w64(present);
    const uint64_t computed_m = __builtin_amdgcn_ballot_w64(computed);
    const uint64_t pad_m = __builtin_amdgcn_ballot_w64(r < d.ns && sd.pad_ != 0);
    const int rep_lim = (int)floor(.1 * d.lq) + 1;  // s->len - p->seedlen0 > .1 * l_query, bwamem.c:685
    // ---- 1. pair masks: lane p = (k, j) = (p / S, p % S) with S the seed count
    // rounded up to a power of two (8..64), 64 / S values of k per pass; pass
    // `it`'s ballots land in lane it (c_*, o_*); seedcov of k's region in lane k
    const int S = d.ns <= 8 ? 8 : d.ns <= 16 ? 16 : d.ns <= 32 ? 32 : 64;
    const int lgS = S == 8 ? 3 : S == 16 ? 4 : S == 32 ? 5 : 6;
    const int npass = (S * S) >> 6;
    uint32_t c_lo = 0, c_hi = 0, o_lo = 0, o_hi = 0;
    int cov = 0;
    const int j = r & (S - 1);
    const int jl = min(j, d.ns - 1) << 2;
    // seed j of this lane (and its region), gathered once
    const int64_t j_rbeg = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)(sd.rbeg >> 32)) << 32 |
                                     (uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)sd.rbeg));
    const int j_qbeg = __builtin_amdgcn_ds_bpermute(jl, sd.qbeg), j_len = __builtin_amdgcn_ds_bpermute(jl, sd.len);
    const int j_cid = __builtin_amdgcn_ds_bpermute(jl, cid);
    const bool j_pad = __builtin_amdgcn_ds_bpermute(jl, sd.pad_) != 0;
    const bool j_done = __builtin_amdgcn_ds_bpermute(jl, computed ? 1 : 0) != 0;
    RegRec pj;
    pj.rb = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)(x.rb >> 32)) << 32 |
                      (uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)x.rb));
    pj.re = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)(x.re >> 32)) << 32 |
                      (uint32_t)__builtin_amdgcn_ds_bpermute(jl, (int)x.re));
    pj.qb = __builtin_amdgcn_ds_bpermute(jl, x.qb);
    pj.qe = __builtin_amdgcn_ds_bpermute(jl, x.qe);
    pj.w = __builtin_amdgcn_ds_bpermute(jl, x.w);
    pj.seedlen0 = j_len;
    for (int it = 0; it < npass; ++it) {
      const int k = (it << (6 - lgS)) + (r >> lgS);
      const int kl = min(k, d.ns - 1) << 2;
      bwagpu_seed_t sk;
      sk.rbeg = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)(sd.rbeg >> 32)) << 32 |
                          (uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)sd.rbeg));
      sk.qbeg = __builtin_amdgcn_ds_bpermute(kl, sd.qbeg);
      sk.len = __builtin_amdgcn_ds_bpermute(kl, sd.len);
      const int k_cid = __builtin_amdgcn_ds_bpermute(kl, cid);
      const bool valid = k < d.ns && j < d.ns;
      // C: the region of seed j holds seed k (bwamem.c:682-696)
      const bool inside = valid && j < k && j_done &&
                          !(sk.rbeg < pj.rb || sk.rbeg + sk.len > pj.re || sk.qbeg < pj.qb || sk.qbeg + sk.len > pj.qe) &&
                          !(sk.len - j_len >= rep_lim);
      uint64_t cm = __builtin_amdgcn_ballot_w64(inside);
      if (cm) cm = __builtin_amdgcn_ballot_w64(inside && seed_near(MG, sk, pj));
      // O: seed j of k's chain overlaps it (bwamem.c:701-704; t->len < s->len * .95 <=> t->len < ceil(...))
      const int len95 = (int)ceil(sk.len * .95);
      const bool a1 = sk.qbeg <= j_qbeg && sk.qbeg + sk.len - j_qbeg >= sk.len >> 2 &&
                      (int64_t)(j_qbeg - sk.qbeg) != j_rbeg - sk.rbeg;
      const bool b1 = j_qbeg <= sk.qbeg && j_qbeg + j_len - sk.qbeg >= sk.len >> 2 &&
                      (int64_t)(sk.qbeg - j_qbeg) != sk.rbeg - j_rbeg;
      const uint64_t om = __builtin_amdgcn_ballot_w64(valid && j < k && j_cid == k_cid && !j_pad && j_len >= len95 && (a1 || b1));
      c_lo = r == it ? (uint32_t)cm : c_lo;
      c_hi = r == it ? (uint32_t)(cm >> 32) : c_hi;
      o_lo = r == it ? (uint32_t)om : o_lo;
      o_hi = r == it ? (uint32_t)(om >> 32) : o_hi;
      if (WRITE) {  // seedcov of k's region over its chain's seeds (bwamem.c:784-788)
        const int64_t krb = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)(x.rb >> 32)) << 32 |
                                      (uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)x.rb));
        const int64_t kre = (int64_t)((uint64_t)(uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)(x.re >> 32)) << 32 |
                                      (uint32_t)__builtin_amdgcn_ds_bpermute(kl, (int)x.re));
        const int kqb = __builtin_amdgcn_ds_bpermute(kl, x.qb), kqe = __builtin_amdgcn_ds_bpermute(kl, x.qe);
        int v = valid && j_cid == k_cid && j_qbeg >= kqb && j_qbeg + j_len <= kqe && j_rbeg >= krb &&
                        j_rbeg + j_len <= kre ? j_len : 0;
        for (int m = 1; m < S; m <<= 1) v += __shfl_xor(v, m, 64);
        // lane k takes the sum of its group (lane (k - first k of the pass) * S)
        const int src = (r - (it << (6 - lgS))) << lgS;
        const int got = __builtin_amdgcn_ds_bpermute(min(max(src, 0), 63) << 2, v);
        cov = (r >= (it << (6 - lgS)) && r < ((it + 1) << (6 - lgS))) ? got : cov;
      }
    }
    // ---- 2. the sequential decisions, on scalar masks
    uint64_t ext = 0, skip = pad_m, pend = 0;
    int miss = -1;
    for (int k = 0; k < d.ns; ++k) {
      const uint64_t bit = 1ull << k;
      if (!(present_m & bit)) continue;
      const int it = (k << lgS) >> 6, sh = (k << lgS) & 63;
      const uint64_t fld = S == 64 ? ~0ull : ((1ull << S) - 1);
      const uint64_t cm = ((uint64_t)__builtin_amdgcn_readlane(c_hi, it) << 32 | (uint32_t)__builtin_amdgcn_readlane(c_lo, it)) >> sh & fld;
      if (cm & ext) {
        const uint64_t om = ((uint64_t)__builtin_amdgcn_readlane(o_hi, it) << 32 | (uint32_t)__builtin_amdgcn_readlane(o_lo, it)) >> sh & fld;
        if (!(om & ~skip)) {  // skipped: srt[k] = 0 (bwamem.c:709)
          skip |= bit;
          continue;
        }
      }
      if (!(computed_m & bit)) {
        if (MODE == SEL_EMULATE) {
          pend |= bit;  // a round-B task; its region stays unknown in this pass
          continue;
        }
        miss = k;
        break;
      }
      ext |= bit;
    }
    // ---- 3. outputs
    if constexpr (MODE == SEL_EMULATE) {
      const int list = kSpecBins + spec_bin(d.lq);
      const bool pnd = (pend >> r) & 1;
      const int p = wave_append(&a.ctr[SPC_CNT + list], pnd);
      if (p >= 0) a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + r, d.c0 + cid);
    } else {
      if (miss >= 0 && d.lq <= kSpecBinLen[0]) {  // extend seed `miss` here, then the read again
        const bwagpu_seed_t sm = uni_seed(a.prog[d.s0 + miss]);
        const int cm_id = uni(__shfl(cid, miss, 64));
        ChainWin cw = a.win[d.c0 + cm_id];
        cw.lo = uni64(cw.lo);
        cw.hi = uni64(cw.hi);
        const SeedExt e = extend_seed<3>(o, ref, sm, d.lq, b.seq + d.qoff, cw, tbl, tbr);
        store_ext(a.ext + d.s0 + miss, e);
        if (r == 0) atomicAdd(&a.ctr[SPC_MISS], 1);
        mem_fence_group();
        __builtin_amdgcn_wave_barrier();
        continue;
      }
      if (miss >= 0) {  // round C + the redo pass (reads > 160 bp)
        const int list = 2 * kSpecBins + spec_bin(d.lq);
        if (r == miss) {
          const int p = atomicAdd(&a.ctr[SPC_CNT + list], 1);
          a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + r, d.c0 + cid);
          a.redo[atomicAdd(&a.ctr[SPC_REDO_N], 1)] = rd;
        }
        break;  // the redo pass writes this read
      }
      const bool mine = (ext >> r) & 1;
      if (mine) {  // the region of seed r, at its rank (bwamem.c:718-792 field by field; rest zero)
        const int slot = (int)__popcll(ext & lt_mask);
        uint2* dst = reinterpret_cast<uint2*>(a.out + d.s0 + slot);
        dst[0] = make_uint2((uint32_t)x.rb, (uint32_t)((uint64_t)x.rb >> 32));
        dst[1] = make_uint2((uint32_t)x.re, (uint32_t)((uint64_t)x.re >> 32));
        dst[2] = make_uint2((uint32_t)x.qb, (uint32_t)x.qe);
        dst[3] = make_uint2((uint32_t)rid, (uint32_t)x.score);
        dst[4] = make_uint2((uint32_t)x.truesc, 0u);
        dst[5] = make_uint2(0u, 0u);
        dst[6] = make_uint2(0u, (uint32_t)x.w);
        dst[7] = make_uint2((uint32_t)cov, 0u);
        dst[8] = make_uint2(0u, (uint32_t)sd.len);
        dst[9] = make_uint2(0u, __float_as_uint(frac));
        dst[10] = make_uint2(0u, 0u);
        tl.cells += x.cells;
        tl.rows += x.rows;
        tl.calls += x.calls - 1;
      }
      if (r == 0) a.out_n[rd] = (int)__popcll(ext);
    }
    trace_read(MODE, b.n_reads, rd, t_start, d.ns, (int)__popcll(ext), 1);
    break;
    }  // the read's attempts
  }
  if constexpr (WRITE) block_stats<64>(tl, a.stats);
}

// HEAVY reads with pair matrices (<= kSelMatMaxSeeds seeds).  The same
// decomposition as the light kernel, at a size where one wave cannot hold the
// read:
//   spec_pairs_kernel — one wave per column k (a seed) of a heavy read, over
//     every column of every such read at once: 64-bit words of C[k] (earlier
//     seeds whose region would hold k: bwamem.c:678-697) and O[k] (earlier
//     seeds of k's chain overlapping it: 698-707), and k's seedcov (784-788);
//   spec_scan_kernel  — one wave per read: the sequential decisions on bit
//     sets (lane w holds word w of the extended / skipped / pending sets), then
//     every extended seed's record lane-parallel at its rank.
__global__ void __launch_bounds__(kBlock) spec_pairs_kernel(DevOpt o, DevBatch b, SpecArgs a, int with_cov) {
  __shared__ int32_t MG[kMglN];
  for (int x = threadIdx.x; x < kMglN; x += kBlock) MG[x] = max_gap_len(o, x);
  __syncthreads();
  const int r = (int)(threadIdx.x & 63);
  const int ncol = uni(__hip_atomic_load(&a.ctr[SPC_HCOLS], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int nwv = (int)gridDim.x * (kBlock / 64);
  for (int x = (int)blockIdx.x * (kBlock / 64) + uni((int)(threadIdx.x >> 6)); x < ncol; x += nwv) {
    const int t = uni(a.colent[x]);
    const int4 hi = a.hinfo[t];
    const int rd = uni(hi.x), woff = uni(hi.y), col = uni(hi.z), ns = uni(hi.w);
    const int k = x - col, nw = (ns + 63) >> 6;
    const ReadDesc d = uniform_desc(a.rdesc[rd]);
    const int rep_lim = (int)floor(.1 * d.lq) + 1;  // s->len - p->seedlen0 > .1 * l_query, bwamem.c:685
    const bwagpu_seed_t s = uni_seed(a.prog[d.s0 + k]);
    const int ck = uni(a.seedchain[d.s0 + k]);
    const int len95 = uni((int)ceil(s.len * .95));  // t->len < s->len * .95 <=> t->len < ceil(...)
    const SeedExt ek = a.ext[d.s0 + k];
    const bool k_done = uni(ek.calls) != 0;
    const int64_t krb = uni64(ek.rb), kre = uni64(ek.re);
    const int kqb = uni(ek.qb), kqe = uni(ek.qe);
    int cov = 0;
    for (int w = 0; w < nw; ++w) {
      const int j = 64 * w + r, jj = min(j, ns - 1);
      const bwagpu_seed_t sj = a.prog[d.s0 + jj];
      const int cj = a.seedchain[d.s0 + jj];
      const SeedExt ej = a.ext[d.s0 + jj];
      RegRec p;
      p.rb = ej.rb;
      p.re = ej.re;
      p.qb = ej.qb;
      p.qe = ej.qe;
      p.w = ej.w;
      p.seedlen0 = sj.len;
      const bool inside = j < k && ej.calls != 0 &&
                          !(s.rbeg < p.rb || s.rbeg + s.len > p.re || s.qbeg < p.qb || s.qbeg + s.len > p.qe) &&
                          !(s.len - sj.len >= rep_lim);
      uint64_t cm = __builtin_amdgcn_ballot_w64(inside);
      if (cm) cm = __builtin_amdgcn_ballot_w64(inside && seed_near(MG, s, p));
      const bool a1 = s.qbeg <= sj.qbeg && s.qbeg + s.len - sj.qbeg >= s.len >> 2 &&
                      (int64_t)(sj.qbeg - s.qbeg) != sj.rbeg - s.rbeg;
      const bool b1 = sj.qbeg <= s.qbeg && sj.qbeg + sj.len - s.qbeg >= s.len >> 2 &&
                      (int64_t)(s.qbeg - sj.qbeg) != s.rbeg - sj.rbeg;
      const uint64_t om = __builtin_amdgcn_ballot_w64(j < k && cj == ck && sj.pad_ == 0 && sj.len >= len95 && (a1 || b1));
      if (r == 0 && 64 * w < k) {
        a.mat[woff + tri_off(k) + w] = cm;
        a.mat[woff + tri_off(ns) + tri_off(k) + w] = om;
      }
      if (with_cov && k_done)
        cov += (j < ns && cj == ck && sj.qbeg >= kqb && sj.qbeg + sj.len <= kqe && sj.rbeg >= krb &&
                sj.rbeg + sj.len <= kre) ? sj.len : 0;
    }
    if (with_cov) {
      cov = (int)grp_sum64(cov, 64);
      if (r == 0) a.cov[d.s0 + k] = cov;
    }
  }
}

constexpr int kScanLds = 64 * 1024;  // a read's C and O matrices staged in LDS when they fit

// The final pass over a heavy read computes a missing extension INLINE (the
// read's wave runs extend_seed, then sets the new region's containment bits in
// column k of C for every later seed, and k's seedcov) and carries on: a
// region only changes the decisions of the seeds after it, so the scan state
// up to k stays valid.  (Deferring such a read to round C + the serial redo
// pass cost 2.4-2.6 ms on one read of 1,167 seeds and 749 regions.)
__device__ __forceinline__ void heavy_fill_missing(const DevOpt& o, const DevRef& ref, const DevBatch& b,
                                                   const SpecArgs& a, const ReadDesc& d, int k, int ns,
                                                   uint64_t* C, uint8_t* tbl, uint8_t* tbr) {
  const int r = (int)(threadIdx.x & 63);
  const bwagpu_seed_t sk = uni_seed(a.prog[d.s0 + k]);
  const int ck = uni(a.seedchain[d.s0 + k]);
  ChainWin cw = a.win[ck];
  cw.lo = uni64(cw.lo);
  cw.hi = uni64(cw.hi);
  const SeedExt e = extend_seed<3>(o, ref, sk, d.lq, b.seq + d.qoff, cw, tbl, tbr);  // reads <= 192 bp
  store_ext(a.ext + d.s0 + k, e);
  if (r == 0) atomicAdd(&a.ctr[SPC_MISS], 1);
  // region k as the containment tests see it (bwamem.c:682-696)
  RegRec p;
  p.rb = e.rb;
  p.re = e.re;
  p.qb = e.qb;
  p.qe = e.qe;
  p.w = e.w;
  p.seedlen0 = sk.len;
  const int rep_lim = (int)floor(.1 * d.lq) + 1;  // s->len - p->seedlen0 > .1 * l_query, bwamem.c:685
  int cov = 0;
  for (int base = 0; base < ns; base += 64) {
    const int j = base + r, jj = min(j, ns - 1);
    const bwagpu_seed_t sj = a.prog[d.s0 + jj];
    // column k of C for the later seeds j > k (the pairs kernel's predicate)
    bool in = j > k && j < ns && !(sj.rbeg < p.rb || sj.rbeg + sj.len > p.re || sj.qbeg < p.qb || sj.qbeg + sj.len > p.qe) &&
              !(sj.len - sk.len >= rep_lim);
    if (in) {
      const int qd1 = sj.qbeg - p.qb;
      const int64_t rd1 = sj.rbeg - p.rb;
      const int g1 = max_gap_len(o, max(qd1 < rd1 ? qd1 : (int)rd1, 0));
      const int bw1 = g1 < p.w ? g1 : p.w;
      const int qd2 = p.qe - (sj.qbeg + sj.len);
      const int64_t rd2 = p.re - (sj.rbeg + sj.len);
      const int g2 = max_gap_len(o, max(qd2 < rd2 ? qd2 : (int)rd2, 0));
      const int bw2 = g2 < p.w ? g2 : p.w;
      in = (qd1 - rd1 < bw1 && rd1 - qd1 < bw1) || (qd2 - rd2 < bw2 && rd2 - qd2 < bw2);
    }
    if (in) C[tri_off(j) + (k >> 6)] |= 1ull << (k & 63);  // word k>>6 of row j: this lane's alone
    // seedcov of k (bwamem.c:784-788): its chain's seeds inside region k
    const int cj = a.seedchain[d.s0 + jj];
    cov += (j < ns && cj == ck && sj.qbeg >= p.qb && sj.qbeg + sj.len <= p.qe && sj.rbeg >= p.rb &&
            sj.rbeg + sj.len <= p.re) ? sj.len : 0;
  }
  cov = (int)grp_sum64(cov, 64);
  if (r == 0) a.cov[d.s0 + k] = cov;
  // the wave re-reads C (LDS or its own global writes) and ext/cov next
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

template <int MODE>
__global__ void __launch_bounds__(64) spec_scan_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int tb_bytes) {
  constexpr bool WRITE = MODE != SEL_EMULATE;
  extern __shared__ __attribute__((aligned(16))) uint64_t M[];
  uint8_t* const tbl = reinterpret_cast<uint8_t*>(M) + kScanLds;
  uint8_t* const tbr = tbl + tb_bytes;
  const int r = (int)(threadIdx.x & 63);
  const uint64_t lt_mask = r ? (~0ull >> (64 - r)) : 0ull;
  const int nh = uni(__hip_atomic_load(&a.ctr[SPC_HEAVY_N], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  Tally tl{0, 0, 0};
  for (int t = (int)blockIdx.x; t < nh; t += (int)gridDim.x) {
    const int4 hi = a.hinfo[t];
    const int rd = uni(hi.x), woff = uni(hi.y), ns = uni(hi.w);
    if (woff < 0) continue;  // no matrix: the per-seed heavy kernel's read
    const uint64_t t_start = g_trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const int nw = (ns + 63) >> 6;
    const ReadDesc d = uniform_desc(a.rdesc[rd]);
    if (d.lq > BWAGPU_MAX_READ_LEN) continue;
    const int64_t tw = tri_off(ns);
    const uint64_t* Cg = a.mat + woff;
    const bool staged = 2 * tw * 8 <= kScanLds;
    if (staged) {
      for (int i = r; i < 2 * tw; i += 64) M[i] = Cg[i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    uint64_t* C = staged ? M : a.mat + woff;
    const uint64_t* O = C + tw;
    // per-word sets: lane w holds word w
    uint64_t present_w = 0, computed_w = 0, skip_w = 0;
    for (int w = 0; w < nw; ++w) {
      const int j = 64 * w + r, jj = min(j, ns - 1);
      const bwagpu_seed_t sj = a.prog[d.s0 + jj];
      const ChainWin cw = a.win[a.seedchain[d.s0 + jj]];
      const bool pres = j < ns && cw.hi >= cw.lo;  // seeds of a flagged chain are never processed
      const uint64_t pm = __builtin_amdgcn_ballot_w64(pres);
      const uint64_t cm = __builtin_amdgcn_ballot_w64(pres && a.ext[d.s0 + jj].calls != 0);
      const uint64_t km = __builtin_amdgcn_ballot_w64(j < ns && sj.pad_ != 0);
      present_w = r == w ? pm : present_w;
      computed_w = r == w ? cm : computed_w;
      skip_w = r == w ? km : skip_w;
    }
    uint64_t ext_w = 0, pend_w = 0;
    int miss = -1;
    for (int k = 0; k < ns; ++k) {
      const int kw = k >> 6;
      const uint64_t kbit = 1ull << (k & 63);
      const uint64_t pres = (uint64_t)__builtin_amdgcn_readlane((uint32_t)(present_w >> 32), kw) << 32 |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)present_w, kw);
      if (!(pres & kbit)) continue;
      const int nwk = (k + 63) >> 6;  // words of row k
      const uint64_t cw = r < nwk ? C[tri_off(k) + r] : 0;
      if (__builtin_amdgcn_ballot_w64((cw & ext_w) != 0)) {
        const uint64_t ow = r < nwk ? O[tri_off(k) + r] : 0;
        if (!__builtin_amdgcn_ballot_w64((ow & ~skip_w) != 0)) {  // skipped: srt[k] = 0 (bwamem.c:709)
          skip_w |= r == kw ? kbit : 0;
          continue;
        }
      }
      const uint64_t comp = (uint64_t)__builtin_amdgcn_readlane((uint32_t)(computed_w >> 32), kw) << 32 |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)computed_w, kw);
      if (!(comp & kbit)) {
        if (MODE == SEL_EMULATE) {
          pend_w |= r == kw ? kbit : 0;  // a round-B task; its region stays unknown
          continue;
        }
        if (d.lq > kSpecBinLen[0]) {  // longer reads: round C + the redo pass
          miss = k;
          break;
        }
        heavy_fill_missing(o, ref, b, a, d, k, ns, C, tbl, tbr);
        computed_w |= r == kw ? kbit : 0;
      }
      ext_w |= r == kw ? kbit : 0;
    }
    int nreg = 0;
    if constexpr (MODE == SEL_EMULATE) {
      const int list = kSpecBins + spec_bin(d.lq);
      for (int w = 0; w < nw; ++w) {
        const uint64_t pw = (uint64_t)__builtin_amdgcn_readlane((uint32_t)(pend_w >> 32), w) << 32 |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)pend_w, w);
        const int j = 64 * w + r;
        const bool pnd = (pw >> r) & 1;
        const int p = wave_append(&a.ctr[SPC_CNT + list], pnd);
        if (p >= 0) a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + j, a.seedchain[d.s0 + j]);
      }
    } else {
      if (miss >= 0) {
        if (r == 0) {
          const int list = 2 * kSpecBins + spec_bin(d.lq);
          const int p = atomicAdd(&a.ctr[SPC_CNT + list], 1);
          a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + miss, a.seedchain[d.s0 + miss]);
          a.redo[atomicAdd(&a.ctr[SPC_REDO_N], 1)] = rd;
        }
        continue;  // the redo pass writes this read
      }
      for (int w = 0; w < nw; ++w) {
        const uint64_t ew = (uint64_t)__builtin_amdgcn_readlane((uint32_t)(ext_w >> 32), w) << 32 |
                            (uint32_t)__builtin_amdgcn_readlane((uint32_t)ext_w, w);
        const int j = 64 * w + r;
        if ((ew >> r) & 1) {  // the region of seed j at its rank (bwamem.c:718-792; rest zero)
          const int slot = nreg + (int)__popcll(ew & lt_mask);
          const SeedExt x = a.ext[d.s0 + j];
          const int c = a.seedchain[d.s0 + j];
          uint2* dst = reinterpret_cast<uint2*>(a.out + d.s0 + slot);
          dst[0] = make_uint2((uint32_t)x.rb, (uint32_t)((uint64_t)x.rb >> 32));
          dst[1] = make_uint2((uint32_t)x.re, (uint32_t)((uint64_t)x.re >> 32));
          dst[2] = make_uint2((uint32_t)x.qb, (uint32_t)x.qe);
          dst[3] = make_uint2((uint32_t)b.chain_rid[c], (uint32_t)x.score);
          dst[4] = make_uint2((uint32_t)x.truesc, 0u);
          dst[5] = make_uint2(0u, 0u);
          dst[6] = make_uint2(0u, (uint32_t)x.w);
          dst[7] = make_uint2((uint32_t)a.cov[d.s0 + j], 0u);
          dst[8] = make_uint2(0u, (uint32_t)a.prog[d.s0 + j].len);
          dst[9] = make_uint2(0u, __float_as_uint(b.chain_frac_rep[c]));
          dst[10] = make_uint2(0u, 0u);
          tl.cells += x.cells;
          tl.rows += x.rows;
          tl.calls += x.calls - 1;
        }
        nreg += (int)__popcll(ew);
      }
      if (r == 0) a.out_n[rd] = nreg;
    }
    trace_read(MODE, b.n_reads, rd, t_start, ns, nreg, 3);
  }
  if constexpr (WRITE) block_stats<64>(tl, a.stats);
}

// spec_scan_kernel's grid: one wave per workgroup, a static stride over the
// heavy reads (256-2048 measured within the noise)
constexpr int kScanGrid = 1024;

// The two selection shapes of one pass: heavy reads on `side` (when given)
// concurrently with the light reads on `st`; `st` continues once both are done.
template <int MODE>
static void launch_select(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a, int tb_bytes,
                          hipStream_t st, const SpecStreams& ss) {
  hipStream_t hs = st;
  if (MODE != SEL_REDO && ss.side) {
    (void)hipEventRecord(ss.fork, st);
    (void)hipStreamWaitEvent(ss.side, ss.fork, 0);
    hs = ss.side;
  }
  if (MODE != SEL_REDO) {
    const size_t lds = (size_t)(kBlock / 64) * 2 * tb_bytes;
    const int nb = resident_blocks(spec_select_light<MODE>, lds);
    hipLaunchKernelGGL((spec_select_light<MODE>), dim3(nb), dim3(kBlock), lds, st, o, ref, b, a, tb_bytes);
  }
  if (MODE != SEL_REDO) {  // heavy reads with pair matrices: all pairs at once, then one scan per read
    const int nb = resident_blocks(spec_pairs_kernel, 0);
    hipLaunchKernelGGL(spec_pairs_kernel, dim3(nb), dim3(kBlock), 0, hs, o, b, a, MODE == SEL_FINAL ? 1 : 0);
    hipLaunchKernelGGL((spec_scan_kernel<MODE>), dim3(kScanGrid), dim3(64), (size_t)kScanLds + 2 * (size_t)tb_bytes, hs, o,
                       ref, b, a, tb_bytes);
  }
  // the rest (no matrix; the redo list): one wave per read, per seed
  hipLaunchKernelGGL((spec_select_kernel<MODE, true>), dim3(MODE == SEL_REDO ? 256 : 1024), dim3(64),
                     (size_t)kSelHeavyLds, hs, o, ref, b, a, tb_bytes);
  if (hs != st) {
    (void)hipEventRecord(ss.join, hs);
    (void)hipStreamWaitEvent(st, ss.join, 0);
  }
}

// The first two length bins' extension kernel: four seeds per wave
// (spec_ext4_kernel, packed 16-bit DP) when every score of the bin fits the
// packed ranges, else two per wave (spec_ext2_kernel, 32-bit).
// bwagpu_debug_ext_form(1) forces two per wave (tests, A/B).
static std::atomic<int> g_ext_form{0};
int ext_form() { return g_ext_form.load(std::memory_order_relaxed); }
int set_ext_form(int form) {  // process-wide; -> the previous form (form < 0: query only)
  const int prev = g_ext_form.load(std::memory_order_relaxed);
  if (form >= 0) g_ext_form.store(form > 1 ? 1 : form, std::memory_order_relaxed);
  return prev;
}
// the packed ranges (extend_quad) for reads up to lq: H <= lq * max(mat) < 4096
// (the row-max key H << KS | c, KS <= 3), H * 2^sk + 128 < 2^15 (2^sk >
// max(mat)), and the scan values H + 33 * CPL * e_ins < 2^15
bool quad_bound_ok(const DevOpt& o, long hb) {  // hb: a bound on every H of the call
  if (o.max_mat < 1 || o.max_mat > 15) return false;
  const int sk = 32 - __builtin_clz((unsigned)o.max_mat);
  for (int k = 0; k < 25; ++k)
    if (o.mat[k] < -127 || o.mat[k] > 127) return false;
  return hb < 4096 && (hb << sk) + 128 < 32768 && hb + 33L * 8 * o.e_ins < 32768 && o.o_del + 128L < 32768 &&
         o.oe_ins + 128L < 32768 && o.e_del < 32768;
}
bool quad_scores_ok(const DevOpt& o, int lq) { return quad_bound_ok(o, (long)lq * o.max_mat); }
// the packed row-end state for calls of up to `rows` target rows: i, |i - j|
// and the z-drop term max((di - dj) e_del, (dj - di) e_ins) (di <= rows,
// dj <= 256) within 16 bits beside H < 4096
bool quad_rows_ok(const DevOpt& o, long rows) {
  return rows >= 0 && rows < 16384 && (rows + 256) * std::max(o.e_del, o.e_ins) < 28672;
}

static void launch_ext_round(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a, int round,
                             int tb_bytes, hipStream_t st, const SpecStreams& ss) {
  const size_t lds = (size_t)(kBlock / 64) * 2 * tb_bytes;
  const int l = round * kSpecBins;
  const bool quad = g_ext_form.load(std::memory_order_relaxed) == 0 && quad_scores_ok(o, kSpecBinLen[1]) &&
                    quad_rows_ok(o, tb_bytes);
  const size_t lds2 = quad ? ext4_lds(tb_bytes) : ext2_lds(tb_bytes);
  // the first two length bins' lists in pair order (spec_sort_*), then two or
  // four seeds per wave; the third (reads > 256 bp) one seed per wave
  hipLaunchKernelGGL(spec_sort_count, dim3(256, 2), dim3(256), 0, st, b, a, round);
  hipLaunchKernelGGL(spec_sort_scan, dim3(2), dim3(256), 0, st, a, round);
  hipLaunchKernelGGL(spec_sort_scatter, dim3(256, 2), dim3(256), 0, st, b, a, round);
  const bool prof = ss.pool && *ss.pool_used + 2 <= ss.pool_n;
  if (prof) (void)hipEventRecord(ss.pool[*ss.pool_used], st);
  if (quad) {
    const int nb = resident_blocks(spec_ext4_kernel<kSpecBinLen[0] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext4_kernel<kSpecBinLen[0] / 32>, dim3(ext2_grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 0, tb_bytes);
  } else {
    const int nb = resident_blocks(spec_ext2_kernel<kSpecBinLen[0] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext2_kernel<kSpecBinLen[0] / 32>, dim3(ext2_grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 0, tb_bytes);
  }
  if (prof) {
    (void)hipEventRecord(ss.pool[*ss.pool_used + 1], st);
    *ss.pool_used += 2;
  }
  if (quad) {
    const int nb = resident_blocks(spec_ext4_kernel<kSpecBinLen[1] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext4_kernel<kSpecBinLen[1] / 32>, dim3(ext2_grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 1, tb_bytes);
  } else {
    const int nb = resident_blocks(spec_ext2_kernel<kSpecBinLen[1] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext2_kernel<kSpecBinLen[1] / 32>, dim3(ext2_grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 1, tb_bytes);
  }
  const int nb = resident_blocks(spec_ext_kernel<16>, lds);
  hipLaunchKernelGGL(spec_ext_kernel<16>, dim3(nb), dim3(kBlock), lds, st, o, ref, b, a, l + 2, tb_bytes);
}

// prep -> round A -> emulate -> round B -> final -> round C -> redo, one stream
hipError_t launch_spec_chain2aln(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a,
                                 int tb_bytes, hipStream_t st, const SpecStreams& ss) {
  if (b.n_reads == 0) return hipSuccess;
  hipLaunchKernelGGL(spec_reads_kernel, dim3((b.n_reads + 255) / 256), dim3(256), 0, st, b, a);
  if (b.n_chains) {
    hipLaunchKernelGGL(spec_chain_kernel, dim3((b.n_chains + 255) / 256), dim3(256), 0, st, o, ref, b, a);
    hipLaunchKernelGGL(spec_order_kernel, dim3(kOrderBlocks), dim3(256), 0, st, o, ref, b, a);
  }
  if (b.n_chains) {
    launch_ext_round(o, ref, b, a, 0, tb_bytes, st, ss);
    launch_select<SEL_EMULATE>(o, ref, b, a, tb_bytes, st, ss);
    launch_ext_round(o, ref, b, a, 1, tb_bytes, st, ss);
  }
  launch_select<SEL_FINAL>(o, ref, b, a, tb_bytes, st, ss);
  if (b.n_chains) {
    launch_ext_round(o, ref, b, a, 2, tb_bytes, st, ss);
    launch_select<SEL_REDO>(o, ref, b, a, tb_bytes, st, ss);
  }
  return hipGetLastError();
}

size_t spec_select_lds(int tb_bytes) { return (size_t)kSelHeavyLds + 0 * tb_bytes; }
int spec_redo_cap(int tb_bytes) { return sel_heavy_cap(SEL_REDO, tb_bytes); }

}  // namespace bwagpu
