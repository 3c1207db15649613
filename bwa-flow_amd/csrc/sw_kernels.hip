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

#include "engine.h"

namespace bwagpu {

const Variant kVariants[kNumVariants] = {{16, 10}, {32, 8}, {64, 16}};

// ---------------------------------------------------------------- group ops
// Cross-lane primitives restricted to one group.  G = 16 is exactly one DPP
// row, so everything is a DPP-modified VALU op (row_shr / row_ror): no LDS
// crossbar round trip on the per-row critical path.  Wider groups fall back to
// ds_bpermute-based shuffles.
constexpr int DPP_ROW_SHR(int n) { return 0x110 + n; }
constexpr int DPP_ROW_ROR(int n) { return 0x120 + n; }

template <int CTRL>
__device__ __forceinline__ int dpp(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xF, 0xF, false);
}

template <int G>
struct Grp {
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & (G - 1)); }
  static __device__ __forceinline__ int gmax(int v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, G));
    return v;
  }
  static __device__ __forceinline__ int gmin(int v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, G));
    return v;
  }
  // max over lanes strictly below this one; `ident` for lane 0
  static __device__ __forceinline__ int excl_max(int v, int ident) {
    const int l = lane();
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      int y = __shfl_up(v, o, G);
      if (l >= o) v = max(v, y);
    }
    int e = __shfl_up(v, 1, G);
    return l == 0 ? ident : e;
  }
  static __device__ __forceinline__ int up1(int v) { return __shfl_up(v, 1, G); }
  static __device__ __forceinline__ int bcast(int v, int src) { return __shfl(v, src, G); }
};

template <>
struct Grp<16> {
  // every step is `x = op(x, dpp(x))` with old == x, the form LLVM's DPP
  // combiner folds into one v_{max,min}_i32_dpp (lanes whose DPP source lies
  // outside the row keep x)
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & 15); }
  static __device__ __forceinline__ int gmax(int v) {
    v = max(v, dpp<DPP_ROW_ROR(8)>(v, v));
    v = max(v, dpp<DPP_ROW_ROR(4)>(v, v));
    v = max(v, dpp<DPP_ROW_ROR(2)>(v, v));
    return max(v, dpp<DPP_ROW_ROR(1)>(v, v));
  }
  static __device__ __forceinline__ int gmin(int v) {
    v = min(v, dpp<DPP_ROW_ROR(8)>(v, v));
    v = min(v, dpp<DPP_ROW_ROR(4)>(v, v));
    v = min(v, dpp<DPP_ROW_ROR(2)>(v, v));
    return min(v, dpp<DPP_ROW_ROR(1)>(v, v));
  }
  static __device__ __forceinline__ int excl_max(int v, int ident) {
    v = max(v, dpp<DPP_ROW_SHR(1)>(v, v));
    v = max(v, dpp<DPP_ROW_SHR(2)>(v, v));
    v = max(v, dpp<DPP_ROW_SHR(4)>(v, v));
    v = max(v, dpp<DPP_ROW_SHR(8)>(v, v));
    return dpp<DPP_ROW_SHR(1)>(ident, v);
  }
  static __device__ __forceinline__ int up1(int v) { return dpp<DPP_ROW_SHR(1)>(v, v); }
  static __device__ __forceinline__ int bcast(int v, int src) { return __shfl(v, src, 16); }
};

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

// cal_max_gap, bwamem.c:630-637
__device__ __forceinline__ int max_gap_len(const DevOpt& o, int qlen) {
  int ld = (int)((double)(qlen * o.a - o.o_del) / o.e_del + 1.);
  int li = (int)((double)(qlen * o.a - o.o_ins) / o.e_ins + 1.);
  int l = ld > li ? ld : li;
  l = l > 1 ? l : 1;
  return l < (o.w << 1) ? l : (o.w << 1);
}

struct ExtOut {
  int score, qle, tle, gtle, gscore, max_off;
};

struct Tally {
  long long cells, rows, calls;
};

constexpr int NEG = -(1 << 29);

// ----------------------------------------------------------- ksw_extend2
// One ksw_extend2 call (bwa/ksw.c:380-479) on a group of G lanes.
//   query column j = qp[qa + qd*j]  (qd = -1 walks the read leftwards)
//   tb             = LDS row buffer holding the target base of every row the
//                    call can reach (filled by the caller)
// Lane r owns columns [r*Cd, r*Cd+Cd), Cd = ceil((qlen+1)/G) <= C; column
// qlen is eh[qlen] of the reference.  Column loops run to the wave-uniform
// CdW = max Cd over the wave's groups, so they branch on scalars.
template <int G, int C, bool T5>
__device__ __forceinline__ ExtOut extend_group(const DevOpt& o, int qlen, const uint8_t* __restrict__ qp, int qa,
                                            int qd, int tlen, const uint8_t* tb, int w, int end_bonus, int zdrop,
                                            int h0, Tally& tl) {
  using GR = Grp<G>;
  const int r = GR::lane();
  const int Cd = (qlen + G) / G;
  const int CdW = wave_umax<G>(Cd);
  const int jb = r * Cd;  // first column of this lane
  // hi / Cd as a multiply-shift: exact for hi < 1024, Cd <= 16
  const int cd_inv = (65536 + Cd - 1) / Cd;
  const int e_del = o.e_del, e_ins = o.e_ins, oe_del = o.oe_del, oe_ins = o.oe_ins;

  int hh[C], ee[C], jE[C], jm1E[C];
  uint32_t pf[C];
  uint32_t pf4[T5 ? C : 1];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    if (c < CdW) {
      const int j = jb + c;
      const int qb = (c < Cd && j < qlen) ? qp[qa + qd * j] : 0;
      const int8_t* m = o.mat;
      // query profile of this column for target bases 0..3 (4 x int8)
      pf[c] = (uint32_t)(uint8_t)m[qb] | (uint32_t)(uint8_t)m[5 + qb] << 8 |
              (uint32_t)(uint8_t)m[10 + qb] << 16 | (uint32_t)(uint8_t)m[15 + qb] << 24;
      if (T5) pf4[c] = (uint32_t)(uint8_t)m[20 + qb];
      // row -1 of eh[] (ksw.c:392-395): H(-1,-1)=h0, then an insertion gap
      const int v = j == 0 ? h0 : max(h0 - oe_ins - (j - 1) * e_ins, 0);
      hh[c] = (c < Cd && j <= qlen) ? v : 0;
      ee[c] = 0;
      // scan offsets: u_j = t_j + j*e_ins; columns past this lane's block never
      // contribute (NEG), F_j = max_{k<j} u_k - (j-1)*e_ins
      jE[c] = c < Cd ? j * e_ins : NEG;
      jm1E[c] = (j - 1) * e_ins;
    }
  }
  {  // band clamp (ksw.c:399-407)
    const int mi = band_cap(qlen, o.max_mat, end_bonus, o.o_ins, e_ins);
    const int md = band_cap(qlen, o.max_mat, end_bonus, o.o_del, e_del);
    w = min(w, min(mi, md));
  }

  int best = h0, bi = -1, bj = -1, ei = -1, esc = -1, off = 0, lo = 0, hi = qlen;
  int cells = 0, rows = 0;
  int tnext = tlen > 0 ? tb[0] : 0;
  for (int i = 0; i < tlen; ++i) {
    const int t = tnext;
    tnext = tb[i + 1];  // prefetch (the buffer is 2 rows longer than any call reads)
    lo = max(lo, i - w);
    hi = min(min(hi, i + w + 1), qlen);
    const int left0 = lo == 0 ? max(h0 - (o.o_del + e_del * (i + 1)), 0) : 0;
    const int sh = (t & 3) << 3;
    // this lane's in-band columns: clo <= c < chi; cend = the column of eh[hi]
    const int clo = max(lo - jb, 0), chi = min(hi - jb, Cd), cend = hi - jb;
    const bool empty = hi <= lo;

    // pass 1: M = H(i-1,j-1)+S (0 if H(i-1,j-1)==0), u = t + j*e_ins for the F scan
    int M[C], U[C];
    int run = NEG;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (c < CdW) {
        int sc;
        if (T5 && t == 4) sc = (int)(int8_t)(pf4[c] & 0xff);
        else sc = __builtin_amdgcn_sbfe((int)pf[c], sh, 8);
        const int m = hh[c] ? hh[c] + sc : 0;
        M[c] = m;
        const bool inb = c >= clo && c < chi;
        const int u = (inb ? max(m - oe_ins, 0) : 0) + jE[c];
        U[c] = u;
        run = max(run, u);
      }
    }
    // F(i,j) = max_{k<j} u_k - (j-1)*e_ins  (the reference's f recurrence, ksw.c:444-447;
    // at j == 0 it comes out negative, which max(M, E>=0, F) ignores exactly like F=0)
    int run2 = GR::excl_max(run, NEG);

    // pass 2: H, E, row max key; next-row state of each column (ksw.c:429,449):
    //   in band:  eh[j] <- {H(i,j-1) (first-column value at j == lo), E(i+1,j)}
    //   j == hi:  eh[hi] <- {H(i,hi-1) (first-column value if the band is empty), 0}
    int prevH = 0, lastH = 0, rkey = 0, en0 = 0, hcol = 0;
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (c < CdW) {
        const int j = jb + c;
        const bool inb = c >= clo && c < chi;
        const int f = run2 - jm1E[c];
        run2 = max(run2, U[c]);
        const int h = max(max(M[c], ee[c]), f);
        const int en = max(max(ee[c] - e_del, M[c] - oe_del), 0);
        rkey = max(rkey, inb ? ((h << 10) | j) : 0);
        if (c == 0) {
          en0 = en;
        } else {
          const bool isend = c == cend;
          const int hnew = (j == lo || (isend && empty)) ? left0 : prevH;
          hh[c] = (inb || isend) ? hnew : hh[c];
          ee[c] = inb ? en : (isend ? 0 : ee[c]);
          hcol = isend ? hh[c] : hcol;
        }
        prevH = h;
        lastH = c == Cd - 1 ? h : lastH;
      }
    }
    {  // column 0 of the lane takes the previous lane's last H
      const int hl = GR::up1(lastH);
      const bool inb = 0 >= clo && 0 < chi;
      const bool isend = cend == 0;
      const int hnew = (jb == lo || (isend && empty)) ? left0 : hl;
      hh[0] = (inb || isend) ? hnew : hh[0];
      ee[0] = inb ? en0 : (isend ? 0 : ee[0]);
      hcol = isend ? hh[0] : hcol;
    }
    rkey = GR::gmax(rkey);
    rows += 1;
    cells += empty ? 0 : hi - lo;
    const int mrow = rkey >> 10, mj = rkey & 1023;
    {  // ksw.c:450-453; h1 now sits in eh[hi]
      const bool endrow = max(lo, hi) == qlen;
      const int h1 = GR::bcast(hcol, (hi * cd_inv) >> 16);  // owner lane of column hi
      ei = (endrow && !(esc > h1)) ? i : ei;
      esc = endrow ? max(esc, h1) : esc;
    }
    if (mrow == 0) break;
    const bool better = mrow > best;
    {
      const int di = i - bi, dj = mj - bj;
      const int drop = di > dj ? best - mrow - (di - dj) * e_del : best - mrow - (dj - di) * e_ins;
      if (!better && zdrop > 0 && drop > zdrop) break;
    }
    off = better ? max(off, abs(mj - i)) : off;
    bi = better ? i : bi;
    bj = better ? mj : bj;
    best = better ? mrow : best;
    // zero-trim the band (ksw.c:466-469): first non-zero column in [lo,hi),
    // last non-zero column in [lo,hi]
    uint32_t nzb = 0;
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (c < CdW) nzb |= (uint32_t)min((uint32_t)(hh[c] | ee[c]), 1u) << c;
    const int cincl = min(cend + 1, Cd);
    const uint32_t mlo = clo >= 32 ? 0u : ~0u << clo;
    const uint32_t mhi = chi <= 0 ? 0u : (chi >= 32 ? ~0u : (1u << chi) - 1u);
    const uint32_t mhi2 = cincl <= 0 ? 0u : (cincl >= 32 ? ~0u : (1u << cincl) - 1u);
    const uint32_t bf = nzb & mlo & mhi, bl = nzb & mlo & mhi2;
    int nzf = bf ? jb + __builtin_ctz(bf) : INT_MAX;
    int nzl = bl ? jb + 31 - __builtin_clz(bl) : -1;
    nzf = GR::gmin(nzf);
    nzl = GR::gmax(nzl);
    const int nlo = nzf == INT_MAX ? hi : nzf;
    const int jl = nzl >= 0 ? nzl : nlo - 1;
    lo = nlo;
    hi = min(jl + 2, qlen);
  }
  tl.cells += cells;
  tl.rows += rows;
  tl.calls += 1;
  return ExtOut{best, bj + 1, bi + 1, ei + 1, esc, off};
}

// rows that extend_group can read for (qlen, w, end_bonus)
__device__ __forceinline__ int rows_needed(const DevOpt& o, int qlen, int tlen, int w, int end_bonus) {
  int mi = band_cap(qlen, o.max_mat, end_bonus, o.o_ins, o.e_ins);
  int md = band_cap(qlen, o.max_mat, end_bonus, o.o_del, o.e_del);
  int we = min(w, min(mi, md));
  return min(tlen, qlen + we + 1);
}

template <int G>
__device__ __forceinline__ void fill_target(uint8_t* tb, const DevRef& ref, int64_t x0, int dir, int n) {
  const int r = Grp<G>::lane();
  for (int k = r; k < n; k += G) tb[k] = (uint8_t)pac_base2(ref.pac, ref.l_pac, x0 + (int64_t)dir * k);
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
                                                         uint64_t* srt, int64_t* stats) {
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
}

// ------------------------------------------------------------ read order
// Each read gets a sort key: [variant | shape], variant = narrowest kernel
// whose G*C covers the read, shape = (left, right) query lengths of the first
// chain's top seed — the first extension mem_chain2aln performs.  Sorting by it
// puts reads whose DP tasks have similar row counts and column widths into the
// same wave (a wave runs as long as its slowest group).  Reads without chains
// sort last.  Per-variant counts are appended with wave-aggregated atomics.
__global__ void __launch_bounds__(256) read_keys_kernel(DevBatch b, uint32_t* keys, int32_t* vals, int32_t* counts,
                                                        int64_t* stats) {
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  int v = -1;
  if (rd < b.n_reads) {
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    for (int k = kNumVariants - 1; k >= 0; --k)
      if (lq <= kVariants[k].G * kVariants[k].C) v = k;
    uint32_t shape = 0x3fff;
    const int c0 = b.read_chain_off[rd], c1 = b.read_chain_off[rd + 1];
    for (int c = c0; c < c1; ++c) {
      const int s0 = b.chain_seed_off[c], s1 = b.chain_seed_off[c + 1];
      if (s1 == s0) continue;
      int best = s0;
      for (int k = s0 + 1; k < s1; ++k)
        if (b.seeds[k].score >= b.seeds[best].score) best = k;
      const bwagpu_seed_t t = b.seeds[best];
      const int left = min(t.qbeg, 1023) >> 3, right = min(lq - t.qbeg - t.len, 1023) >> 3;
      shape = (uint32_t)(left << 7 | right);
      break;
    }
    if (v < 0) {
      atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_LEN);
      v = kNumVariants - 1;
    }
    keys[rd] = (uint32_t)v << 14 | shape;
    vals[rd] = rd;
  }
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < kNumVariants; ++k) {
    const unsigned long long m = __ballot(v == k);
    if (m != 0 && lane == __ffsll((long long)m) - 1) atomicAdd(&counts[k], __popcll(m));
  }
}

hipError_t launch_read_keys(const DevBatch& b, uint32_t* keys, int32_t* vals, int32_t* counts, int64_t* stats,
                            hipStream_t st) {
  if (b.n_reads == 0) return hipSuccess;
  hipLaunchKernelGGL(read_keys_kernel, dim3((b.n_reads + 255) / 256), dim3(256), 0, st, b, keys, vals, counts, stats);
  return hipGetLastError();
}

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
  constexpr int GPB = kBlock / G;
  const int gib = threadIdx.x / G;
  const int r = GR::lane();
  int base = 0;
  for (int v = 0; v < variant; ++v) base += counts[v];
  const int n_list = counts[variant];
  Tally tl{0, 0, 0};
  uint8_t* tb = lds + gib * tb_bytes;

  for (int li = blockIdx.x * GPB + gib; li < n_list; li += gridDim.x * GPB) {
    const int rd = read_list[base + li];
    const int64_t qoff = b.seq_off[rd];
    const int lq = (int)(b.seq_off[rd + 1] - qoff);
    const uint8_t* q = b.seq + qoff;
    const int c0 = b.read_chain_off[rd], c1 = b.read_chain_off[rd + 1];
    bwagpu_alnreg_t* av = out + b.chain_seed_off[c0];
    int nreg = 0;
    for (int c = c0; c < c1; ++c) {
      const int s0 = b.chain_seed_off[c], ns = b.chain_seed_off[c + 1] - s0;
      if (ns == 0) continue;
      const ChainWin cw = win[c];
      if (cw.hi < cw.lo) continue;  // flagged by prep (reference would assert)
      const int rid = b.chain_rid[c];
      const float frac_rep = b.chain_frac_rep[c];
      uint64_t* key = srt + s0;
      const bwagpu_seed_t* sd = b.seeds + s0;
      for (int k = ns - 1; k >= 0; --k) {
        mem_fence_group();
        const uint64_t kk = __hip_atomic_load(&key[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const bwagpu_seed_t s = sd[(uint32_t)kk];
        // containment test against the read's regions so far (bwamem.c:678-697)
        int hit = INT_MAX;
        for (int base = 0; base < nreg && hit == INT_MAX; base += G) {
          const int i = base + r;
          bool p = false;
          if (i < nreg) {
            const bwagpu_alnreg_t* pr = &av[i];
            const int64_t prb = __hip_atomic_load(&pr->rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int64_t pre = __hip_atomic_load(&pr->re, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int pqb = __hip_atomic_load(&pr->qb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int pqe = __hip_atomic_load(&pr->qe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int pw = __hip_atomic_load(&pr->w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const int psl = __hip_atomic_load(&pr->seedlen0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (!(s.rbeg < prb || s.rbeg + s.len > pre || s.qbeg < pqb || s.qbeg + s.len > pqe) &&
                !(s.len - psl > .1 * lq)) {
              int qd = s.qbeg - pqb;
              int64_t rd64 = s.rbeg - prb;
              int g = max_gap_len(o, qd < rd64 ? qd : (int)rd64);
              int bw = g < pw ? g : pw;
              if (qd - rd64 < bw && rd64 - qd < bw) p = true;
              else {
                qd = pqe - (s.qbeg + s.len);
                rd64 = pre - (s.rbeg + s.len);
                g = max_gap_len(o, qd < rd64 ? qd : (int)rd64);
                bw = g < pw ? g : pw;
                if (qd - rd64 < bw && rd64 - qd < bw) p = true;
              }
            }
          }
          hit = GR::gmin(p ? i : INT_MAX);
        }
        if (hit != INT_MAX) {
          // overlapping-seed check among seeds already visited (bwamem.c:698-707)
          int ov = INT_MAX;
          for (int base = k + 1; base < ns && ov == INT_MAX; base += G) {
            const int i = base + r;
            bool p = false;
            if (i < ns) {
              const uint64_t ki = __hip_atomic_load(&key[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              if (ki != 0) {
                const bwagpu_seed_t t = sd[(uint32_t)ki];
                if (!(t.len < s.len * .95)) {
                  if (s.qbeg <= t.qbeg && s.qbeg + s.len - t.qbeg >= s.len >> 2 &&
                      (int64_t)(t.qbeg - s.qbeg) != t.rbeg - s.rbeg)
                    p = true;
                  else if (t.qbeg <= s.qbeg && t.qbeg + t.len - s.qbeg >= s.len >> 2 &&
                           (int64_t)(s.qbeg - t.qbeg) != s.rbeg - t.rbeg)
                    p = true;
                }
              }
            }
            ov = GR::gmin(p ? i : INT_MAX);
          }
          if (ov == INT_MAX) {  // skip; mark like srt[k] = 0 (bwamem.c:709)
            if (r == 0) __hip_atomic_store(&key[k], (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
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
            x = extend_group<G, C, false>(o, qlen, q, qa, dir, tlen, tb, aw[side], eb, o.zdrop, h0, tl);
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
        for (int i = r; i < ns; i += G) {
          const bwagpu_seed_t t = sd[i];
          if (t.qbeg >= qb && t.qbeg + t.len <= qe && t.rbeg >= rb && t.rbeg + t.len <= re) cov += t.len;
        }
        cov = grp_sum64(cov, G);
        if (r == 0) {
          bwagpu_alnreg_t a;
          a.rb = rb;
          a.re = re;
          a.qb = qb;
          a.qe = qe;
          a.rid = rid;
          a.score = score;
          a.truesc = truesc;
          a.sub = a.alt_sc = a.csub = a.sub_n = 0;
          a.w = aw0 > aw1 ? aw0 : aw1;
          a.seedcov = (int)cov;
          a.secondary = a.secondary_all = 0;
          a.seedlen0 = s.len;
          a.n_comp_is_alt = 0;
          a.frac_rep = frac_rep;
          a.hash = 0;
          av[nreg] = a;
        }
        ++nreg;
        mem_fence_group();
      }
    }
    if (r == 0) out_n[rd] = nreg;
  }
  if (r != 0) tl = Tally{0, 0, 0};
  block_stats<G>(tl, stats);
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
      for (int i = r; i < nr; i += G) tb[i] = tp[i];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      x = extend_group<G, C, T5>(o, t.qlen, q, 0, 1, t.tlen, tb, t.w, t.end_bonus, t.zdrop, t.h0, tl);
    }
    if (r == 0) res[k] = bwagpu_ext_result_t{x.score, x.qle, x.tle, x.gtle, x.gscore, x.max_off};
    if (r != 0) tl = Tally{0, 0, 0};
  }
  block_stats<G>(tl, stats);
}

// ------------------------------------------------------------ launchers
hipError_t launch_chain_prep(const DevOpt& o, const DevRef& ref, const DevBatch& b, int64_t,
                             ChainWin* win, uint64_t* srt, int64_t* stats, hipStream_t st) {
  if (b.n_chains == 0) return hipSuccess;
  const int nb = (b.n_chains + 255) / 256;
  hipLaunchKernelGGL(chain_prep_kernel, dim3(nb), dim3(256), 0, st, o, ref, b, win, srt, stats);
  return hipGetLastError();
}

template <int G, int C>
static hipError_t launch_c2a_t(const DevOpt& o, const DevRef& ref, const DevBatch& b, const int32_t* list,
                               const int32_t* cnt, int variant, int32_t n, int tb, const ChainWin* win, uint64_t* srt,
                               bwagpu_alnreg_t* out, int32_t* out_n, int64_t* stats, hipStream_t st) {
  constexpr int GPB = kBlock / G;
  // grid-stride over the (device-side) list: the count is only known on the GPU
  const int nb = std::min((n + GPB - 1) / GPB, 2048);
  hipLaunchKernelGGL((chain2aln_kernel<G, C>), dim3(nb), dim3(kBlock), (size_t)GPB * tb, st, o, ref, b, list, cnt,
                     variant, tb, win, srt, out, out_n, stats);
  return hipGetLastError();
}

hipError_t launch_chain2aln(int variant, const DevOpt& o, const DevRef& ref, const DevBatch& b,
                            const int32_t* read_list, const int32_t* d_count, int32_t max_list, int tb_bytes,
                            const ChainWin* win, uint64_t* srt, bwagpu_alnreg_t* out, int32_t* out_n,
                            int64_t* stats, hipStream_t st) {
  if (max_list == 0) return hipSuccess;
  switch (variant) {
    case 0: return launch_c2a_t<16, 10>(o, ref, b, read_list, d_count, 0, max_list, tb_bytes, win, srt, out, out_n, stats, st);
    case 1: return launch_c2a_t<32, 8>(o, ref, b, read_list, d_count, 1, max_list, tb_bytes, win, srt, out, out_n, stats, st);
    case 2: return launch_c2a_t<64, 16>(o, ref, b, read_list, d_count, 2, max_list, tb_bytes, win, srt, out, out_n, stats, st);
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
    EXT_CASE(0, 16, 10)
    EXT_CASE(1, 32, 8)
    EXT_CASE(2, 64, 16)
  }
#undef EXT_CASE
  return hipErrorInvalidValue;
}

}  // namespace bwagpu
