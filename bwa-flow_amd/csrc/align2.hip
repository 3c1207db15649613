// align2.hip — MI355X (gfx950) batched ksw_align2: the local Smith-Waterman of
// bwa's mate rescue.
//
// Reference: ksw_align2 (bwa/ksw.c:337-357) over ksw_u8 (111-232) / ksw_i16
// (234-328), called by mem_matesw (bwa/bwamem_pair.c:150-151) once per
// (read, orientation) whose mate was not found in a consistent pair.
//
// One task per wave.  Columns are blocked over the wave (lane r holds query
// columns r*CD .. r*CD+CD-1); the target is walked row by row.  The reference's results depend on its striped SIMD layout
// (p = 16 lanes in u8, 8 in i16; lane k covers the column SEGMENT
// [k*slen, (k+1)*slen), slen = ceil(qlen/p), columns qlen..p*slen-1 are
// padding scoring 0), so the kernel computes exactly what that layout does:
//
//   first pass   h(c) = max(M(c), E(c), Fseg(c))  with Fseg the horizontal gap
//                restarted at every segment start, E(i+1) from h, row max of h
//                over all p*slen columns (padding included);
//   lazy F       H(c) = max(h(c), Ffull(c)), Ffull across segments.
//
// Both F's are one max-plus prefix scan each (F(c) = max(0, max_{c'<c}
// (T(c') - oe_ins - (c-c'-1)*e_ins)), T = max(M, E)); the segmented one adds
// BIG*segment to the scanned value so an earlier segment can never win.  The
// closed form equals the reference's lazy-F loop with its early exit whenever
// o_ins > 0 (oracle/ksw_align.c has the argument); o_ins == 0 is refused on
// the host (E_UNSUPPORTED).
//
// The row-maxima list the 2nd-best score is taken from (ksw.c:191-198) is
// streamed to a per-task global scratch region, one single-lane store per
// closed entry, and resolved by a wave reduction after the last row.
// The start (XSTART) is the reference's reverse pass: the same kernel body
// run again with reversed index maps, no copies.
//
// Integer VALU work throughout (no MFMA); per row ~17 VALU per column register
// plus ~25 for the row (three 64-lane scans, shifts, profile words).
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>

#include "align2.h"
#include "scan_asm.h"
#include "wave_ops.h"

namespace bwagpu {

const int kA2CD[kA2Buckets] = {1, 2, 3, 4, 6, 8, 12, 16};

namespace {

__device__ __forceinline__ int usat(int a, int b) {  // max(a - b, 0) for a, b >= 0 (v_sub_u32 clamp)
  return (int)__builtin_elementwise_sub_sat((unsigned)a, (unsigned)b);
}

__device__ __forceinline__ int wave_max(int v) {
  v = max_bc31(max_bc15(max_ror1(max_ror2(max_ror4(max_ror8(v))))));
  return __builtin_amdgcn_readlane(v, 63);
}
__device__ __forceinline__ int wave_min(int v) {
  v = min_bc31(min_bc15(min_ror1(min_ror2(min_ror4(min_ror8(v))))));
  return __builtin_amdgcn_readlane(v, 63);
}

struct PassOut {
  int score, te, qe, score2, te2;
};

__device__ __forceinline__ int med3_i32(int a, int hi) {  // clamp(a, 0, hi), hi >= 0
  int d;
  asm("v_med3_i32 %0, %1, 0, %2" : "=v"(d) : "v"(a), "v"(hi));
  return d;
}

// One striped pass (ksw_u8 when U8, ksw_i16 otherwise) over target rows
// [0, tlen).  Query column j is q[j] (qrev < 0) or q[qrev - j]; target row i
// is t[i], or t[trev - i] for i <= trev (the XSTART reverse pass, ksw.c:345-348).
//
// Columns are BLOCKED over the wave: lane r holds j = r*CD + c, c < CD.  Per
// row and column:
//   M = H(i-1, j-1) + S        (u8: clamp to [0, 255-shift] = adds/subs_epu8)
//   T = max(M, E)              X = T + j*e_ins        W = X + BIG*seg(j)
//   exclusive prefix maxima of X and W = in-lane running max + one 64-lane
//   scan of the lane totals (the row maximum rides along: rowmax_j h(j) =
//   rowmax_j T(j), since Fseg(j) < max_{j'<j} T(j') when o_ins > 0)
//   h = max(T, Fseg), Fseg = Wprefix - BIG*seg - oe_ins - (j-1)*e_ins, >= 0
//   E' = max(E - e_del, h - oe_del, 0)     H = max(h, Ffull), Ffull likewise from X
// H(i-1, j-1) is the lane's own previous register, or for c = 0 lane r-1's
// last one: one DPP shift per row.  Columns past p*slen are pinned to 0 by
// their constants (M <= 0, both F offsets "infinite"): nothing is masked.
template <int CD, bool U8>
__device__ __forceinline__ PassOut a2_pass(const A2Prof& P, const uint8_t* __restrict__ q, int qlen, int qrev,
                                           const uint8_t* __restrict__ t, int tlen, int trev, int minsc,
                                           int endsc, int2* __restrict__ bs, long long& rows_done,
                                           long long& cells_done) {
  const int r = (int)(threadIdx.x & 63);
  constexpr int p = U8 ? 16 : 8;
  constexpr int BIG = 1 << 26;  // > any T + j*e_ins (host checks), 16*BIG < 2^31
  constexpr int KINF = 0x7fffffff;
  const int slen = (qlen + p - 1) / p, ncol = slen * p;
  const int e_del = P.e_del, oe_del = P.oe_del, e_ins = P.e_ins, oe_ins = P.oe_ins;
  const int shift = P.shift;
  uint32_t sel[CD];
  int Xk[CD], Wk[CD], Ks[CD], Kf[CD], Mk[CD];
  int H[CD], E[CD], Hm[CD];
#pragma unroll
  for (int c = 0; c < CD; ++c) {
    const int j = r * CD + c;
    const bool valid = j < ncol;
    // v_perm selector: profile byte 0..4 = query base, 5 = padding (scores 0)
    const int code = j < qlen ? q[qrev < 0 ? j : qrev - j] : 5;
    sel[c] = 0x0c0c0c00u | (uint32_t)code;
    const int seg = slen ? min(j / slen, p) : 0;
    Xk[c] = j * e_ins;
    Wk[c] = BIG * seg;
    Kf[c] = valid ? oe_ins + (j - 1) * e_ins : KINF;  // o_ins > 0 keeps it >= 0
    Ks[c] = valid ? BIG * seg + oe_ins + (j - 1) * e_ins : KINF;
    Mk[c] = U8 ? (valid ? 255 - shift : 0) : (valid ? -128 : -BIG);
    H[c] = 0;
    E[c] = 0;
    Hm[c] = 0;
  }
  int gmax = 0, te = -1, nb = 0, bsc = 0, brow = 0;
  int rows = 0;
  auto tidx = [&](int i) { return i <= trev ? trev - i : i; };
  // target rows in windows of 64, one base per lane; the next window is
  // fetched while this one is processed and consumed only at the window
  // boundary, so no row waits on memory.  Per window each lane turns its base
  // into the row's two profile words; a row reads them with v_readlane.
  int tvn = r < tlen ? t[tidx(r)] : 0;
  for (int i0 = 0; i0 < tlen; i0 += 64) {
    const int tv = tvn;
    {
      const int k = i0 + 64 + r;
      tvn = k < tlen ? t[tidx(k)] : 0;
    }
    uint32_t lov = P.lo[0], hiv = P.hi[0];
#pragma unroll
    for (int b = 1; b < 5; ++b) {
      lov = tv == b ? P.lo[b] : lov;
      hiv = tv == b ? P.hi[b] : hiv;
    }
    const int iend = min(tlen - i0, 64);
    for (int ii = 0; ii < iend; ++ii) {
      const int i = i0 + ii;
      const uint32_t lo = __builtin_amdgcn_readlane(lov, ii), hi = __builtin_amdgcn_readlane(hiv, ii);
      int T[CD], Xl[CD], Wl[CD];
      // H(i-1, j-1) of c = 0: lane r-1's last column; lane 0 reads 0 (bound_ctrl)
      const int hd0 = __builtin_amdgcn_update_dpp(0, H[CD - 1], DPP_WAVE_SHR1, 0xF, 0xF, true);
      int R = 0;
#pragma unroll
      for (int c = 0; c < CD; ++c) {
        const int hd = c ? H[c - 1] : hd0;
        const int pv = (int)__builtin_amdgcn_perm(hi, lo, sel[c]);
        int m;
        if (U8) m = med3_i32(hd + pv - shift, Mk[c]);  // adds_epu8 + subs_epu8 (ksw.c:153-154)
        else m = hd + pv + Mk[c];                      // adds_epi16 (ksw.c:270); host bounds the scores
        T[c] = max(m, E[c]);
        const int x = T[c] + Xk[c], w = x + Wk[c];
        Xl[c] = c ? max(Xl[c - 1], x) : x;  // in-lane inclusive prefix maxima
        Wl[c] = c ? max(Wl[c - 1], w) : w;
        R = max(R, T[c]);
      }
      int sX = Xl[CD - 1], sW = Wl[CD - 1];
      scan_max3(sX, sW, R);
      const int rm = __builtin_amdgcn_readlane(R, 63);
      // maxima over the lanes before this one (lane 0: none -> 0, the identity)
      const int Xin = __builtin_amdgcn_update_dpp(0, sX, DPP_WAVE_SHR1, 0xF, 0xF, true);
      const int Win = __builtin_amdgcn_update_dpp(0, sW, DPP_WAVE_SHR1, 0xF, 0xF, true);
#pragma unroll
      for (int c = 0; c < CD; ++c) {
        const int px = c ? max(Xin, Xl[c - 1]) : Xin;
        const int pw = c ? max(Win, Wl[c - 1]) : Win;
        const int h = max(T[c], usat(pw, Ks[c]));  // first-pass H (segment-local F)
        E[c] = max(usat(E[c], e_del), usat(h, oe_del));
        H[c] = max(h, usat(px, Kf[c]));            // after the lazy-F loop
      }
      ++rows;
      if (rm >= minsc) {  // b[] of row maxima (ksw.c:191-198)
        if (nb == 0 || brow + 1 != i) {
          if (nb && r == 0) bs[nb - 1] = make_int2(bsc, brow);
          ++nb;
          bsc = rm;
          brow = i;
        } else if (bsc < rm) {
          bsc = rm;
          brow = i;
        }
      }
      if (rm > gmax) {  // ksw.c:199-204
        gmax = rm;
        te = i;
#pragma unroll
        for (int c = 0; c < CD; ++c) Hm[c] = H[c];
        if ((U8 && gmax + shift >= 255) || gmax >= endsc) goto rows_done_;
      }
    }
  }
rows_done_:
  rows_done += rows;
  cells_done += (long long)rows * qlen;
  PassOut o{};
  const bool sat = U8 && gmax + shift >= 255;
  o.score = sat ? 255 : gmax;
  o.te = te;
  o.qe = -1;
  o.score2 = -1;
  o.te2 = -1;
  if (sat) return o;
  if (ncol > 0) {  // qe: the smallest column holding the row's maximum (ksw.c:210-213)
    // columns past p*slen hold 0 and come after every real one: no masking
    int mx = 0;
#pragma unroll
    for (int c = 0; c < CD; ++c) mx = max(mx, Hm[c]);
    mx = wave_max(mx);
    int jm = INT_MAX;
#pragma unroll
    for (int c = CD - 1; c >= 0; --c) jm = Hm[c] == mx ? r * CD + c : jm;
    o.qe = wave_min(jm);
  }
  if (nb) {  // 2nd best outside [te-k, te+k] (ksw.c:215-225)
    if (r == 0) bs[nb - 1] = make_int2(bsc, brow);
    // this wave's own stores must be visible to its loads below (L1 is not
    // coherent with them): release + acquire at agent scope
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int k = (o.score + P.qmax - 1) / P.qmax;
    const int low = te - k, high = te + k;
    for (int base = 0; base < nb; base += 64) {
      const int idx = base + r;
      int s = -1, row = INT_MAX;
      if (idx < nb) {
        const int2 e = bs[idx];
        if (e.y < low || e.y > high) s = e.x, row = e.y;
      }
      const int bm = wave_max(s);
      if (bm > o.score2) {  // entries are in row order: the first maximum wins
        o.te2 = wave_min(s == bm ? row : INT_MAX);
        o.score2 = bm;
      }
    }
  }
  return o;
}

}  // namespace

template <int CD, bool U8>
__global__ __launch_bounds__(256) void align2_kernel(A2Args a, A2Prof P) {
  // tasks are claimed one at a time from the bin's cursor (the host orders
  // each list longest first): no static deal, no tail of unequal rounds
  const int n = __builtin_amdgcn_readfirstlane(*a.count);
  long long rows = 0, cells = 0;
  int calls = 0;
  for (;;) {
    int k = 0;
    if ((threadIdx.x & 63) == 0) k = atomicAdd(a.cursor, 1);
    k = __builtin_amdgcn_readfirstlane(k);
    if (k >= n) break;
    const int id = __builtin_amdgcn_readfirstlane(a.list[k]);
    const bwagpu_align2_task_t tk = a.tasks[id];
    const int64_t qoff = tk.qoff, toff = tk.toff;
    const int qlen = __builtin_amdgcn_readfirstlane(tk.qlen);
    const int tlen = __builtin_amdgcn_readfirstlane(tk.tlen);
    const int xtra = __builtin_amdgcn_readfirstlane(tk.xtra);
    const uint8_t* q = a.q + qoff;
    const uint8_t* t = a.t + toff;
    int2* bs = a.bscratch + a.boff[id];
    const bool subo = (xtra & BWAGPU_KSW_XSUBO) != 0;
    const int minsc = subo ? (xtra & 0xffff) : 0x10000;
    const int endsc = (xtra & BWAGPU_KSW_XSTOP) ? (xtra & 0xffff) : 0x10000;
    PassOut r1 = a2_pass<CD, U8>(P, q, qlen, -1, t, tlen, -1, minsc, endsc, bs, rows, cells);
    ++calls;
    int tb = -1, qb = -1;
    if ((xtra & BWAGPU_KSW_XSTART) && !(subo && r1.score < (xtra & 0xffff))) {
      // ksw.c:345-355: reversed query [0, qe] against the target with its
      // first te+1 bases reversed, stop at the score
      PassOut r2;
      if (r1.qe + 1 > 0) {
        r2 = a2_pass<CD, U8>(P, q, r1.qe + 1, r1.qe, t, tlen, r1.te, 0x10000, r1.score & 0xffff, bs, rows,
                             cells);
        ++calls;
      } else {  // an empty query scores 0 everywhere: no rows needed
        r2 = PassOut{0, -1, -1, -1, -1};
      }
      if (r1.score == r2.score) tb = r1.te - r2.te, qb = r1.qe - r2.qe;
    }
    if ((threadIdx.x & 63) == 0) {
      bwagpu_kswr_t& o = a.out[id];
      o.score = r1.score;
      o.te = r1.te;
      o.qe = r1.qe;
      o.score2 = r1.score2;
      o.te2 = r1.te2;
      o.tb = tb;
      o.qb = qb;
    }
  }
  if (a.stats && (threadIdx.x & 63) == 0 && calls) {
    atomicAdd((unsigned long long*)&a.stats[ST_CELLS], (unsigned long long)cells);
    atomicAdd((unsigned long long*)&a.stats[ST_ROWS], (unsigned long long)rows);
    atomicAdd((unsigned long long*)&a.stats[ST_CALLS], (unsigned long long)calls);
  }
}

// Device-side binning for bwagpu_align2_device: bucket of the first pass's
// segment count and width, scratch region from a cursor; wave-aggregated
// atomics (one per distinct bin per wave).
__global__ __launch_bounds__(256) void align2_bin_kernel(const bwagpu_align2_task_t* __restrict__ tasks, int n,
                                                         int32_t* __restrict__ lists, int32_t* __restrict__ counts,
                                                         int64_t* __restrict__ boff, unsigned long long* cursor,
                                                         bwagpu_kswr_t* __restrict__ out, int64_t* stats) {
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int lane = (int)(threadIdx.x & 63);
  bool live = k < n;
  int bin = -1;
  long long need = 0;
  if (live) {
    const bwagpu_align2_task_t t = tasks[k];
    if (t.qlen < 0 || t.qlen > BWAGPU_MAX_READ_LEN || t.tlen < 0) {
      out[k] = bwagpu_kswr_t{-1, -1, -1, -1, -1, -1, -1};
      atomicOr((unsigned long long*)&stats[ST_ERR], (unsigned long long)ERR_LEN);
      live = false;
    } else {
      bin = a2_bin_of(t.qlen, (t.xtra & BWAGPU_KSW_XBYTE) != 0);
      need = (long long)t.tlen + 1;
    }
  }
  // scratch: one atomic per wave
  long long incl = need;
  for (int o = 1; o < 64; o <<= 1) {
    const long long v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  const long long total = __shfl(incl, 63, 64);
  unsigned long long base = 0;
  if (lane == 63 && total) base = atomicAdd(cursor, (unsigned long long)total);
  base = __shfl(base, 63, 64);
  if (live) boff[k] = (int64_t)(base + (unsigned long long)(incl - need));
  // bins: one atomic per distinct bin in the wave
  unsigned long long todo = __builtin_amdgcn_ballot_w64(live);
  while (todo) {
    const int leader = __builtin_ctzll(todo);
    const int b = __shfl(bin, leader, 64);
    const unsigned long long m = __builtin_amdgcn_ballot_w64(live && bin == b);
    int pos0 = 0;
    if (lane == leader) pos0 = atomicAdd(&counts[b], __builtin_popcountll(m));
    pos0 = __shfl(pos0, leader, 64);
    if (live && bin == b) lists[(int64_t)b * n + pos0 + __builtin_popcountll(m & ((1ull << lane) - 1))] = k;
    todo &= ~m;
  }
}

namespace {
template <int CD, bool U8>
hipError_t launch_one(const A2Args& a, const A2Prof& P, int n_hint, hipStream_t st) {
  // no dynamic LDS, so the resident grid depends on the kernel alone; a
  // function-local static initialiser runs once even with several worker threads
  static const int cap = [] {
    int per_cu = 0, dev = 0, ncu = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, align2_kernel<CD, U8>, 256, 0);
    return std::max(1, per_cu) * std::max(1, ncu);
  }();
  const int want = n_hint > 0 ? (n_hint + 3) / 4 : cap;
  const int grid = std::max(1, std::min(want, cap));
  hipLaunchKernelGGL((align2_kernel<CD, U8>), dim3(grid), dim3(256), 0, st, a, P);
  return hipGetLastError();
}

template <bool U8>
hipError_t launch_bucket(int bucket, const A2Args& a, const A2Prof& P, int n_hint, hipStream_t st) {
  switch (bucket) {
    case 0: return launch_one<1, U8>(a, P, n_hint, st);
    case 1: return launch_one<2, U8>(a, P, n_hint, st);
    case 2: return launch_one<3, U8>(a, P, n_hint, st);
    case 3: return launch_one<4, U8>(a, P, n_hint, st);
    case 4: return launch_one<6, U8>(a, P, n_hint, st);
    case 5: return launch_one<8, U8>(a, P, n_hint, st);
    case 6: return launch_one<12, U8>(a, P, n_hint, st);
    default: return launch_one<16, U8>(a, P, n_hint, st);
  }
}
}  // namespace

hipError_t launch_align2(int bin, const A2Args& a, const A2Prof& P, int n_hint, hipStream_t st) {
  return bin >= kA2Buckets ? launch_bucket<true>(bin - kA2Buckets, a, P, n_hint, st)
                           : launch_bucket<false>(bin, a, P, n_hint, st);
}

hipError_t launch_align2_bins(const bwagpu_align2_task_t* tasks, int n, int32_t* lists, int32_t* counts,
                              int64_t* boff, unsigned long long* cursor, bwagpu_kswr_t* out, int64_t* stats,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(align2_bin_kernel, dim3((n + 255) / 256), dim3(256), 0, st, tasks, n, lists, counts, boff,
                     cursor, out, stats);
  return hipGetLastError();
}

}  // namespace bwagpu
