// spec.hip — the speculative mem_chain2aln (default path of
// bwagpu_chain2aln): extension task rounds on persistent grids
// (one, two or four ksw_extend2 calls per wave, ksw_dev.h) and the selection
// passes that replay bwa's sequential seed logic (bwamem.c:641-795) exactly
// over the precomputed extensions.
#include "ksw_dev.h"

namespace bwagpu {

// The selection and bookkeeping kernels are latency-bound chains that share
// CUs with the other caller stream's persistent extension kernel; at wave
// priority 3 their instructions issue ahead of its (priority 0) waves.
__device__ __forceinline__ void sel_prio() { __builtin_amdgcn_s_setprio(3); }

// per-read selection trace (bwagpu_debug_set_trace; this file's copy)
__device__ uint32_t* g_trace = nullptr;
hipError_t set_trace_spec(void* p) { return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &p, sizeof(p)); }

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

// lane per chain: window (bwamem.c:648-668 + bns_fetch_seq's clipping), the
// round-A task (the chain's first seed in processing order) and, for chains
// of up to kOrderLane seeds, the processing order; longer chains are listed
// for spec_order_kernel, which does their window and order one workgroup
// each (a lane looping over ~170 seeds was this kernel's tail).  chain_read
// comes from spec_reads_kernel.
__global__ void __launch_bounds__(256) spec_chain_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a) {
  sel_prio();
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
        task = lq <= a.lq_bound;
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
  sel_prio();
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  bool heavy = false;
  int ns = 0;
  if (rd < b.n_reads) {
    const int lq = (int)(b.seq_off[rd + 1] - b.seq_off[rd]);
    if (lq > a.lq_bound) atomicOr((unsigned long long*)&a.stats[ST_ERR], (unsigned long long)ERR_LEN);
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
  sel_prio();
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
template <int G = 32>
__device__ __forceinline__ void fill_two_half(uint8_t* tbl, int64_t x0l, int nl, uint8_t* tbr, int64_t x0r, int nr,
                                              const DevRef& ref) {
  const int r = (int)(threadIdx.x & (G - 1));
  const int64_t two1 = (ref.l_pac << 1) - 1;
  const int n = max(nl, nr);
  for (int base = 0; base < n; base += 4 * G) {
    uint32_t raw[8];
    int sh[8], kk[8];
    bool rev[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const bool left = m < 4;
      const int nn = left ? nl : nr;
      const int k = min(base + (m & 3) * G + r, max(nn - 1, 0));
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

// The same gather in ONE memory round trip (the packed kernels' task starts):
// lane r of the group takes rows [r R, r R + R) of each side, R = ceil(n / G)
// <= 32, i.e. a run of <= 32 consecutive bases of one strand, and loads the
// three aligned words of the pac that hold them (<= 9 bytes from a word
// boundary); each row's base is a 2-bit field of those words.  fill_two_half
// takes 4 rows per side per lane per pass, one dependent round trip per pass
// (5-6 for a 150 bp read's windows).  A run that leaves the pac's last 12
// bytes, or would straddle the two strands (a chain window never does), takes
// the per-row loads of fill_two_half's kind.
template <int G>
__device__ __forceinline__ void fill_side_run(uint8_t* tb, int64_t x0, int dir, int k0, int k1, const DevRef& ref,
                                              int64_t pac_bytes) {
  if (k1 <= k0) return;
  const int64_t two1 = (ref.l_pac << 1) - 1;
  const int64_t xa = x0 + (int64_t)dir * k0, xb = x0 + (int64_t)dir * (k1 - 1);
  const bool rev = xa >= ref.l_pac;
  const int64_t fa = rev ? two1 - xa : xa, fb = rev ? two1 - xb : xb;
  const int64_t fmin = fa < fb ? fa : fb;
  const int64_t w0 = (fmin >> 2) & ~(int64_t)3;  // first byte of the aligned words
  const bool fast = (xb >= ref.l_pac) == rev && fmin >= 0 && (fa > fb ? fa : fb) < ref.l_pac && w0 + 12 <= pac_bytes;
  const int df = (dir > 0) == !rev ? 1 : -1;  // f along the run
  if (fast) {
    const uint32_t* pw = reinterpret_cast<const uint32_t*>(ref.pac + w0);
    const uint32_t d0 = pw[0], d1 = pw[1], d2 = pw[2];
    const int o0 = (int)(fa - (w0 << 2));  // the first row's base offset in the 48 loaded bases
#pragma unroll
    for (int j = 0; j < 32; ++j) {
      if (k0 + j >= k1) break;
      const int o = o0 + df * j;
      const uint32_t w = o < 16 ? d0 : (o < 32 ? d1 : d2);
      const int bit = ((o >> 2) & 3) * 8 + 6 - 2 * (o & 3);
      const uint32_t bse = (w >> bit) & 3u;
      tb[k0 + j] = (uint8_t)(rev ? 3u - bse : bse);
    }
  } else {
    for (int k = k0; k < k1; ++k) {
      const int64_t x = x0 + (int64_t)dir * k;
      const bool rv = x >= ref.l_pac;
      int64_t f = rv ? two1 - x : x;
      f = f < 0 ? 0 : (f >= ref.l_pac ? ref.l_pac - 1 : f);
      const int bse = (ref.pac[f >> 2] >> ((~f & 3) << 1)) & 3;
      tb[k] = (uint8_t)(rv ? 3 - bse : bse);
    }
  }
}

template <int G>
__device__ __forceinline__ void fill_two_fast(uint8_t* tbl, int64_t x0l, int nl, uint8_t* tbr, int64_t x0r, int nr,
                                              const DevRef& ref) {
  const int n = max(nl, nr);
  const int R = (n + G - 1) / G;
  if (R > 32) {  // options with bands wider than the packed kernels' defaults
    fill_two_half<G>(tbl, x0l, nl, tbr, x0r, nr, ref);
    return;
  }
  const int r = (int)(threadIdx.x & (G - 1));
  const int64_t pac_bytes = (ref.l_pac >> 2) + 1;  // bwa.c:281-282
  const int k0 = r * R;
  fill_side_run<G>(tbl, x0l, -1, k0, min(k0 + R, nl), ref, pac_bytes);
  fill_side_run<G>(tbr, x0r, 1, k0, min(k0 + R, nr), ref, pac_bytes);
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

template <int G = 32>
__device__ __forceinline__ void store_ext_half(SeedExt* dst, const SeedExt& e) {
  static_assert(G >= 12, "a SeedExt is 12 words");
  const int d = (int)(threadIdx.x & (G - 1));
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
template <int G>
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
  fill_two_half<G>(tl, t.rbeg - 1, qlenL ? rows_needed(o, qlenL, (int)(t.rbeg - t.wlo), o.w << 1, o.pen_clip5) : 0, tr,
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

#ifdef BWAGPU_OCC_DIAG
// Occupancy of one extend_quad generation (a diagnostic build's counters,
// bwagpu_debug_occupancy): the wave runs rows until its longest call ends and
// CPL x G columns per call for its longest query; of those call-slot cells,
// the ones of calls that already ended, the ones beyond a live call's query,
// outside ksw's band, and the cells computed.  int64 counters at ctr words
// 32..47: generations, rows run, call-slot rows, live call rows, slot cells,
// live slot cells, query cells, computed cells.
template <int G>
__device__ __forceinline__ void occ_diag(unsigned long long* acc, const QCall& ca, const QCall& cb, const Tally32& ta,
                                         const Tally32& tb) {
  int qm = 0, rm = 0;
  long long lr = 0, lq = 0, cc = 0;
#pragma unroll
  for (int g = 0; g < 64; g += G) {
    const int qa = __builtin_amdgcn_readlane(ca.qlen, g), qb = __builtin_amdgcn_readlane(cb.qlen, g);
    const int ra = __builtin_amdgcn_readlane(ta.rows, g), rb = __builtin_amdgcn_readlane(tb.rows, g);
    qm = max(qm, max(qa, qb));
    rm = max(rm, max(ra, rb));
    lr += ra + rb;
    lq += (long long)ra * (qa + 1) + (long long)rb * (qb + 1);
    cc += __builtin_amdgcn_readlane(ta.cells, g) + __builtin_amdgcn_readlane(tb.cells, g);
  }
  const int cpl = (qm + G) / G;
  // summed per wave in registers, added to ctr words 32.. once at the kernel's end
  // (atomics here would put their round trips on the next generation start)
  acc[0] += 1ull;
  acc[1] += (unsigned long long)rm;
  acc[2] += (unsigned long long)rm * (2 * 64 / G);
  acc[3] += (unsigned long long)lr;
  acc[4] += (unsigned long long)rm * 128ull * cpl;
  acc[5] += (unsigned long long)lr * G * cpl;
  acc[6] += (unsigned long long)lq;
  acc[7] += (unsigned long long)cc;
}
#endif

// the same from the task's FatTask record (spec_sort_scatter)
template <int G>
__device__ __forceinline__ void qtask_start_fat(QTask& t, const DevOpt& o, const DevRef& ref, const FatTask& f,
                                                uint8_t* tl, uint8_t* tr) {
  t.pos = f.pos;
  t.rbeg = f.rbeg;
  t.wlo = f.rbeg - f.dlo;
  t.whi = f.rbeg + f.dhi;
  t.qoff = f.qoff;
  t.qbeg = (int)(f.qls & 1023u);
  t.len = (int)((f.qls >> 10) & 1023u);
  t.lq = (int)(f.qls >> 20);
  const int qlenL = t.qbeg, qlenR = t.lq - (t.qbeg + t.len);
  const int64_t x0R = t.rbeg + t.len;
  fill_two_fast<G>(tl, t.rbeg - 1, qlenL ? rows_needed(o, qlenL, f.dlo, o.w << 1, o.pen_clip5) : 0, tr, x0R,
                   qlenR ? rows_needed(o, qlenR, (int)(t.whi - x0R), o.w << 1, o.pen_clip3) : 0, ref);
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
  // rows past qlen + w + 1 have an empty band (ksw.c:415-419: m == 0 breaks
  // there), so the cap changes no result; it keeps tlen inside the packed
  // kernels' 16-bit row counters for chain windows of 32 kb and more
  q.tlen = rows_needed(o, q.qlen, q.tlen, q.w, q.eb);
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
// Not volatile: a volatile access makes the memory legalizer wait for every
// outstanding global access first (s_waitcnt vmcnt(0) at each qload / qpark:
// the SeedExt stores and the task loads of the other sub-slots, ~30 % of the
// waves' cycles outside the DP in the diagnostic build's clock split).  An
// empty asm with a memory clobber after the stores and before the loads keeps
// the state really parked in LDS (LLVM may not carry it in VGPRs across it).
typedef __attribute__((address_space(3))) QTask LdsQ;
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
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ QTask qload(LdsQ* p) {
  asm volatile("" ::: "memory");
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

// Extension tasks of one list (in pair order, spec_sort_*), two per G-lane
// group: four (G = 32) or eight (G = 16) per wave.
// PMAX = the bin's largest CPL: ceil(read length / G).
// Every sub-slot keeps its NEXT task's FatTask record in registers, claimed and
// loaded one generation ahead: the loads run while the current generation's
// DP runs (the row loop has no global memory operation), so a sub-slot whose
// task ends starts the next at once — only its target rows (fill_two_half)
// are fetched at the call boundary.  At one wave per SIMD nothing else hides a
// generation start's dependent loads (the claim, the task entry, its seed,
// window and read).
template <int G, int PMAX, bool K8>
__global__ void __launch_bounds__(kBlock) spec_ext4_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                           int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  // the groups' first lanes, and those below this lane's group
  constexpr uint64_t kLead = G == 16 ? 0x0001000100010001ull : 0x0000000100000001ull;
  const uint64_t below = kLead & ((1ull << ((int)threadIdx.x & (64 - G))) - 1);
  // per group: A left, A right, B left, B right target rows, then A's and B's task states
  uint8_t* const tal = lds + (size_t)(threadIdx.x / G) * (4 * (size_t)tb_bytes + 2 * kQTaskLds);
  uint8_t* const tar = tal + tb_bytes;
  uint8_t* const tbl = tar + tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  LdsQ* const qa = (LdsQ*)(tbr + tb_bytes);
  LdsQ* const qb = (LdsQ*)(tbr + tb_bytes + kQTaskLds);
  const int n = uni(__hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const FatTask* fl = a.ftask + spec_list_off(list, b.n_chains, b.n_seeds);
  ShardQ qq;
  qq.init(a.qh + 8 * kQHStride * list, n);
  // ha / hb: the sub-slot has a task (state parked in LDS); pa / pb: its next
  // task's record (fa / fb) is claimed and loaded (or in flight)
  bool ha = false, hb = false, pa = false, pb = false, more = n > 0;
  FatTask fa{}, fb{};
  long long spec_cells = 0;
  // claim-ahead while plenty of the list is left (a.ext_prefetch): near the
  // end, tasks held ahead by a busy wave would idle the others
  const int ahead_min = a.ext_prefetch * 8 * (int)((gridDim.x * (kBlock / 64) + 7) / 8);
  int rem = n;
#ifdef BWAGPU_OCC_DIAG
  unsigned long long tw[6] = {0, 0, 0, 0, 0, 0}, occ[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  for (;;) {
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
    // sub-slots without a task start their prefetched one
    if (!ha && pa) {
      QTask t;
      qtask_start_fat<G>(t, o, ref, fa, tal, tar);
      if (t.phase >= 4) store_ext_half<G>(a.ext + t.pos, qtask_ext(t));  // a whole-read seed (bwamem.c:753, 781)
      else qpark(qa, t);
      ha = t.phase < 4;
      pa = false;
    }
    if (!hb && pb) {
      QTask t;
      qtask_start_fat<G>(t, o, ref, fb, tbl, tbr);
      if (t.phase >= 4) store_ext_half<G>(a.ext + t.pos, qtask_ext(t));
      else qpark(qb, t);
      hb = t.phase < 4;
      pb = false;
    }
    if (more) {  // one claim for the wave: sub-slots without a next task (ahead) / without a task (on demand)
      const bool ahead = ahead_min > 0 && rem > ahead_min;
      const bool wa = ahead ? !pa : (!ha && !pa), wb = ahead ? !pb : (!hb && !pb);
      const uint64_t na = __builtin_amdgcn_ballot_w64(wa) & kLead, nb = __builtin_amdgcn_ballot_w64(wb) & kLead;
      const int nn = __popcll(na) + __popcll(nb);
      if (nn > 0) {
        int m0, cap;
#ifdef BWAGPU_OCC_DIAG
        const unsigned long long ca0 = __builtin_amdgcn_s_memtime();
#endif
        const bool got = qq.claim(nn, m0, cap);
#ifdef BWAGPU_OCC_DIAG
        const unsigned long long ca1 = __builtin_amdgcn_s_memtime();
        tw[4] += ca1 - ca0;
#endif
        if (got) {
          rem = (cap - m0 - nn) * 8;
          const int ia = m0 + __popcll(na & below) + __popcll(nb & below), ib = ia + (wa ? 1 : 0);
          if (wa && ia < cap) {
            fa = fl[qq.shard + 8 * ia];
            pa = true;
          }
          if (wb && ib < cap) {
            fb = fl[qq.shard + 8 * ib];
            pb = true;
          }
#ifdef BWAGPU_OCC_DIAG
          __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the task records, timed on their own
          tw[5] += __builtin_amdgcn_s_memtime() - ca1;
#endif
          if (!ahead) {  // on demand: start them now
            if (!ha && pa) {
              QTask t;
              qtask_start_fat<G>(t, o, ref, fa, tal, tar);
              if (t.phase >= 4) store_ext_half<G>(a.ext + t.pos, qtask_ext(t));
              else qpark(qa, t);
              ha = t.phase < 4;
              pa = false;
            }
            if (!hb && pb) {
              QTask t;
              qtask_start_fat<G>(t, o, ref, fb, tbl, tbr);
              if (t.phase >= 4) store_ext_half<G>(a.ext + t.pos, qtask_ext(t));
              else qpark(qb, t);
              hb = t.phase < 4;
              pb = false;
            }
          }
        } else {
          more = false;
        }
      }
    }
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    tw[0] += c1 - c0;
#endif
    if (!__builtin_amdgcn_ballot_w64(ha || hb)) {
      if (!more && !__builtin_amdgcn_ballot_w64(pa || pb)) break;
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
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c2 = __builtin_amdgcn_s_memtime();
    tw[1] += c2 - c1;
#endif
    extend_quad_dispatch<G, PMAX, K8>(o, ca, cb, xa, xb, ta, tb);
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c3 = __builtin_amdgcn_s_memtime();
    tw[2] += c3 - c2;
    occ_diag<G>(occ, ca, cb, ta, tb);
#endif
    if (ha) {
      QTask t = qload(qa);
      if (qtask_advance(t, o, xa, ta)) {
        store_ext_half<G>(a.ext + t.pos, qtask_ext(t));
        spec_cells += t.cells;
        ha = false;
      } else {
        qpark(qa, t);
      }
    }
    if (hb) {
      QTask t = qload(qb);
      if (qtask_advance(t, o, xb, tb)) {
        store_ext_half<G>(a.ext + t.pos, qtask_ext(t));
        spec_cells += t.cells;
        hb = false;
      } else {
        qpark(qb, t);
      }
    }
#ifdef BWAGPU_OCC_DIAG
    tw[3] += __builtin_amdgcn_s_memtime() - c3;
#endif
  }
  if ((threadIdx.x & (G - 1)) == 0 && spec_cells)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
#ifdef BWAGPU_OCC_DIAG
  // shader-clock cycles of the waves: task starts + claims, call setup, DP (extend_quad), result
  // advance; of the first, the claims' and the task records' own
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 32) + k, occ[k]);
    for (int k = 0; k < 6; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 48) + k, tw[k]);
  }
#endif
}

// LDS bytes of a spec_ext4_kernel workgroup
static size_t ext4_lds(int tb_bytes, int g) { return (size_t)(kBlock / g) * (4 * (size_t)tb_bytes + 2 * kQTaskLds); }

// Task order for the pair kernel: the two seeds a wave takes should need the
// same phases for about as long — a half whose seed has no left side, or a
// much shorter one, idles while the other runs (EXEC).  A counting sort of
// the first two bins' lists of a round by key = (the longer side's qlen / 8,
// the shorter's / 8) — with calls of left and right phases mixed in one row
// loop, the longer side sets the columns run (by (left, right): 37.8 against
// 38.1-38.2 Mreads/s with eight per wave):
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
  // descending: the longest tasks first, so the grid's tail is short ones
  const int hi = max(ql, qr), lo = min(ql, qr);
  return (kSortKeys - 1) - ((hi >> 3) << 5 | (lo >> 3));
}

// the task's FatTask record (engine.h): its seed, its chain's window, its read
__device__ __forceinline__ FatTask fat_task(const DevBatch& b, const SpecArgs& a, int2 tk) {
  const bwagpu_seed_t sd = a.prog[tk.x];
  const ChainWin cw = a.win[tk.y];
  const int rd = a.chain_read[tk.y];
  FatTask f;
  f.rbeg = sd.rbeg;
  f.qoff = b.seq_off[rd];
  f.pos = tk.x;
  f.dlo = (int32_t)(sd.rbeg - cw.lo);
  f.dhi = (int32_t)(cw.hi - sd.rbeg);
  const int lq = (int)(b.seq_off[rd + 1] - f.qoff);
  f.qls = (uint32_t)sd.qbeg | (uint32_t)sd.len << 10 | (uint32_t)lq << 20;
  return f;
}

__global__ void __launch_bounds__(256) spec_sort_count(DevBatch b, SpecArgs a, int round, int bin0) {
  sel_prio();
  __shared__ int hist[kSortKeys];
  const int bin = bin0 + (int)blockIdx.y;
  const int list = round * kSpecBins + bin;
  int32_t* gh = a.sorth + (round * 2 + bin) * kSortKeys;
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

__global__ void __launch_bounds__(256) spec_sort_scan(SpecArgs a, int round, int bin0) {
  sel_prio();
  __shared__ int part[256];
  int32_t* gh = a.sorth + (round * 2 + bin0 + (int)blockIdx.x) * kSortKeys;
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

__global__ void __launch_bounds__(256) spec_sort_scatter(DevBatch b, SpecArgs a, int round, int bin0) {
  sel_prio();
  __shared__ int cnt[kSortKeys];
  const int bin = bin0 + (int)blockIdx.y;
  const int list = round * kSpecBins + bin;
  int32_t* gh = a.sorth + (round * 2 + bin) * kSortKeys;
  for (int k = threadIdx.x; k < kSortKeys; k += 256) cnt[k] = 0;
  __syncthreads();
  const int n = __hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const size_t off = spec_list_off(list, b.n_chains, b.n_seeds);
  const int2* tl = a.tasks + off;
  int2* out = a.stasks + off;
  FatTask* fout = a.ftask + off;
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
      if (keys[m] >= 0) {
        const int at = cnt[keys[m]] + rank[m];
        out[at] = tk[m];
        fout[at] = fat_task(b, a, tk[m]);
      }
    __syncthreads();
    for (int k = threadIdx.x; k < kSortKeys; k += 256) cnt[k] = 0;
    __syncthreads();
  }
}

// ---------------------------------------------- phased extension (round 6)
// The extension tasks of the first two length bins run as two launches per
// round: every task's LEFT call(s) (ksw_extend2 with the band retry,
// bwamem.c:717-751), then every task's RIGHT call(s) (752-792, h0 = the left
// score).  Each launch takes calls in the order of their own query length
// (longest first), so the eight calls of a wave have about the same length:
// with a task's left and right calls in one wave generation after another
// (spec_ext4_kernel), a wave ran until its longest call ended while shorter
// ones had ended (25 % of its call-slot cells) and set its columns by its
// longest query (10 %), tools_dev/occ_diag.py.  Lists: the tasks with a left
// side (FatTask, key = left query length) and those with a right side; a
// whole-read seed (neither side) is written by the scatter itself.
__device__ __forceinline__ int side_key(int qlen) { return 255 - min(qlen, 255); }  // descending

__global__ void __launch_bounds__(256) spec_sort2_count(DevBatch b, SpecArgs a, int round, int bin0) {
  sel_prio();
  __shared__ int hist[2][256];
  __shared__ int tot[2];
  const int bin = bin0 + (int)blockIdx.y;
  const int list = round * kSpecBins + bin;
  int32_t* ghL = a.sorth + (round * 2 + bin) * kSortKeys;
  int32_t* ghR = ghL + kSortWordsR;
  for (int k = threadIdx.x; k < 2 * 256; k += 256) hist[k >> 8][k & 255] = 0;
  if (threadIdx.x < 2) tot[threadIdx.x] = 0;
  __syncthreads();
  const int n = __hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int2* tl = a.tasks + spec_list_off(list, b.n_chains, b.n_seeds);
  const int chunk = (n + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  for (int i = i0 + (int)threadIdx.x; i < i1; i += 256) {
    const FatTask f = fat_task(b, a, tl[i]);
    const int qb = (int)(f.qls & 1023u), ln = (int)((f.qls >> 10) & 1023u), lq = (int)(f.qls >> 20);
    const int qr = lq - qb - ln;
    if (qb > 0) atomicAdd(&hist[0][side_key(qb)], 1);
    if (qr > 0) atomicAdd(&hist[1][side_key(qr)], 1);
  }
  __syncthreads();
  for (int k = threadIdx.x; k < 2 * 256; k += 256) {
    const int c = hist[k >> 8][k & 255];
    if (c) {
      atomicAdd((k >> 8) ? &ghR[k & 255] : &ghL[k & 255], c);
      atomicAdd(&tot[k >> 8], c);
    }
  }
  __syncthreads();
  if (threadIdx.x < 2 && tot[threadIdx.x])
    atomicAdd(&a.ctr[(threadIdx.x ? SPC_RCNT : SPC_LCNT) + list], tot[threadIdx.x]);
}

// exclusive scan of the 256 keys of each (side, bin) histogram: one block each
// (bins bin0 .. bin0 + nbins - 1)
__global__ void __launch_bounds__(256) spec_sort2_scan(SpecArgs a, int round, int bin0, int nbins) {
  sel_prio();
  __shared__ int part[256];
  const int bin = bin0 + (int)blockIdx.x % nbins, side = (int)blockIdx.x / nbins;
  int32_t* gh = a.sorth + (round * 2 + bin) * kSortKeys + side * kSortWordsR;
  const int t = (int)threadIdx.x;
  const int v = gh[t];
  part[t] = v;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const int x = t >= o ? part[t - o] : 0;
    __syncthreads();
    part[t] += x;
    __syncthreads();
  }
  gh[t] = part[t] - v;  // the key's first position (a cursor from here on)
}

__global__ void __launch_bounds__(256) spec_sort2_scatter(DevOpt o, DevBatch b, SpecArgs a, int round, int bin0) {
  sel_prio();
  __shared__ int cnt[2][256];
  const int bin = bin0 + (int)blockIdx.y;
  const int list = round * kSpecBins + bin;
  int32_t* ghL = a.sorth + (round * 2 + bin) * kSortKeys;
  int32_t* ghR = ghL + kSortWordsR;
  for (int k = threadIdx.x; k < 2 * 256; k += 256) cnt[k >> 8][k & 255] = 0;
  __syncthreads();
  const int n = __hip_atomic_load(&a.ctr[SPC_CNT + list], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const size_t off = spec_list_off(list, b.n_chains, b.n_seeds);
  const int2* tl = a.tasks + off;
  FatTask* foL = a.ftask + off;
  FatTask* foR = a.ftaskR + off;
  const int chunk = (n + (int)gridDim.x - 1) / (int)gridDim.x;
  const int i0 = (int)blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  constexpr int kPer = 8;  // entries per thread held across the barrier
  int kl[kPer], kr[kPer], rl[kPer], rr[kPer];
  FatTask ft[kPer];
  for (int base = i0; base < i1; base += 256 * kPer) {
#pragma unroll
    for (int m = 0; m < kPer; ++m) {
      const int i = base + m * 256 + (int)threadIdx.x;
      kl[m] = kr[m] = -1;
      if (i < i1) {
        ft[m] = fat_task(b, a, tl[i]);
        const int qb = (int)(ft[m].qls & 1023u), ln = (int)((ft[m].qls >> 10) & 1023u), lq = (int)(ft[m].qls >> 20);
        const int qr = lq - qb - ln;
        if (qb > 0) {
          kl[m] = side_key(qb);
          rl[m] = atomicAdd(&cnt[0][kl[m]], 1);
        }
        if (qr > 0) {
          kr[m] = side_key(qr);
          rr[m] = atomicAdd(&cnt[1][kr[m]], 1);
        }
        if (qb == 0 && qr == 0) {  // a whole-read seed (bwamem.c:753, 781): no ksw_extend2 call
          SeedExt e;
          e.rb = ft[m].rbeg;
          e.re = ft[m].rbeg + ln;
          e.qb = 0;
          e.qe = lq;
          e.score = e.truesc = ln * o.a;
          e.w = o.w;
          e.cells = e.rows = 0;
          e.calls = 1;
          a.ext[ft[m].pos] = e;
        }
      }
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * 256; k += 256) {
      const int c = cnt[k >> 8][k & 255];
      cnt[k >> 8][k & 255] = c ? atomicAdd((k >> 8) ? &ghR[k & 255] : &ghL[k & 255], c) : 0;  // this pass's range
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kPer; ++m) {
      if (kl[m] >= 0) foL[cnt[0][kl[m]] + rl[m]] = ft[m];
      if (kr[m] >= 0) foR[cnt[1][kr[m]] + rr[m]] = ft[m];
    }
    __syncthreads();
    for (int k = threadIdx.x; k < 2 * 256; k += 256) cnt[k >> 8][k & 255] = 0;
    __syncthreads();
  }
}

// One side of a task in flight (LDS, per sub-slot, between its calls).
struct SideTask {
  int64_t rbeg, qoff, rb;
  int32_t pos, dlo, dhi, qbeg, len, lq;
  int32_t tt, score, h0, truesc, qb, aw0, cells, rows, calls, pad_;
};
static_assert(sizeof(SideTask) <= 96, "SideTask layout");
constexpr int kSideLds = 96;
typedef __attribute__((address_space(3))) SideTask LdsS;
#define SIDE_FIELDS(X) X(rbeg) X(qoff) X(rb) X(pos) X(dlo) X(dhi) X(qbeg) X(len) X(lq) X(tt) X(score) X(h0) \
  X(truesc) X(qb) X(aw0) X(cells) X(rows) X(calls)
__device__ __forceinline__ void spark(LdsS* p, const SideTask& t) {
#define X(f) p->f = t.f;
  SIDE_FIELDS(X)
#undef X
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ SideTask sload(LdsS* p) {
  asm volatile("" ::: "memory");
  SideTask t;
#define X(f) t.f = p->f;
  SIDE_FIELDS(X)
#undef X
  return t;
}
#undef SIDE_FIELDS

// a sub-slot's start: the side's target rows into its LDS buffer, the state
// of the side's first call (a right side reads what the left launch left in
// the seed's SeedExt slot)
template <int G, bool RIGHT>
__device__ __forceinline__ void side_start(SideTask& t, const DevOpt& o, const DevRef& ref, const SpecArgs& a,
                                           const FatTask& f, uint8_t* tb) {
  t.rbeg = f.rbeg;
  t.qoff = f.qoff;
  t.pos = f.pos;
  t.dlo = f.dlo;
  t.dhi = f.dhi;
  t.qbeg = (int)(f.qls & 1023u);
  t.len = (int)((f.qls >> 10) & 1023u);
  t.lq = (int)(f.qls >> 20);
  t.tt = 0;
  const int64_t pac_bytes = (ref.l_pac >> 2) + 1;
  const int r = (int)(threadIdx.x & (G - 1));
  if constexpr (!RIGHT) {
    const int n = rows_needed(o, t.qbeg, t.dlo, o.w << 1, o.pen_clip5);
    const int R = (n + G - 1) / G;
    if (R <= 32) fill_side_run<G>(tb, t.rbeg - 1, -1, r * R, min(r * R + R, n), ref, pac_bytes);
    else fill_two_half<G>(tb, t.rbeg - 1, n, tb, 0, 0, ref);
    t.score = -1;  // bwamem.c:753 (a left side: the retry test compares with -1)
    t.h0 = t.len * o.a;
    t.truesc = -1;
    t.qb = 0;
    t.rb = t.rbeg;
    t.aw0 = o.w;
    t.cells = t.rows = t.calls = 0;
  } else {
    const int64_t x0 = t.rbeg + t.len;
    const int qr = t.lq - t.qbeg - t.len;
    const int n = rows_needed(o, qr, (int)(t.rbeg + t.dhi - x0), o.w << 1, o.pen_clip3);
    const int R = (n + G - 1) / G;
    if (R <= 32) fill_side_run<G>(tb, x0, 1, r * R, min(r * R + R, n), ref, pac_bytes);
    else fill_two_half<G>(tb, 0, 0, tb, x0, n, ref);
    if (t.qbeg > 0) {  // the left launch's result (the same wave wrote... another wave did: SeedExt slot)
      const SeedExt e = a.ext[t.pos];
      t.score = e.score;
      t.truesc = e.truesc;
      t.qb = e.qb;
      t.rb = e.rb;
      t.aw0 = e.w;
      t.cells = e.cells;
      t.rows = e.rows;
      t.calls = e.calls;
    } else {
      t.score = t.truesc = t.len * o.a;  // bwamem.c:753
      t.qb = 0;
      t.rb = t.rbeg;
      t.aw0 = o.w;
      t.cells = t.rows = t.calls = 0;
    }
    t.h0 = t.score;  // sc0 (bwamem.c:761)
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <bool RIGHT>
__device__ __forceinline__ QCall side_call(const SideTask& t, const DevOpt& o, const uint8_t* seq, const uint8_t* tb) {
  QCall q;
  if constexpr (!RIGHT) {
    q.qlen = t.qbeg;
    q.tlen = t.dlo;
    q.qa = t.qbeg - 1;
    q.qd = -1;
    q.eb = o.pen_clip5;
  } else {
    const int64_t x0 = t.rbeg + t.len;
    q.qlen = t.lq - t.qbeg - t.len;
    q.tlen = (int)(t.rbeg + t.dhi - x0);
    q.qa = t.qbeg + t.len;
    q.qd = 1;
    q.eb = o.pen_clip3;
  }
  q.h0 = t.h0;
  q.w = o.w << t.tt;
  q.zdrop = o.zdrop;
  q.q = seq + t.qoff;
  q.tb = tb;
  q.tlen = rows_needed(o, q.qlen, q.tlen, q.w, q.eb);  // as qtask_call
  return q;
}

// the call's result (bwamem.c:737-751 / 770-792); true = the side is done,
// its result written to the seed's SeedExt slot (partial after a left side
// with a right side to come, else final)
template <int G, bool RIGHT>
__device__ __forceinline__ bool side_advance(SideTask& t, const DevOpt& o, const SpecArgs& a, const ExtOut& x,
                                             const Tally32& tl, long long& spec_cells) {
  t.cells += tl.cells;
  t.rows += tl.rows;
  t.calls += tl.calls;
  const int prev = t.score;
  t.score = x.score;
  const int aw = o.w << t.tt;
  if (t.tt == 0 && !(x.score == prev || x.max_off < (aw >> 1) + (aw >> 2))) {  // the band retry (MAX_BAND_TRY)
    t.tt = 1;
    return false;
  }
  const int eb = RIGHT ? o.pen_clip3 : o.pen_clip5;
  const bool local = x.gscore <= 0 || x.gscore <= x.score - eb;
  SeedExt e;
  if constexpr (!RIGHT) {
    const int qr = t.lq - t.qbeg - t.len;
    e.rb = t.rbeg - (local ? x.tle : x.gtle);
    e.qb = local ? t.qbeg - x.qle : 0;
    e.score = t.score;
    e.truesc = local ? x.score : x.gscore;
    if (qr != 0) {  // partial: the right launch goes on from here
      e.re = 0;
      e.qe = 0;
      e.w = aw;
      e.cells = t.cells;
      e.rows = t.rows;
      e.calls = t.calls;
    } else {
      e.re = t.rbeg + t.len;
      e.qe = t.lq;
      e.w = max(aw, o.w);
      e.cells = t.cells;
      e.rows = t.rows;
      e.calls = t.calls + 1;  // + 1: a computed slot is never all-zero
      spec_cells += t.cells;
    }
  } else {
    e.rb = t.rb;
    e.qb = t.qb;
    e.qe = local ? t.qbeg + t.len + x.qle : t.lq;
    e.re = t.rbeg + t.len + (local ? x.tle : x.gtle);
    e.score = t.score;
    e.truesc = t.truesc + (local ? x.score : x.gscore) - t.h0;
    e.w = max(t.aw0, aw);
    e.cells = t.cells;
    e.rows = t.rows;
    e.calls = t.calls + 1;
    spec_cells += t.cells;
  }
  store_ext_half<G>(a.ext + t.pos, e);
  return true;
}

// a side's query bytes into LDS in column order (qd[j] = column j), so the DP
// has no global load (its prologue read them from HBM: a dependent round trip
// per generation)
template <int G, bool RIGHT>
__device__ __forceinline__ void side_query(const DevBatch& b, const FatTask& f, uint8_t* qd, int qb) {
  const int r = (int)(threadIdx.x & (G - 1));
  const int qbeg = (int)(f.qls & 1023u), len = (int)((f.qls >> 10) & 1023u), lq = (int)(f.qls >> 20);
  const int qlen = min(RIGHT ? lq - qbeg - len : qbeg, qb);
  const uint8_t* q = b.seq + f.qoff + (RIGHT ? qbeg + len : qbeg - 1);
  for (int j = r; j < qlen; j += G) qd[j] = q[RIGHT ? j : -j];
}

// The phased extension's kernel: one side (RIGHT = false: left calls, true:
// right calls) of the tasks of one list, eight calls per wave (G = 16) or four
// (G = 32) in the packed 16-bit DP (extend_quad), claimed in the list's
// order (the side's query length, longest first).
template <int G, int PMAX, bool K8, bool RIGHT>
__global__ void __launch_bounds__(kBlock) spec_side4_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                            int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr uint64_t kLead = G == 16 ? 0x0001000100010001ull : 0x0000000100000001ull;
  const uint64_t below = kLead & ((1ull << ((int)threadIdx.x & (64 - G))) - 1);
  // per group: A's and B's target rows, their states, their query bytes
  constexpr int QB = PMAX * G;
  uint8_t* const ta_ = lds + (size_t)(threadIdx.x / G) * (2 * (size_t)tb_bytes + 2 * kSideLds + 2 * QB);
  uint8_t* const tb_ = ta_ + tb_bytes;
  LdsS* const sa = (LdsS*)(tb_ + tb_bytes);
  LdsS* const sb = (LdsS*)(tb_ + tb_bytes + kSideLds);
  uint8_t* const qa_ = tb_ + tb_bytes + 2 * kSideLds;
  uint8_t* const qb_ = qa_ + QB;
  const int n = uni(__hip_atomic_load(&a.ctr[(RIGHT ? SPC_RCNT : SPC_LCNT) + list], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT));
  const FatTask* fl = (RIGHT ? a.ftaskR : a.ftask) + spec_list_off(list, b.n_chains, b.n_seeds);
  ShardQ qq;
  qq.init(a.qh + 8 * kQHStride * (RIGHT ? kSpecRounds * kSpecBins + list : list) , n);
  bool ha = false, hb = false, more = n > 0;
  long long spec_cells = 0;
#ifdef BWAGPU_OCC_DIAG
  unsigned long long tw[6] = {0, 0, 0, 0, 0, 0}, occ[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  for (;;) {
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
    if (more) {  // every sub-slot without a call takes the next entry: one claim for the wave
      const uint64_t na = __builtin_amdgcn_ballot_w64(!ha) & kLead, nb = __builtin_amdgcn_ballot_w64(!hb) & kLead;
      const int nn = __popcll(na) + __popcll(nb);
      if (nn > 0) {
        int m0, cap;
        if (qq.claim(nn, m0, cap)) {
          const int ia = m0 + __popcll(na & below) + __popcll(nb & below), ib = ia + (ha ? 0 : 1);
          if (!ha && ia < cap) {
            SideTask t;
            const FatTask f = fl[qq.shard + 8 * ia];
            side_query<G, RIGHT>(b, f, qa_, QB);
            side_start<G, RIGHT>(t, o, ref, a, f, ta_);
            spark(sa, t);
            ha = true;
          }
          if (!hb && ib < cap) {
            SideTask t;
            const FatTask f = fl[qq.shard + 8 * ib];
            side_query<G, RIGHT>(b, f, qb_, QB);
            side_start<G, RIGHT>(t, o, ref, a, f, tb_);
            spark(sb, t);
            hb = true;
          }
        } else {
          more = false;
        }
      }
    }
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c1 = __builtin_amdgcn_s_memtime();
    tw[0] += c1 - c0;
#endif
    if (!__builtin_amdgcn_ballot_w64(ha || hb)) {
      if (!more) break;
      continue;
    }
    QCall ca = quad_idle(qa_, ta_), cb = quad_idle(qb_, tb_);  // every query pointer in LDS
    if (ha) {
      ca = side_call<RIGHT>(sload(sa), o, b.seq, ta_);
      ca.q = qa_;
      ca.qa = 0;
      ca.qd = 1;
    }
    if (hb) {
      cb = side_call<RIGHT>(sload(sb), o, b.seq, tb_);
      cb.q = qb_;
      cb.qa = 0;
      cb.qd = 1;
    }
    ExtOut xa, xb;
    Tally32 tla{0, 0, 0}, tlb{0, 0, 0};
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c2 = __builtin_amdgcn_s_memtime();
    tw[1] += c2 - c1;
#endif
    extend_quad_dispatch<G, PMAX, K8>(o, ca, cb, xa, xb, tla, tlb);
#ifdef BWAGPU_OCC_DIAG
    const unsigned long long c3 = __builtin_amdgcn_s_memtime();
    tw[2] += c3 - c2;
    occ_diag<G>(occ, ca, cb, tla, tlb);
#endif
    if (ha) {
      SideTask t = sload(sa);
      if (side_advance<G, RIGHT>(t, o, a, xa, tla, spec_cells)) ha = false;
      else spark(sa, t);
    }
    if (hb) {
      SideTask t = sload(sb);
      if (side_advance<G, RIGHT>(t, o, a, xb, tlb, spec_cells)) hb = false;
      else spark(sb, t);
    }
#ifdef BWAGPU_OCC_DIAG
    tw[3] += __builtin_amdgcn_s_memtime() - c3;
#endif
  }
#ifdef BWAGPU_OCC_DIAG
  if ((threadIdx.x & 63) == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 32) + k, occ[k]);
    for (int k = 0; k < 4; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 48) + k, tw[k]);
  }
#endif
  if ((threadIdx.x & (G - 1)) == 0 && spec_cells)
    atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
}

static size_t side4_lds(int tb_bytes, int g, int pmax) {
  return (size_t)(kBlock / g) * (2 * (size_t)tb_bytes + 2 * kSideLds + 2 * (size_t)pmax * g);
}

// ------------------------------------ the side kernel with a producer wave
// spec_side4_kernel's waves spent 17.5 % of their cycles at call starts: the
// claim, then the FatTask, then the target rows, three dependent round trips
// with nothing to hide them at one wave per SIMD (tools_dev/occ_diag.py,
// r06h).  spec_sidep_kernel pairs every DP wave with a producer wave that
// does only that: every call slot has a second buffer (the side's state, its
// target rows and its query bytes, all in LDS), and the producer keeps those
// filled, so a DP wave's next call starts from LDS.  A DP wave claims and
// fills its own first calls (as spec_side4_kernel) while its producer fills
// the second buffers.  Buffer b = k * 32 + group * 2 + half (k: which of the
// slot's two): kBufBusy = the DP wave's, kBufEmpty = the producer's to fill,
// kBufReady = filled.  A producer raises its `ex` once it leaves (the queue's
// tail: BWAGPU_SIDEP_RETIRE), after its last kBufReady; the DP wave then
// claims for itself.
constexpr int kBufEmpty = 0, kBufReady = 1, kBufBusy = 2;
__host__ __device__ constexpr int sidep_buf_bytes(int tb_bytes, int qb) { return (tb_bytes + qb + kSideLds + 15) & ~15; }

__device__ __forceinline__ int lds_ld(int* p) { return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP); }
// a buffer state after every LDS access of this wave before it (the DP's reads
// of the rows; the producer's writes of them): lgkmcnt only, so that the
// wave's outstanding global stores (SeedExt) are not waited for
__device__ __forceinline__ void lds_publish(int* p, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// a call slot's buffer: target rows (tb_bytes) | query bytes in column order (qb) | SideTask
template <int G, bool RIGHT>
__device__ __forceinline__ void side_prep(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a,
                                          const FatTask& f, uint8_t* buf, int tb_bytes, int qb) {
  uint8_t* const qd = buf + tb_bytes;
  side_query<G, RIGHT>(b, f, qd, qb);
  SideTask t;
  side_start<G, RIGHT>(t, o, ref, a, f, buf);
  spark((LdsS*)(qd + qb), t);
}

__device__ __forceinline__ FatTask shfl_fat(const FatTask& f, int src) {
  FatTask g;
  g.rbeg = (int64_t)((uint64_t)(uint32_t)__shfl((int)(f.rbeg >> 32), src, 64) << 32 | (uint32_t)__shfl((int)f.rbeg, src, 64));
  g.qoff = (int64_t)((uint64_t)(uint32_t)__shfl((int)(f.qoff >> 32), src, 64) << 32 | (uint32_t)__shfl((int)f.qoff, src, 64));
  g.pos = __shfl(f.pos, src, 64);
  g.dlo = __shfl(f.dlo, src, 64);
  g.dhi = __shfl(f.dhi, src, 64);
  g.qls = (uint32_t)__shfl((int)f.qls, src, 64);
  return g;
}

template <int G, int PMAX>
static size_t sidep_lds(int tb_bytes) {
  constexpr int nbuf = 4 * (kBlock / G);
  return (size_t)nbuf * sidep_buf_bytes(tb_bytes, PMAX * G) + 4 * (size_t)(nbuf + 4);
}

template <int G, int PMAX, bool K8, bool RIGHT>
__global__ void __launch_bounds__(2 * kBlock) spec_sidep_kernel(DevOpt o, DevRef ref, DevBatch b, SpecArgs a, int list,
                                                                int tb_bytes, int retire) {
  static_assert(G == 16, "a producer wave per DP wave: 2 buffers x 2 halves x 4 groups = 16 buffers");
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int QB = PMAX * G;            // query bytes per buffer (the widest call's columns)
  constexpr int NBUF = 4 * (kBlock / G);  // 64
  const int SB = sidep_buf_bytes(tb_bytes, QB);
  int* const st = reinterpret_cast<int*>(lds + (size_t)NBUF * SB);
  int* const ex = st + NBUF;  // per DP wave: its producer has left
  for (int k = threadIdx.x; k < NBUF + 4; k += 2 * kBlock) st[k] = k < NBUF / 2 ? kBufBusy : kBufEmpty;
  __syncthreads();
  const int n = uni(__hip_atomic_load(&a.ctr[(RIGHT ? SPC_RCNT : SPC_LCNT) + list], __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT));
  const FatTask* fl = (RIGHT ? a.ftaskR : a.ftask) + spec_list_off(list, b.n_chains, b.n_seeds);
  int32_t* const heads = a.qh + 8 * kQHStride * (RIGHT ? kSpecRounds * kSpecBins + list : list);
  ShardQ qq;
  qq.init(heads, n);
#ifdef BWAGPU_OCC_DIAG
  unsigned long long tw[6] = {0, 0, 0, 0, 0, 0}, occ[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
  const int lane = (int)(threadIdx.x & 63);
  if (threadIdx.x >= kBlock) {  // ---- a producer wave: DP wave pw's 16 buffers, lane l < 16 = buffer bmap(l)
    // above the DP wave it shares a SIMD with: the arbiter prefers the older
    // of two ready waves, and a DP wave is nearly always ready
    __builtin_amdgcn_s_setprio(2);
    const int pw = (int)(threadIdx.x - kBlock) >> 6;
    const auto bmap = [pw](int l) { return (l >> 3) << 5 | (4 * pw + ((l >> 1) & 3)) << 1 | (l & 1); };
    const uint64_t below = (1ull << lane) - 1;
    bool more = n > 0;
    while (more) {
#ifdef BWAGPU_OCC_DIAG
      const unsigned long long p0 = __builtin_amdgcn_s_memtime();
#endif
      const uint64_t em = __builtin_amdgcn_ballot_w64(lane < 16 && lds_ld(st + bmap(lane & 15)) == kBufEmpty);
      if (!em) {
        __builtin_amdgcn_s_sleep(2);
#ifdef BWAGPU_OCC_DIAG
        tw[5] += __builtin_amdgcn_s_memtime() - p0;
#endif
        continue;
      }
      int m0, cap;
      if (!qq.claim(__popcll(em), m0, cap)) break;
      const int idx = m0 + __popcll(em & below);
      const bool mine = ((em >> lane) & 1) && idx < cap;
      uint64_t v = __builtin_amdgcn_ballot_w64(mine);
      FatTask f{};
      if (mine) f = fl[qq.shard + 8 * idx];
      while (v) {  // four buffers at a time, a group of G lanes each
        int bsel = -1;
#pragma unroll
        for (int g = 0; g < 64 / G; ++g) {
          const int bq = v ? __builtin_ctzll(v) : -1;
          v &= v - 1;
          bsel = lane / G == g ? bq : bsel;
        }
        const FatTask g = shfl_fat(f, max(bsel, 0));
        const int bb = bmap(max(bsel, 0));
        if (bsel >= 0) side_prep<G, RIGHT>(o, ref, b, a, g, lds + (size_t)bb * SB, tb_bytes, QB);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the buffers' rows, query and state first
        if (bsel >= 0) __hip_atomic_store(st + bb, kBufReady, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
#ifdef BWAGPU_OCC_DIAG
      tw[4] += __builtin_amdgcn_s_memtime() - p0;
#endif
      // the queue's tail goes to the DP waves' own claims: a call claimed ahead
      // waits behind its slot's current one while other slots run dry
      if (cap - m0 - __popcll(em) < retire) break;
    }
    lds_publish(ex + pw, 1);
  } else {  // ---- a DP wave: eight call slots, half A / B of four groups
    const int gi = (int)threadIdx.x / G, gw = lane / G;
    const auto bidx = [gi](int h, int k) { return (k << 5) | (gi << 1) | h; };
    const auto bufp = [&](int h, int k) { return lds + (size_t)bidx(h, k) * SB; };
    constexpr uint64_t kLead = 0x0001000100010001ull;  // each group's first lane
    const uint64_t below = kLead & ((1ull << (lane & (64 - G))) - 1);
    bool ha = false, hb = false, fa = false, fb = false, dry = false;
    int ka = 0, kb = 0;  // the buffer of the slot's call (or its last one)
    long long spec_cells = 0;
    {  // the first calls: this wave's own claim (the producer fills the second buffers meanwhile)
      int m0, cap;
      if (n > 0 && qq.claim(2 * (64 / G), m0, cap)) {
        const int ia = m0 + 2 * gw, ib = ia + 1;
        if (ia < cap) {
          side_prep<G, RIGHT>(o, ref, b, a, fl[qq.shard + 8 * ia], bufp(0, 0), tb_bytes, QB);
          ha = true;
        }
        if (ib < cap) {
          side_prep<G, RIGHT>(o, ref, b, a, fl[qq.shard + 8 * ib], bufp(1, 0), tb_bytes, QB);
          hb = true;
        }
      }
      lds_publish(st + bidx(0, 0), ha ? kBufBusy : kBufEmpty);  // a slot without a first call: the producer's
      lds_publish(st + bidx(1, 0), hb ? kBufBusy : kBufEmpty);
    }
    for (;;) {
#ifdef BWAGPU_OCC_DIAG
      const unsigned long long c0 = __builtin_amdgcn_s_memtime();
#endif
      // a slot without a call takes a filled buffer: its other one (filled
      // while this call ran), else the one it just gave back (the producer may
      // have refilled that first).  Once the producer has left (`ex`, after
      // its last kBufReady) and neither is filled, the wave claims for the slot
      // itself (the queue's tail), into the slot's free buffer.
      const auto take = [&](int h, int& k, bool& has, bool& own, bool last) {
        own = false;
        if (has) return;
        const int so = lds_ld(st + bidx(h, k ^ 1)), sk = lds_ld(st + bidx(h, k));
        if (so == kBufReady) {
          has = true;
          k ^= 1;
        } else if (sk == kBufReady) {
          has = true;
        } else {
          own = last;
        }
      };
      for (;;) {
        const bool last = __hip_atomic_load(ex + (threadIdx.x >> 6), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != 0;  // before the states
        bool oa, ob;
        take(0, ka, ha, oa, last && !fa);
        take(1, kb, hb, ob, last && !fb);
        const uint64_t na = __builtin_amdgcn_ballot_w64(oa) & kLead, nb = __builtin_amdgcn_ballot_w64(ob) & kLead;
        if (na | nb) {
          int m0, cap;
          if (!dry && qq.claim(__popcll(na) + __popcll(nb), m0, cap)) {
            const int ia = m0 + __popcll(na & below) + __popcll(nb & below), ib = ia + (oa ? 1 : 0);
            if (oa && ia < cap) {
              side_prep<G, RIGHT>(o, ref, b, a, fl[qq.shard + 8 * ia], bufp(0, ka), tb_bytes, QB);
              ha = true;
            }
            if (ob && ib < cap) {
              side_prep<G, RIGHT>(o, ref, b, a, fl[qq.shard + 8 * ib], bufp(1, kb), tb_bytes, QB);
              hb = true;
            }
          } else {
            dry = true;
            fa = fa || oa;
            fb = fb || ob;
          }
        }
        if (!__builtin_amdgcn_ballot_w64((!ha && !fa) || (!hb && !fb))) break;
        if (!(na | nb)) __builtin_amdgcn_s_sleep(1);
      }
      if (!__builtin_amdgcn_ballot_w64(ha || hb)) break;
#ifdef BWAGPU_OCC_DIAG
      const unsigned long long c1 = __builtin_amdgcn_s_memtime();
      tw[0] += c1 - c0;
#endif
      uint8_t* const pa = bufp(0, ka);
      uint8_t* const pb = bufp(1, kb);
      LdsS* const sa = (LdsS*)(pa + tb_bytes + QB);
      LdsS* const sb = (LdsS*)(pb + tb_bytes + QB);
      QCall ca = quad_idle(pa + tb_bytes, pa), cb = quad_idle(pb + tb_bytes, pb);  // every query pointer in LDS
      if (ha) {
        ca = side_call<RIGHT>(sload(sa), o, b.seq, pa);
        ca.q = pa + tb_bytes;
        ca.qa = 0;
        ca.qd = 1;
      }
      if (hb) {
        cb = side_call<RIGHT>(sload(sb), o, b.seq, pb);
        cb.q = pb + tb_bytes;
        cb.qa = 0;
        cb.qd = 1;
      }
      ExtOut xa, xb;
      Tally32 tla{0, 0, 0}, tlb{0, 0, 0};
#ifdef BWAGPU_OCC_DIAG
      const unsigned long long c2 = __builtin_amdgcn_s_memtime();
      tw[1] += c2 - c1;
#endif
      extend_quad_dispatch<G, PMAX, K8>(o, ca, cb, xa, xb, tla, tlb);
#ifdef BWAGPU_OCC_DIAG
      const unsigned long long c3 = __builtin_amdgcn_s_memtime();
      tw[2] += c3 - c2;
      occ_diag<G>(occ, ca, cb, tla, tlb);
#endif
      if (ha) {
        SideTask t = sload(sa);
        if (side_advance<G, RIGHT>(t, o, a, xa, tla, spec_cells)) {
          ha = false;
          lds_publish(st + bidx(0, ka), kBufEmpty);
        } else {
          spark(sa, t);
        }
      }
      if (hb) {
        SideTask t = sload(sb);
        if (side_advance<G, RIGHT>(t, o, a, xb, tlb, spec_cells)) {
          hb = false;
          lds_publish(st + bidx(1, kb), kBufEmpty);
        } else {
          spark(sb, t);
        }
      }
#ifdef BWAGPU_OCC_DIAG
      tw[3] += __builtin_amdgcn_s_memtime() - c3;
#endif
    }
    if ((threadIdx.x & (G - 1)) == 0 && spec_cells)
      atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + SPC_SPEC64), (unsigned long long)spec_cells);
  }
#ifdef BWAGPU_OCC_DIAG
  if (lane == 0) {
    for (int k = 0; k < 8; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 32) + k, occ[k]);
    for (int k = 0; k < 6; ++k) atomicAdd(reinterpret_cast<unsigned long long*>(a.ctr + 48) + k, tw[k]);
  }
#endif
}

// The pair kernel's grid: its waves pull tasks from the queue, so the grid
// only sets its occupancy.  2 workgroups per CU (8 waves per CU, 2 per SIMD)
// instead of the resident capacity (5 per SIMD): the batch on the other caller
// stream (the bench's ping-pong) and this batch's selection kernels keep the
// rest, and an even count per CU beats an uneven one.  Same-box sweep
// (DESIGN.md §3): capacity 19.87, 60 % 20.74, 50 % 20.66, 2/CU (40 %) 21.74,
// 30 % 20.16, 1/CU 19.72 Mreads/s.  The packed kernels (two 209 / 198-VGPR
// waves per SIMD at 2/CU) run at 1 workgroup per CU: 37.97-38.04 against
// 36.99-37.17 Mreads/s on C2, C3 0.66 against 0.78-0.79 ms per batch (same
// box).  BWAGPU_EXT2_BLOCKS_PER_CU overrides both.
static int ext2_grid(int nb, bool packed) {
  static const int env_cu = [] {
    const char* e = getenv("BWAGPU_EXT2_BLOCKS_PER_CU");
    const int v = e ? atoi(e) : 0;
    return v < 0 ? 0 : v;
  }();
  const int per_cu = env_cu ? env_cu : (packed ? 1 : 2);
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      ncu <= 0)
    return nb;
  return std::max(1, std::min(nb, per_cu * ncu));
}


// The sequential logic of mem_chain2aln over one read's chains, by one wave.
// A seed that is extended but has no result yet:
//   SEL_EMULATE  becomes a round-B task (its region stays unknown in this pass);
//   SEL_FINAL    is listed (the round-C list, a diagnostic count) and the read goes to the redo list
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
  sel_prio();
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
    if (d.lq > a.lq_bound) continue;  // flagged by spec_reads_kernel
    const uint8_t* const q = b.seq + d.qoff;
    const int rep_lim = (int)floor(.1 * d.lq) + 1;  // s->len - p->seedlen0 > .1 * l_query, bwamem.c:685
    bool redo = false;
    Tally rt{0, 0, 0};
    int nreg = 0, n_inline = 0;
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
            ++n_inline;
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
    // (the redo pass as pass 2, its inline extensions in the shape word's upper bits)
    trace_read(MODE, b.n_reads, rd, t_start, d.ns, nreg, 2 | (MODE == SEL_REDO ? n_inline << 4 : 0));
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
// extend has no result: 10-30 per C2 batch before round 6's strict emulation)
// was extended inline, which took the kernel to 129 VGPRs (3 waves per SIMD);
// sending it to the redo pass instead lost in rounds 3-4 (19.8-19.9 vs
// 21.6-21.7 Mreads/s on C2, then 29.4-30.2 vs 36.9-37.3), while
// the misses were there to extend.
// With the strict emulation (BWAGPU_EMU_STRICT, default) a light read's final
// pass has no miss; -DBWAGPU_LIGHT_INLINE=0 leaves the inline extension out
// (84 VGPRs instead of 131, no LDS rows; a miss, with BWAGPU_EMU_STRICT=0,
// then goes to the redo pass like one of a longer read), but the larger
// resident grid competes with the other records' extension kernels: C2
// fixture 49.3 / 50.6 vs 51.0 / 52.5 Mreads/s, stream 50.5 vs 51.8 (r06p).
#ifndef BWAGPU_LIGHT_INLINE
#define BWAGPU_LIGHT_INLINE 1
#endif
template <int MODE>
__global__ void __launch_bounds__(kBlock) spec_select_light(DevOpt o, DevRef ref, DevBatch b, SpecArgs a,
                                                            int tb_bytes) {
  sel_prio();
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
  // same; no queue atomics), the next read's descriptor in flight meanwhile.
  // The final pass first takes, in its static share, only the reads the
  // emulate pass left a round-B task in (rbits): only those can miss, and a
  // miss is extended inline (one wave, ~0.1 ms per extension, cascades of
  // several in a read) — so they start first, and every other read is claimed
  // afterwards in chunks of kLightChunk by whichever wave is free, instead of
  // waiting behind a wave's misses in its static share.
  const int NW = (int)gridDim.x * (kBlock / 64);
  const int w0 = (int)blockIdx.x * (kBlock / 64) + uni((int)(threadIdx.x >> 6));
  constexpr int kLightChunk = 16;
  int ph = 0, cb = 0, ce = 0, pbase = w0 - 64 * NW;
  uint64_t pm = 0;
  const auto risky = [&](int x) { return ((a.rbits[x >> 5] >> (x & 31)) & 1u) != 0; };
  const auto next_read = [&]() -> int {
    if (ph == 0) {  // this wave's static share, the reads with a round-B task, 64 at a time
      for (;;) {
        if (pm) {
          const int i = __builtin_ctzll(pm);
          pm &= pm - 1;
          return pbase + i * NW;
        }
        pbase += 64 * NW;
        if (pbase >= b.n_reads) break;
        const int x = pbase + r * NW;
        pm = __builtin_amdgcn_ballot_w64(x < b.n_reads && risky(x));
      }
      ph = 1;
    }
    for (;;) {  // the rest, claimed
      if (cb >= ce) {
        int c = 0;
        if (r == 0) c = atomicAdd(&a.ctr[SPC_LIGHT_CUR], kLightChunk);
        c = __builtin_amdgcn_readfirstlane(__shfl(c, 0, 64));
        if (c >= b.n_reads) return b.n_reads;
        cb = c;
        ce = min(c + kLightChunk, b.n_reads);
      }
      const int y = cb++;
      if (!risky(y)) return y;
    }
  };
  const bool dyn = MODE == SEL_FINAL && a.risky_first;
  int rd = dyn ? next_read() : w0;
  ReadDesc dn{};
  if (rd < b.n_reads) dn = a.rdesc[rd];
  for (int nx; rd < b.n_reads; rd = nx) {
    const uint64_t t_start = g_trace ? __builtin_amdgcn_s_memrealtime() : 0;
    const ReadDesc d = uniform_desc(dn);
    nx = dyn ? next_read() : rd + NW;
    if (nx < b.n_reads) dn = a.rdesc[nx];
    if (d.ns > kSelLight || d.nch > kSelLight) continue;  // the heavy kernel's read
    if (d.lq > a.lq_bound) continue;                      // flagged by spec_reads_kernel
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
    // (emulate) unc: the seeds whose decisions the final pass may take
    // otherwise — the pending ones, every seed extended after one, and every
    // skip that is not certain; a seed skipped here but maybe not there gets
    // a round-B task too (spend), so the final pass never misses
    uint64_t ext = 0, skip = pad_m, pend = 0, spend = 0, unc = 0;
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
          // certainly skipped in the final pass too iff a region of a seed
          // decided before any pending one holds it and no seed it overlaps
          // has an uncertain decision
          if (MODE == SEL_EMULATE && a.emu_strict && (!(cm & ext & ~unc) || (om & unc))) {
            unc |= bit;
            if (!(computed_m & bit)) spend |= bit;
          }
          continue;
        }
      }
      if (!(computed_m & bit)) {
        if (MODE == SEL_EMULATE) {
          pend |= bit;  // a round-B task; its region stays unknown in this pass
          unc |= bit;
          continue;
        }
        miss = k;
        break;
      }
      ext |= bit;
      if (MODE == SEL_EMULATE && pend) unc |= bit;  // a pending seed's region may hold it
    }
    // ---- 3. outputs
    if constexpr (MODE == SEL_EMULATE) {
      const int list = kSpecBins + spec_bin(d.lq);
      const bool pnd = ((pend | spend) >> r) & 1;
      const int p = wave_append(&a.ctr[SPC_CNT + list], pnd);
      if (p >= 0) a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + r, d.c0 + cid);
      if (pend && r == 0) atomicOr(&a.rbits[rd >> 5], 1u << (rd & 31));  // the final pass takes it first
    } else {
      if (BWAGPU_LIGHT_INLINE && miss >= 0 && d.lq <= kSpecBinLen[0]) {  // extend seed `miss` here, then the read again
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
      if (miss >= 0) {  // the redo pass (reads > 160 bp)
        // round C extends the miss and every later seed without a result: the
        // redo replay's next misses are among them (one region changes the
        // decisions after it), and the packed kernels take them all at once
        // instead of the redo wave one after another
        const int list = 2 * kSpecBins + spec_bin(d.lq);
        const int p = wave_append(&a.ctr[SPC_CNT + list], r >= miss && present && !computed);
        if (p >= 0) a.tasks[spec_list_off(list, b.n_chains, b.n_seeds) + p] = make_int2(d.s0 + r, d.c0 + cid);
        if (r == miss) a.redo[atomicAdd(&a.ctr[SPC_REDO_N], 1)] = rd;
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
  sel_prio();
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

__device__ __forceinline__ uint64_t lane64(uint64_t v, int l) { return (uint64_t)readlane64((int64_t)v, l); }

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
  const SeedExt e = d.lq <= 192 ? extend_seed<3>(o, ref, sk, d.lq, b.seq + d.qoff, cw, tbl, tbr)
                                 : extend_seed<4>(o, ref, sk, d.lq, b.seq + d.qoff, cw, tbl, tbr);  // <= 256 bp
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
  sel_prio();
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
    if (d.lq > a.lq_bound) continue;  // flagged by spec_reads_kernel
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
    // Blocks of 64 seeds: the tests of seed k against the regions and skips of
    // the earlier blocks (final by then) run lane-parallel, lane r for seed
    // 64 * bw + r over its row's earlier words; only the in-block word is
    // decided seed by seed, on scalar masks.  (One seed per step cost ~256 ns:
    // a dependent row load, a ballot and a branch per seed.)
    // (emulate, BWAGPU_EMU_STRICT) as in spec_select_light: the seeds of
    // uncertain decision (unc_w: lane w's word) — pending, extended after the
    // first pending one (fp), or skipped without certainty — and a seed
    // skipped here that the final pass might extend gets a round-B task
    uint64_t ext_w = 0, pend_w = 0, unc_w = 0;
    const bool strict = MODE == SEL_EMULATE && a.emu_strict;
    int fp = ns;
    int miss = -1;
    for (int bw = 0; bw < nw && miss < 0; ++bw) {
      const int kb = 64 * bw, k = kb + r;
      const bool valid = k < ns;
      const int64_t row = tri_off(valid ? k : ns - 1);
      bool cb = false, cbc = false;
      for (int w = 0; w < bw; ++w) {
        const uint64_t x = C[row + w] & lane64(ext_w, w);
        cb |= x != 0;
        if (strict) cbc |= (x & ~lane64(unc_w, w)) != 0;  // held by a region decided before fp
      }
      uint64_t cin = valid && r > 0 ? C[row + bw] : 0;
      // O matters only where a region contains seed k
      bool need = valid && (cb || cin != 0), ob = false, ou = false;
      uint64_t oin = 0;
      if (__builtin_amdgcn_ballot_w64(need)) {
        if (need) {
          for (int w = 0; w < bw; ++w) {
            const uint64_t x = O[row + w];
            ob |= (x & ~lane64(skip_w, w)) != 0;
            if (strict) ou |= (x & lane64(unc_w, w)) != 0;  // overlaps a seed of uncertain decision
          }
          oin = r > 0 ? O[row + bw] : 0;
        }
      }
      const uint64_t cbm = __builtin_amdgcn_ballot_w64(valid && cb);
      uint64_t obm = __builtin_amdgcn_ballot_w64(valid && ob);
      const uint64_t cbcm = __builtin_amdgcn_ballot_w64(valid && cbc), oum = __builtin_amdgcn_ballot_w64(valid && ou);
      const uint64_t pres = lane64(present_w, bw);
      uint64_t comp = lane64(computed_w, bw), skp = lane64(skip_w, bw), ext = 0, pend = 0, spend = 0;
      uint64_t uncb = 0;  // this block's seeds of uncertain decision
      const int nb = min(64, ns - kb);
      for (int i = 0; i < nb; ++i) {
        const uint64_t bit = 1ull << i;
        if (!(pres & bit)) continue;
        if ((cbm & bit) || (lane64(cin, i) & ext)) {
          if (!(obm & bit) && !(lane64(oin, i) & ~skp)) {  // skipped: srt[k] = 0 (bwamem.c:709)
            skp |= bit;
            if (strict && (!((cbcm & bit) || (lane64(cin, i) & ext & ~uncb)) || (oum & bit) || (lane64(oin, i) & uncb))) {
              uncb |= bit;
              if (!(comp & bit)) spend |= bit;
            }
            continue;
          }
        }
        if (!(comp & bit)) {
          if (MODE == SEL_EMULATE) {
            pend |= bit;  // a round-B task; its region stays unknown
            uncb |= bit;
            fp = min(fp, kb + i);
            continue;
          }
          if (d.lq > kSpecBinLen[1]) {  // longer reads: the redo pass
            miss = kb + i;
            break;
          }
          heavy_fill_missing(o, ref, b, a, d, kb + i, ns, C, tbl, tbr);
          comp |= bit;
          cin = valid && r > 0 ? C[row + bw] : 0;  // column kb + i of the later rows
          const bool fresh = valid && !need && cin != 0;
          if (__builtin_amdgcn_ballot_w64(fresh)) {
            if (fresh) {
              for (int w = 0; w < bw; ++w) ob |= (O[row + w] & ~lane64(skip_w, w)) != 0;
              oin = O[row + bw];
            }
            need = need || fresh;
            obm = __builtin_amdgcn_ballot_w64(valid && ob);
          }
        }
        ext |= bit;
        if (strict && fp < kb + i) uncb |= bit;  // a pending seed's region may hold it
      }
      ext_w = r == bw ? ext : ext_w;
      skip_w = r == bw ? skp : skip_w;
      pend_w = r == bw ? pend | spend : pend_w;
      unc_w = r == bw ? uncb : unc_w;
      computed_w = r == bw ? comp : computed_w;
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
  if (MODE != SEL_REDO) {  // target rows in LDS only for the final pass's inline extension
    const size_t lds = BWAGPU_LIGHT_INLINE && MODE == SEL_FINAL ? (size_t)(kBlock / 64) * 2 * tb_bytes : 0;
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

// The first two length bins' extension kernel: eight seeds per wave for the
// first bin and four for the second (spec_ext4_kernel, packed 16-bit DP) when
// every score of the bin fits the packed ranges, else two per wave
// (spec_ext2_kernel, 32-bit).  Form 1 (bwagpu_ctx_ext_form, per context)
// forces two per wave, 2 four per wave in the first bin too (tests, A/B).
// the phased extension (spec_side4_kernel) per length bin: BWAGPU_EXT_PHASED
// is a mask (bit 0: the first bin, bit 1: the second); unset = 1.  The second
// bin (161-256 bp) stays on the task state machine of spec_ext4_kernel by
// default: its calls run ~250 rows, so the tail of each side launch (one long
// call on a nearly empty chip) cost more than the phasing saved (C5: 3.42 ms
// per batch with both bins phased, 2.81 with neither, r06h).
static int ext_phased_mask() {
  static const int m = [] {
    const char* e = getenv("BWAGPU_EXT_PHASED");
    return e && e[0] ? atoi(e) & 3 : 1;
  }();
  return m;
}

// the phased pair with producer waves (spec_sidep_kernel; the first bin's
// eight-per-wave form only): BWAGPU_EXT_PRODUCER=1.  Off by default: it lost
// on every A/B (C2 43.6-47.4 vs 50.9-54.5 Mreads/s)
static bool ext_producer() {
  static const bool on = [] {
    const char* e = getenv("BWAGPU_EXT_PRODUCER");
    return e && e[0] == '1';
  }();
  return on;
}
static std::atomic<int> g_ext_form{0};
int ext_form() { return g_ext_form.load(std::memory_order_relaxed); }
int ext_kernel_for(const DevOpt& o, int form, int tb_bytes) {  // launch_ext_round's choice, first bin
  const bool quad = form != 1 && quad_scores_ok(o, kSpecBinLen[1]) && quad_rows_ok(o, tb_bytes);
  const bool key8 = quad && quad_key8_ok(o, kSpecBinLen[0]);
  const int k = key8 ? (form == 0 ? 8 : 4) : (quad ? 5 : 2);
  if (!quad || !(ext_phased_mask() & 1)) return k;
  // the phased pair: 28 with the producer wave (spec_sidep_kernel), 1x spec_side4_kernel
  return k == 8 && ext_producer() && sidep_lds<16, kSpecBinLen[0] / 16>(tb_bytes) <= 64 * 1024 ? 28 : 10 + k;
}
int set_ext_form(int form) {  // the default of contexts made later; -> the previous one (form < 0: query only)
  const int prev = g_ext_form.load(std::memory_order_relaxed);
  if (form >= 0) g_ext_form.store(form > 2 ? 1 : form, std::memory_order_relaxed);
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
// the 8-bit-column row-max key (extend_quad<.., true>): every H of reads up to lq < 256
bool quad_key8_ok(const DevOpt& o, int lq) { return (long)lq * o.max_mat <= 255; }
// the packed row-end state for calls of up to `rows` target rows: i, |i - j|
// and the z-drop term max((di - dj) e_del, (dj - di) e_ins) (di <= rows,
// dj <= 256) within 16 bits beside H < 4096
bool quad_rows_ok(const DevOpt& o, long rows) {
  return rows >= 0 && rows < 16384 && (rows + 256) * std::max(o.e_del, o.e_ins) < 28672;
}

// one side launch of the phased extension for list l: G calls per group
template <int G, int PMAX, bool K8>
static void launch_side_pair(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a, int l,
                             int tb_bytes, hipStream_t st, int grid_cap, int round) {
  const size_t lds = side4_lds(tb_bytes, G, PMAX);
  const int nb = resident_blocks(spec_side4_kernel<G, PMAX, K8, false>, lds);
  const int gr = round == 2 ? std::min(nb, 64) : std::min(nb, grid_cap);
  hipLaunchKernelGGL((spec_side4_kernel<G, PMAX, K8, false>), dim3(gr), dim3(kBlock), lds, st, o, ref, b, a, l,
                     tb_bytes);
  hipLaunchKernelGGL((spec_side4_kernel<G, PMAX, K8, true>), dim3(gr), dim3(kBlock), lds, st, o, ref, b, a, l,
                     tb_bytes);
}

template <int G, int PMAX, bool K8>
static bool launch_sidep_pair(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a, int l,
                              int tb_bytes, hipStream_t st, int grid_cap, int round) {
  const size_t lds = sidep_lds<G, PMAX>(tb_bytes);
  if (!ext_producer() || lds > 64 * 1024) return false;
  // the producer leaves its shard's last `retire` entries to the DP waves'
  // own claims (BWAGPU_SIDEP_RETIRE; 1 024 = one call per call slot of an XCD)
  static const int retire = [] {
    const char* e = getenv("BWAGPU_SIDEP_RETIRE");
    return e && e[0] ? std::max(atoi(e), 0) : 1024;
  }();
  const int nb = resident_blocks(spec_sidep_kernel<G, PMAX, K8, false>, lds, 2 * kBlock);
  const int gr = round == 2 ? std::min(nb, 64) : std::min(nb, grid_cap);
  hipLaunchKernelGGL((spec_sidep_kernel<G, PMAX, K8, false>), dim3(gr), dim3(2 * kBlock), lds, st, o, ref, b, a, l,
                     tb_bytes, retire);
  hipLaunchKernelGGL((spec_sidep_kernel<G, PMAX, K8, true>), dim3(gr), dim3(2 * kBlock), lds, st, o, ref, b, a, l,
                     tb_bytes, retire);
  return true;
}

// the length bins' lists in the order their kernels take them: pair order
// (spec_sort_*) for the task state machine, one list per side in its query
// length order (spec_sort2_*) for the phased launches
static void launch_sort(const DevOpt& o, const DevBatch& b, const SpecArgs& a, int round, bool phased, int bin0,
                        int nbins, hipStream_t st) {
  if (phased) {
    hipLaunchKernelGGL(spec_sort2_count, dim3(256, nbins), dim3(256), 0, st, b, a, round, bin0);
    hipLaunchKernelGGL(spec_sort2_scan, dim3(2 * nbins), dim3(256), 0, st, a, round, bin0, nbins);
    hipLaunchKernelGGL(spec_sort2_scatter, dim3(256, nbins), dim3(256), 0, st, o, b, a, round, bin0);
  } else {
    hipLaunchKernelGGL(spec_sort_count, dim3(256, nbins), dim3(256), 0, st, b, a, round, bin0);
    hipLaunchKernelGGL(spec_sort_scan, dim3(nbins), dim3(256), 0, st, a, round, bin0);
    hipLaunchKernelGGL(spec_sort_scatter, dim3(256, nbins), dim3(256), 0, st, b, a, round, bin0);
  }
}

// Only the bins the batch's longest read reaches are launched: a persistent
// grid over an empty list still waits for CU slots that the other caller
// stream's extension kernel holds, and its stream waits with it.  Round C
// (mispredicted seeds of long reads: rare) runs on small grids for the same
// reason.
static void launch_ext_round(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a, int round,
                             int tb_bytes, int lq_max, hipStream_t st, const SpecStreams& ss) {
  const size_t lds = (size_t)(kBlock / 64) * 2 * tb_bytes;
  const int l = round * kSpecBins;
  const bool bin1 = lq_max > kSpecBinLen[0], bin2 = lq_max > kSpecBinLen[1];
  const int form = ss.form;
  const bool quad = form != 1 && quad_scores_ok(o, kSpecBinLen[1]) && quad_rows_ok(o, tb_bytes);
  const auto grid = [round, quad](int nb) { return round == 2 ? std::min(nb, 64) : ext2_grid(nb, quad); };
  const bool key8 = quad && quad_key8_ok(o, kSpecBinLen[0]), oct = key8 && form == 0;
  const size_t lds2 = quad ? ext4_lds(tb_bytes, 32) : ext2_lds(tb_bytes);
  const int pm = quad ? ext_phased_mask() : 0;
  const bool p0 = pm & 1, p1 = (pm >> 1) & 1;
  if (!bin1 || p0 == p1) {
    launch_sort(o, b, a, round, p0, 0, bin1 ? 2 : 1, st);
  } else {
    launch_sort(o, b, a, round, p0, 0, 1, st);
    launch_sort(o, b, a, round, p1, 1, 1, st);
  }
  const int cap = ext2_grid(1 << 30, true);
  const bool prof = ss.pool && *ss.pool_used + 2 <= ss.pool_n;
  if (prof) (void)hipEventRecord(ss.pool[*ss.pool_used], st);
  if (p0) {
    if (oct) {
      if (!launch_sidep_pair<16, kSpecBinLen[0] / 16, true>(o, ref, b, a, l + 0, tb_bytes, st, cap, round))
        launch_side_pair<16, kSpecBinLen[0] / 16, true>(o, ref, b, a, l + 0, tb_bytes, st, cap, round);
    } else if (key8) launch_side_pair<32, kSpecBinLen[0] / 32, true>(o, ref, b, a, l + 0, tb_bytes, st, cap, round);
    else launch_side_pair<32, kSpecBinLen[1] / 32, false>(o, ref, b, a, l + 0, tb_bytes, st, cap, round);
  } else if (oct) {
    const size_t lds8 = ext4_lds(tb_bytes, 16);
    const int nb = resident_blocks(spec_ext4_kernel<16, kSpecBinLen[0] / 16, true>, lds8);
    hipLaunchKernelGGL((spec_ext4_kernel<16, kSpecBinLen[0] / 16, true>), dim3(grid(nb)), dim3(kBlock), lds8, st, o,
                       ref, b, a, l + 0, tb_bytes);
  } else if (key8) {
    const int nb = resident_blocks(spec_ext4_kernel<32, kSpecBinLen[0] / 32, true>, lds2);
    hipLaunchKernelGGL((spec_ext4_kernel<32, kSpecBinLen[0] / 32, true>), dim3(grid(nb)), dim3(kBlock), lds2, st, o,
                       ref, b, a, l + 0, tb_bytes);
  } else if (quad) {
    const int nb = resident_blocks(spec_ext4_kernel<32, kSpecBinLen[1] / 32, false>, lds2);
    hipLaunchKernelGGL((spec_ext4_kernel<32, kSpecBinLen[1] / 32, false>), dim3(grid(nb)), dim3(kBlock), lds2, st, o,
                       ref, b, a, l + 0, tb_bytes);
  } else {
    const int nb = resident_blocks(spec_ext2_kernel<kSpecBinLen[0] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext2_kernel<kSpecBinLen[0] / 32>, dim3(grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 0, tb_bytes);
  }
  if (prof) {
    (void)hipEventRecord(ss.pool[*ss.pool_used + 1], st);
    *ss.pool_used += 2;
  }
  if (!bin1) return;
  if (p1) {
    if (form == 0) launch_side_pair<16, kSpecBinLen[1] / 16, false>(o, ref, b, a, l + 1, tb_bytes, st, cap, round);
    else launch_side_pair<32, kSpecBinLen[1] / 32, false>(o, ref, b, a, l + 1, tb_bytes, st, cap, round);
  } else if (quad && form == 0) {  // eight per wave, the row-max key widened per call (H may reach 256 and more)
    const size_t lds8 = ext4_lds(tb_bytes, 16);
    const int nb = resident_blocks(spec_ext4_kernel<16, kSpecBinLen[1] / 16, false>, lds8);
    hipLaunchKernelGGL((spec_ext4_kernel<16, kSpecBinLen[1] / 16, false>), dim3(grid(nb)), dim3(kBlock), lds8, st, o,
                       ref, b, a, l + 1, tb_bytes);
  } else if (quad) {
    const int nb = resident_blocks(spec_ext4_kernel<32, kSpecBinLen[1] / 32, false>, lds2);
    hipLaunchKernelGGL((spec_ext4_kernel<32, kSpecBinLen[1] / 32, false>), dim3(grid(nb)), dim3(kBlock), lds2, st, o,
                       ref, b, a, l + 1, tb_bytes);
  } else {
    const int nb = resident_blocks(spec_ext2_kernel<kSpecBinLen[1] / 32>, lds2);
    hipLaunchKernelGGL(spec_ext2_kernel<kSpecBinLen[1] / 32>, dim3(grid(nb)), dim3(kBlock), lds2, st, o, ref, b, a,
                       l + 1, tb_bytes);
  }
  if (!bin2) return;
  const int nb = resident_blocks(spec_ext_kernel<16>, lds);
  hipLaunchKernelGGL(spec_ext_kernel<16>, dim3(round == 2 ? std::min(nb, 64) : nb), dim3(kBlock), lds, st, o, ref, b, a,
                     l + 2, tb_bytes);
}

// prep -> round A -> emulate -> round B -> final -> [round C] -> redo, one
// stream.  The final pass sends a read over 160 bp that misses an extension,
// and a heavy read without a pair matrix, to the redo pass, and their
// missing seeds to the round-C lists (a light read: the miss and every later
// seed without a result).  Batches with reads over 160 bp run round C with
// the packed kernels first (C5: one read's chain of 12 misses took the redo
// wave 2.3 ms one extension at a time), so the redo pass mostly replays; on
// shorter batches (C2: no such miss) round C stays unlaunched — a launch
// waited ~0.18 ms per batch for CU slots the other caller stream's extension
// kernel held, even over an empty list — and the redo pass extends the rare
// misses inline.  With the strict emulation (BWAGPU_EMU_STRICT, default) the
// light and matrix-heavy reads have no miss left, so round C stays unlaunched
// on every batch; a heavy read without a matrix can still miss, and the redo
// pass extends that inline.
hipError_t launch_spec_chain2aln(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a,
                                 int tb_bytes, int lq_max, hipStream_t st, const SpecStreams& ss) {
  if (b.n_reads == 0) return hipSuccess;
  hipLaunchKernelGGL(spec_reads_kernel, dim3((b.n_reads + 255) / 256), dim3(256), 0, st, b, a);
  if (b.n_chains) {
    hipLaunchKernelGGL(spec_chain_kernel, dim3((b.n_chains + 255) / 256), dim3(256), 0, st, o, ref, b, a);
    hipLaunchKernelGGL(spec_order_kernel, dim3(kOrderBlocks), dim3(256), 0, st, o, ref, b, a);
  }
  if (b.n_chains) {
    launch_ext_round(o, ref, b, a, 0, tb_bytes, lq_max, st, ss);
    launch_select<SEL_EMULATE>(o, ref, b, a, tb_bytes, st, ss);
    launch_ext_round(o, ref, b, a, 1, tb_bytes, lq_max, st, ss);
  }
  launch_select<SEL_FINAL>(o, ref, b, a, tb_bytes, st, ss);
  if (b.n_chains && lq_max > kSpecBinLen[0] && !a.emu_strict) launch_ext_round(o, ref, b, a, 2, tb_bytes, lq_max, st, ss);
  if (b.n_chains) launch_select<SEL_REDO>(o, ref, b, a, tb_bytes, st, ss);
  return hipGetLastError();
}

// a batch's zeroed state in one launch (blockIdx.y = which array)
__global__ void __launch_bounds__(256) spec_clear_kernel(SpecArgs a, int nr, int ns) {
  const int t0 = (int)(blockIdx.x * 256 + threadIdx.x), nt = (int)(gridDim.x * 256);
  switch (blockIdx.y) {
    case 0:
      for (int i = t0; i < 3 * ns; i += nt) reinterpret_cast<uint4*>(a.ext)[i] = make_uint4(0, 0, 0, 0);  // 48 B each
      break;
    case 1:
      for (int i = t0; i < nr; i += nt) a.out_n[i] = 0;
      break;
    case 2:
      for (int i = t0; i < nr / 32 + 1; i += nt) a.rbits[i] = 0;
      break;
    case 3:
      for (int i = t0; i < kQHWords; i += nt) a.qh[i] = 0;
      break;
    case 4:
      for (int i = t0; i < kSortWords; i += nt) a.sorth[i] = 0;
      break;
    default:
      for (int i = t0; i < SPC_WORDS; i += nt) a.ctr[i] = 0;
  }
}
static_assert(sizeof(SeedExt) == 48, "spec_clear_kernel clears SeedExt as three uint4");

hipError_t launch_spec_clear(const SpecArgs& a, int n_reads, int n_seeds, hipStream_t st) {
  hipLaunchKernelGGL(spec_clear_kernel, dim3(256, 6), dim3(256), 0, st, a, n_reads, n_seeds);
  return hipGetLastError();
}

size_t spec_select_lds(int tb_bytes) { return (size_t)kSelHeavyLds + 0 * tb_bytes; }
int spec_redo_cap(int tb_bytes) { return sel_heavy_cap(SEL_REDO, tb_bytes); }

}  // namespace bwagpu
