// sw_kernels.hip — MI355X (gfx950) per-read mem_chain2aln and bare
// ksw_extend2 task lists.
//
// The hot path of bwa-flow's ChainsToRegions stage (src/Pipeline.cpp:503-544):
// for every read, every chain goes through mem_chain2aln (bwa/bwamem.c:641-795),
// whose inner loop is the banded affine-gap extension ksw_extend2
// (bwa/ksw.c:380-479).  Integer DP, VALU-bound, no MFMA.  The DP cores live in
// ksw_dev.h; the default (speculative) mem_chain2aln in spec.hip.  This file:
//  * the per-read path (BWAGPU_C2A_PATH=fast; the independent cross-check of
//    the speculative one): chain windows and seed order (chain_prep_kernel),
//    reads cost-sorted into bins (read_bins/bin_scan/read_scatter), then one
//    wave owns one read for the whole of mem_chain2aln — window, seed order,
//    containment, left/right extensions with band retries, seedcov, region
//    output — chain2aln_fast_kernel for reads of <= 256 bp with <= 32 seeds and
//    chains (the read's table in LDS, double-buffered DMA), chain2aln_kernel
//    for the rest;
//  * bwagpu_extend_batch's task lists: one call per wave (extend_kernel) or
//    four per wave where the packed ranges hold (extend4_kernel).
#include <hip/hip_runtime.h>
#include <limits.h>

#include <algorithm>
#include <atomic>
#include <map>
#include <mutex>
#include <tuple>

#include "engine.h"
#include "wave_ops.h"
#include "ksw_dev.h"

namespace bwagpu {

const Variant kVariants[kNumVariants] = {{64, 3, VK_FAST}, {64, 4, VK_FAST}, {64, 16, VK_GENERIC}};
const Variant kExtVariants[kNumExtVariants] = {{64, 3, VK_FAST}, {64, 4, VK_FAST}, {64, 16, VK_GENERIC}};

// Optional per-read trace (bwagpu_debug_set_trace): 8 words per read index:
// start/end s_memrealtime (100 MHz), DP rows, DP cells, HW_ID, XCC_ID.
__device__ uint32_t* g_trace = nullptr;

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
    extend_quad_dispatch<32, PMAX, false>(o, ca, cb, xa, xb, ta, tb);
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

}  // namespace bwagpu
