// chain.hip — seeding's chaining on the device (bwa-flow SeqsToChains after
// the interval search, src/bwa_wrapper.cpp:105-115): mem_chain's body
// (bwa/bwamem.c:260-330), test_and_merge (199-221), mem_chain_flt (336-396)
// and mem_flt_chained_seeds (607-624; mem_seed_sw 580-605 becomes a batch of
// ksw_align2 tasks for align2.hip).  Layout: chain.h.
//
// The work of one read is a strictly sequential walk — every seed either
// joins the chain kb_intervalp finds for it or opens a new one, and the
// chain's last seed decides the next merge — so a read runs on one wave that
// executes the walk wave-uniformly, with its kbtree, chain records and lists
// in LDS: each step of the walk is a chain of dependent accesses (~25 per
// seed), which LDS answers in ~100 cycles where L2 takes several hundred.
// Reads are binned by their SA position count (LDS arenas for 32 / 128 / 512 /
// 1536 positions, kBinCap in chain.h, up to ~154 KB: gfx950's 160 KB LDS;
// run_chaining refuses a device with less); the rare larger reads run the same code on a
// global-memory arena.  The kbtree is restated as a B-tree of chain ids with
// the reference's node search, split and in-order traversal (t = 5): chains
// with EQUAL positions exist (tandem repeats), and their order — and which of
// them kb_intervalp returns — follows the tree's shape.  mem_chain_weight is
// accumulated as seeds are appended (its two sweeps run in append order), so
// mem_chain_flt needs no second pass over the seeds.  Positions are expanded
// by a wave per read and resolved by bwt_sa (seed.hip) in between.
#include <hip/hip_runtime.h>

#include "chain.h"

namespace bwagpu {
namespace {

__device__ __forceinline__ int pcmp(int64_t a, int64_t b) { return (b < a) - (a < b); }

// ---- per read: interval count -> SA positions, frac_rep (bwamem.c:272-290)
__global__ void __launch_bounds__(256) chain_count_kernel(ChainArgs a) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads) return;
  const int len = (int)(a.seq_off[r + 1] - a.seq_off[r]);
  int n = a.intv_n[r];
  if (n < 0) {  // more intervals than the slots: the host reruns with room for them
    atomicMax(a.need, -n);
    n = 0;
  }
  if (len < a.min_seed_len) n = 0;  // bwamem.c:270
  const bwagpu_intv_t* iv = a.intv + (int64_t)r * a.max_per_read;
  int b = 0, e = 0, l_rep = 0, np = 0;
  for (int i = 0; i < n; ++i) {
    const uint64_t x2 = iv[i].x[2], info = iv[i].info;
    const int sb = (int)(info >> 32), se = (int)(uint32_t)info;
    np += (int)(x2 < (uint64_t)a.max_occ ? x2 : (uint64_t)a.max_occ);
    if (x2 <= (uint64_t)a.max_occ) continue;
    if (sb > e) l_rep += e - b, b = sb, e = se;
    else e = e > se ? e : se;
  }
  l_rep += e - b;
  a.n_pos[r] = np;
  a.frac_rep[r] = len > 0 ? (float)l_rep / len : 0.f;
}

// ---- one wave per read: the BWT rows of mem_chain's loop (bwamem.c:284-288)
__global__ void __launch_bounds__(256) chain_emit_kernel(ChainArgs a) {
  const int r = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = (int)(threadIdx.x & 63);
  if (r >= a.n_reads || a.n_pos[r] == 0) return;
  const bwagpu_intv_t* iv = a.intv + (int64_t)r * a.max_per_read;
  const int n = a.intv_n[r];
  int64_t o = a.pos_off[r];
  for (int i = 0; i < n; ++i) {
    const uint64_t x0 = iv[i].x[0], x2 = iv[i].x[2], info = iv[i].info;
    const int cnt = (int)(x2 < (uint64_t)a.max_occ ? x2 : (uint64_t)a.max_occ);
    const int step = x2 > (uint64_t)a.max_occ ? (int)(x2 / (uint64_t)a.max_occ) : 1;
    const int qbeg = (int)(info >> 32), slen = (int)((uint32_t)info - (uint32_t)(info >> 32));
    for (int c = lane; c < cnt; c += 64) {
      a.kpos[o + c] = x0 + (uint64_t)((int64_t)c * step);
      a.qinfo[o + c] = make_int2(qbeg, slen);
      a.score[o + c] = slen;
    }
    o += cnt;
  }
}

// ---- the kbtree (kbtree.h:54-197, 336-358) of one read.  CH / ND are the
// chain and node pointer types: LDS (address space 3) or global.  The tree is
// walked by the whole wave: a node's keys are read one per lane and its
// search is a ballot (keys are sorted, so the count of keys below pos is the
// lower bound the reference's binary search finds); insertion shifts and
// splits move one key per lane.
__device__ __forceinline__ int64_t readlane64(int64_t v, int l) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)v, l), hi = __builtin_amdgcn_readlane((int)(v >> 32), l);
  return (int64_t)((uint64_t)(uint32_t)hi << 32 | (uint32_t)lo);
}
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront"); }

template <class CH, class ND>
struct Tree {
  CH* ch;
  ND* nd;
  int root, n_nodes, n_keys;

  // a node in registers, loaded in one round of independent LDS reads: lane l
  // holds key[l] (l < kBN) and child[l] (l <= kBN)
  struct Row {
    int n, internal, k, c;
  };
  __device__ Row row(int x) const {
    const int lane = (int)(threadIdx.x & 63);
    Row v;
    v.n = nd[x].n;
    v.internal = nd[x].internal;
    v.k = lane < kBN ? (int)nd[x].key[lane] : 0;
    v.c = lane <= kBN ? (int)nd[x].child[lane] : 0;
    return v;
  }

  // first key >= pos (r = 0 if equal, else -1 after stepping back to the last
  // key < pos); past the end the last key with r = 1 (kbtree.h:100-113);
  // *key = the key at the returned index
  __device__ int find(const Row& v, int64_t pos, int& r, int& key) const {
    const int lane = (int)(threadIdx.x & 63);
    const int n = v.n;
    if (n == 0) {
      r = -1;
      return -1;
    }
    int64_t kp = 0;
    if (lane < n) kp = ch[v.k].s0_rbeg;
    const int b = __builtin_popcountll(__builtin_amdgcn_ballot_w64(lane < n && kp < pos));
    int i;
    if (b == n) {
      r = 1;
      i = n - 1;
    } else {
      r = pcmp(pos, readlane64(kp, b));
      i = r < 0 ? b - 1 : b;
    }
    key = i >= 0 ? __builtin_amdgcn_readlane(v.k, i) : -1;
    return i;
  }
  __device__ int find(int x, int64_t pos, int& r, int& key) const { return find(row(x), pos, r, key); }

  __device__ int lower(int64_t pos) const {  // kb_intervalp's lower (kbtree.h:130-147)
    int lo = -1, r = 0, key;
    for (int x = root;;) {
      const Row v = row(x);
      const int i = find(v, pos, r, key);
      if (i >= 0 && r == 0) return key;
      if (i >= 0) lo = key;
      if (!v.internal) return lo;
      x = __builtin_amdgcn_readlane(v.c, i + 1);
    }
  }

  // lower() that also remembers where kb_putp would insert pos: when the
  // descent reached a leaf and no node on it is full, kb_putp's own descent
  // (the same finds on the same nodes, no split on the way) ends at that leaf
  // after key index `leaf_i` — put_at() then inserts there without a second
  // walk from the root.  Otherwise leaf = -1 and put() walks.
  __device__ int lower_at(int64_t pos, int& leaf, int& leaf_i) const {
    int lo = -1, r = 0, key;
    bool full = false;
    leaf = -1;
    for (int x = root;;) {
      const Row v = row(x);
      const int i = find(v, pos, r, key);
      full = full || v.n == kBN;
      if (i >= 0 && r == 0) return key;
      if (i >= 0) lo = key;
      if (!v.internal) {
        if (!full) {
          leaf = x;
          leaf_i = i;
        }
        return lo;
      }
      x = __builtin_amdgcn_readlane(v.c, i + 1);
    }
  }

  // lower() for a tree whose keys are distinct, per lane (each lane its own
  // pos and path): the key of the largest position <= pos, or -1
  __device__ int lower_lane(int64_t pos) const {
    int lo = -1;
    for (int x = root;;) {
      const int n = nd[x].n;
      int c = 0;
      for (int j = 0; j < kBN; ++j) {
        if (j < n) {
          const int k = nd[x].key[j];
          const int64_t kp = ch[k].s0_rbeg;
          if (kp == pos) return k;
          if (kp < pos) {
            c = j + 1;
            lo = k;
          }
        }
      }
      if (!nd[x].internal) return lo;
      x = nd[x].child[c];
    }
  }

  __device__ void put_at(int k, int x, int i) {  // kb_putp's leaf insertion (kbtree.h:186-195)
    const int lane = (int)(threadIdx.x & 63);
    ++n_keys;
    const int xn = nd[x].n;
    int kv = 0;
    const bool mv = lane > i && lane < xn;  // keys i+1..xn-1 move up one
    if (mv) kv = nd[x].key[lane];
    wave_sync();
    if (mv) nd[x].key[lane + 1] = kv;
    wave_sync();
    nd[x].key[i + 1] = k;
    nd[x].n = xn + 1;
    wave_sync();
  }

  __device__ void split(int x, int i, int y) {  // __kb_split (kbtree.h:152-167)
    const int lane = (int)(threadIdx.x & 63);
    const int z = n_nodes++;
    const int yi = nd[y].internal, xn = nd[x].n;
    const int med = nd[y].key[kBT - 1];
    if (lane < kBT - 1) nd[z].key[lane] = nd[y].key[kBT + lane];
    if (yi && lane < kBT) nd[z].child[lane] = nd[y].child[kBT + lane];
    // x's children i+1..xn move up one, keys i..xn-1 likewise (read, then write)
    int cv = 0, kv = 0;
    const bool mc = lane > i && lane <= xn, mk = lane >= i && lane < xn;
    if (mc) cv = nd[x].child[lane];
    if (mk) kv = nd[x].key[lane];
    wave_sync();
    if (mc) nd[x].child[lane + 1] = cv;
    if (mk) nd[x].key[lane + 1] = kv;
    wave_sync();
    nd[z].internal = yi;
    nd[z].n = kBT - 1;
    nd[y].n = kBT - 1;
    nd[x].child[i + 1] = z;
    nd[x].key[i] = med;
    nd[x].n = xn + 1;
    wave_sync();
  }

  __device__ void put(int k, int64_t pos) {  // kb_putp (kbtree.h:168-197)
    const int lane = (int)(threadIdx.x & 63);
    int r, key;
    ++n_keys;
    if (nd[root].n == kBN) {
      const int s = n_nodes++;
      nd[s].internal = 1;
      nd[s].n = 0;
      nd[s].child[0] = root;
      wave_sync();
      split(s, 0, root);
      root = s;
    }
    for (int x = root;;) {
      if (!nd[x].internal) {
        const int i = find(x, pos, r, key);
        const int xn = nd[x].n;
        int kv = 0;
        const bool mv = lane > i && lane < xn;  // keys i+1..xn-1 move up one
        if (mv) kv = nd[x].key[lane];
        wave_sync();
        if (mv) nd[x].key[lane + 1] = kv;
        wave_sync();
        nd[x].key[i + 1] = k;
        nd[x].n = xn + 1;
        wave_sync();
        return;
      }
      int i = find(x, pos, r, key) + 1;
      const int c = nd[x].child[i];
      if (nd[c].n == kBN) {
        split(x, i, c);
        if (pos > ch[nd[x].key[i]].s0_rbeg) ++i;
      }
      x = nd[x].child[i];
    }
  }
};

__device__ int pos2rid(const ChainArgs& a, int64_t pos_f) {  // bns_pos2rid (bntseq.c:349-363)
  int left = 0, mid = 0, right = a.n_seqs;
  if (pos_f >= a.l_pac) return -1;
  while (left < right) {
    mid = (left + right) >> 1;
    if (pos_f >= a.ann_off[mid]) {
      if (mid == a.n_seqs - 1) break;
      if (pos_f < a.ann_off[mid + 1]) break;
      left = mid + 1;
    } else {
      right = mid;
    }
  }
  return mid;
}

__device__ __forceinline__ int64_t depos(int64_t l_pac, int64_t pos) { return pos >= l_pac ? (l_pac << 1) - 1 - pos : pos; }

__device__ int intv2rid(const ChainArgs& a, int64_t rb, int64_t re) {  // bntseq.c:365-373
  if (rb < a.l_pac && re > a.l_pac) return -2;
  const int b = pos2rid(a, depos(a.l_pac, rb));
  const int e = rb < re ? pos2rid(a, depos(a.l_pac, re - 1)) : b;
  return b == e ? b : -1;
}

// klib introsort (ksort.h:146-226) by weight, greater first (mem_flt's
// flt_lt, bwamem.c:333-334), step for step: it is not stable.  The values are
// packed keys w << 32 | chain id (one LDS access per comparison); only w is
// compared.
struct ByW {
  __device__ bool operator()(int64_t x, int64_t y) const { return (x >> 32) > (y >> 32); }
};
template <class I, class LT>
__device__ void c_insert(I* a, int s, int t, LT lt) {  // [s, t)
  for (int i = s + 1; i < t; ++i)
    for (int j = i; j > s && lt(a[j], a[j - 1]); --j) {
      const int64_t x = a[j];
      a[j] = a[j - 1];
      a[j - 1] = x;
    }
}
template <class I, class LT>
__device__ void c_comb(I* a, int s, int n, LT lt) {  // a[s, s+n)
  const double shrink = 1.2473309501039786540366528676643;
  int gap = n;
  bool swapped;
  do {
    if (gap > 2) {
      gap = (int)(gap / shrink);
      if (gap == 9 || gap == 10) gap = 11;
    }
    swapped = false;
    for (int i = s; i < s + n - gap; ++i)
      if (lt(a[i + gap], a[i])) {
        const int64_t x = a[i];
        a[i] = a[i + gap];
        a[i + gap] = x;
        swapped = true;
      }
  } while (swapped || gap > 2);
  if (gap != 1) c_insert(a, s, s + n, lt);
}
template <class I, class LT>
__device__ void c_introsort(int n, I* a, LT lt) {
  if (n < 1) return;
  if (n == 2) {
    if (lt(a[1], a[0])) {
      const int64_t x = a[0];
      a[0] = a[1];
      a[1] = x;
    }
    return;
  }
  int d = 2;
  while ((1 << d) < n) ++d;
  struct Frame {
    int l, r, d;
  } stack[64];
  int top = 0, s = 0, t = n - 1;
  d <<= 1;
  for (;;) {
    if (s < t) {
      if (--d == 0) {
        c_comb(a, s, t - s + 1, lt);
        t = s;
        continue;
      }
      int i = s, j = t, k = i + ((j - i) >> 1) + 1;
      if (lt(a[k], a[i])) {
        if (lt(a[k], a[j])) k = j;
      } else {
        k = lt(a[j], a[i]) ? i : j;
      }
      const int64_t rp = a[k];
      if (k != t) {
        a[k] = a[t];
        a[t] = rp;
      }
      for (;;) {
        do ++i; while (lt(a[i], rp));
        do --j; while (i <= j && lt(rp, a[j]));
        if (j <= i) break;
        const int64_t x = a[i];
        a[i] = a[j];
        a[j] = x;
      }
      {
        const int64_t x = a[i];
        a[i] = a[t];
        a[t] = x;
      }
      if (i - s > t - i) {
        if (i - s > 16) stack[top++] = Frame{s, i - 1, d};
        s = t - i > 16 ? i + 1 : t;
      } else {
        if (t - i > 16) stack[top++] = Frame{i + 1, t, d};
        t = i - s > 16 ? i - 1 : s;
      }
    } else {
      if (top == 0) {
        c_insert(a, 0, n, lt);
        return;
      }
      --top;
      s = stack[top].l;
      t = stack[top].r;
      d = stack[top].d;
    }
  }
}

// ---- one read on one wave: mem_chain's loop, the kbtree traversal,
// mem_chain_flt, the chains out.  Every lane runs the same sequential code
// on the same data (wave-uniform: LDS reads broadcast, every lane stores the
// same value), except the final copy-out, which is lane-parallel.  CH / ND /
// IX: pointer types of the chains, nodes and index lists (LDS or global).
template <bool STAGED, class CH, class ND, class IX, class RB, class QI, class S64>
__device__ void chain_read(const ChainArgs& a, int r, CH* ch, ND* nd, IX* label, IX* slist, IX* ord, RB* rbeg,
                           QI* qi, S64* sc) {
  const int lane = (int)(threadIdx.x & 63);
  const int np = a.n_pos[r];
  const int64_t base = a.pos_off[r];
  uint64_t* dbg = a.dbg ? a.dbg + 8 * (int64_t)r : nullptr;
  auto stamp = [&](int k) {
    if (dbg && lane == 0) dbg[k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  if constexpr (STAGED) {  // an LDS arena: the seeds staged in, coalesced
    for (int p = lane; p < np; p += 64) {
      rbeg[p] = a.rbeg[base + p];
      qi[p] = reinterpret_cast<const int64_t*>(a.qinfo)[base + p];
    }
    wave_sync();
  }
  Tree<CH, ND> t{ch, nd, 0, 1, 0};
  nd[0].n = 0;
  nd[0].internal = 0;
  int n_ch = 0;
  // bns_pos2rid's answer for the last contig looked up (its [offset, next
  // offset) span): a read's seeds mostly fall in one contig
  int64_t c_lo = 1, c_hi = 0;
  int c_rid = -1;
  auto rid_of = [&](int64_t pos_f) -> int {
    if (pos_f >= a.l_pac) return -1;
    if (pos_f >= c_lo && pos_f < c_hi) return c_rid;
    const int m = pos2rid(a, pos_f);
    c_lo = a.ann_off[m];
    c_hi = m == a.n_seqs - 1 ? a.l_pac : a.ann_off[m + 1];
    c_rid = m;
    return m;
  };
  // Blocks of 64 seeds.  Lane-parallel per block: the seed, its contig
  // (bns_intv2rid) and, while no two chains share a position, its lower bound
  // in the tree as it stands — the chain with the largest position <= the
  // seed's, the only one kb_intervalp can return when positions are
  // distinct.  Serially: test_and_merge against that chain, and for a new
  // chain its insertion, after which the block's later seeds whose bound the
  // new position becomes take it.  Once two chains share a position (tandem
  // repeats), which of them kbtree returns depends on the tree's shape, and
  // every seed walks the tree itself (lower_at) as before.
  bool dup = false;
  for (int p0 = 0; p0 < np; p0 += 64) {  // bwamem.c:286-311
    const int nb = min(64, np - p0);
    const bool in = lane < nb;
    const int pl = p0 + (in ? lane : 0);
    const int64_t sr_l = (int64_t)rbeg[pl];
    const int64_t q_l = qi[pl];  // qbeg | len << 32
    const int qb_l = (int)(uint32_t)q_l, sl_l = (int)(q_l >> 32);
    int rid_l = -1;
    if (in) {  // bns_intv2rid (bntseq.c:365-373)
      if (sr_l < a.l_pac && sr_l + sl_l > a.l_pac) {
        rid_l = -2;
      } else {
        const int rb_ = rid_of(depos(a.l_pac, sr_l));
        const int re_ = sl_l > 0 ? rid_of(depos(a.l_pac, sr_l + sl_l - 1)) : rb_;
        rid_l = rb_ == re_ ? rb_ : -1;
      }
    }
    int lo_l = -1, lab_l = -1;
    if (!dup && t.n_keys && in && rid_l >= 0) lo_l = t.lower_lane(sr_l);
    int64_t lp_l = lo_l >= 0 ? (int64_t)ch[lo_l].s0_rbeg : INT64_MIN;
    const uint64_t live = __builtin_amdgcn_ballot_w64(in && rid_l >= 0);
    for (int q = 0; q < nb; ++q) {
      if (!((live >> q) & 1)) continue;
      const int rid = __builtin_amdgcn_readlane(rid_l, q);
      const int64_t sr = readlane64(sr_l, q);
      const int qb = __builtin_amdgcn_readlane(qb_l, q), sl = __builtin_amdgcn_readlane(sl_l, q);
      int lab = -1;
      bool add = true;
      int leaf = -1, leaf_i = 0;
      const int lo = !dup ? __builtin_amdgcn_readlane(lo_l, q) : (t.n_keys ? t.lower_at(sr, leaf, leaf_i) : -1);
      if (lo >= 0) {
        // test_and_merge (bwamem.c:199-221)
        const int64_t c_last_rbeg = ch[lo].last_rbeg, c_s0_rbeg = ch[lo].s0_rbeg;
        const int c_last_qbeg = ch[lo].last_qbeg, c_last_len = ch[lo].last_len, c_s0_qbeg = ch[lo].s0_qbeg;
        const int64_t qend = c_last_qbeg + c_last_len, rend = c_last_rbeg + c_last_len;
        if (rid == ch[lo].rid) {
          if (qb >= c_s0_qbeg && qb + sl <= qend && sr >= c_s0_rbeg && sr + sl <= rend) {
            add = false;  // contained: dropped
          } else if (!((c_last_rbeg < a.l_pac || c_s0_rbeg < a.l_pac) && sr >= a.l_pac)) {
            const int64_t x = qb - c_last_qbeg, y = sr - c_last_rbeg;
            if (y >= 0 && x - y <= a.w && y - x <= a.w && x - c_last_len < a.max_chain_gap &&
                y - c_last_len < a.max_chain_gap) {
              ch[lo].last_qbeg = (int16_t)qb;
              ch[lo].last_rbeg = sr;
              ch[lo].last_len = (int16_t)sl;
              ch[lo].n = ch[lo].n + 1;
              {  // mem_chain_weight's two sweeps, one seed further (bwamem.c:227-240)
                const int eq = ch[lo].endq;
                int wq = ch[lo].wq;
                if (qb >= eq) wq += sl;
                else if (qb + sl > eq) wq += qb + sl - eq;
                ch[lo].wq = (int16_t)wq;
                ch[lo].endq = (int16_t)(eq > qb + sl ? eq : qb + sl);
                const int64_t er = ch[lo].endr;
                int wr = ch[lo].wr;
                if (sr >= er) wr += sl;
                else if (sr + sl > er) wr += (int)(sr + sl - er);
                ch[lo].wr = (int16_t)(wr < 32767 ? wr : 32767);  // only min(wq, wr) is read
                ch[lo].endr = er > sr + sl ? er : sr + sl;
              }
              lab = lo;
              add = false;
            }
          }
        }
        if (add && c_s0_rbeg == sr) dup = true;  // the new chain will share lo's position
      }
      if (add) {
        CH* c = ch + n_ch;
        c->s0_rbeg = c->last_rbeg = sr;
        c->endr = sr + sl;
        c->s0_qbeg = c->last_qbeg = (int16_t)qb;
        c->last_len = (int16_t)sl;
        c->endq = (int16_t)(qb + sl);
        c->wq = c->wr = (int16_t)sl;
        c->rid = rid;
        c->n = 1;
        c->is_alt = (int8_t)(a.is_alt ? (a.is_alt[rid] != 0) : 0);
        c->kept = 0;
        c->first = -1;
        c->w = 0;
        lab = n_ch;
        if (leaf >= 0) t.put_at(n_ch, leaf, leaf_i);
        else t.put(n_ch, sr);
        // the later seeds of the block whose lower bound the new position becomes
        const bool aff = lane > q && lp_l < sr && sr <= sr_l;
        lo_l = aff ? n_ch : lo_l;
        lp_l = aff ? sr : lp_l;
        ++n_ch;
      }
      lab_l = lane == q ? lab : lab_l;
    }
    if (in) label[p0 + lane] = lab_l;
    wave_sync();
  }
  stamp(1);
  // in-order traversal (__kb_traverse, kbtree.h:336-358): the chain order
  int no = 0;
  {
    int sn[24], si[24], top = -1;
    for (int x = t.root;;) {  // the leftmost path
      sn[++top] = x;
      si[top] = 0;
      if (!nd[x].internal) break;
      x = nd[x].child[0];
    }
    while (top >= 0) {
      const int x = sn[top], i = si[top];
      if (i < nd[x].n) {
        ord[no++] = nd[x].key[i];
        si[top] = i + 1;
        if (nd[x].internal)
          for (int y = nd[x].child[i + 1];;) {
            sn[++top] = y;
            si[top] = 0;
            if (!nd[y].internal) break;
            y = nd[y].child[0];
          }
      } else {
        --top;
      }
    }
  }
  {  // seed lists in kbtree order, each in merge (= processing) order
    int s = 0;
    for (int k = 0; k < no; ++k) {
      const int id = ord[k];
      ch[id].soff = s;
      ch[id].cur = 0;
      s += ch[id].n;
    }
    for (int p = 0; p < np; ++p) {
      const int l = label[p];
      if (l >= 0) {
        const int c = ch[l].cur;
        slist[ch[l].soff + c] = p;
        ch[l].cur = c + 1;
      }
    }
  }
  stamp(2);
  int nout = no;
  if (!a.raw) {  // mem_chain_flt (bwamem.c:336-396)
    int nf = 0;
    for (int k = 0; k < no; ++k) {
      const int id = ord[k];
      int w = ch[id].wr < ch[id].wq ? ch[id].wr : ch[id].wq;  // mem_chain_weight
      w = w < (1 << 30) ? w : (1 << 30) - 1;
      w &= (1 << 29) - 1;  // the 29-bit field of mem_chain_t
      ch[id].w = (int16_t)w;
      ch[id].first = -1;
      ch[id].kept = 0;
      if (w >= a.min_chain_weight) ord[nf++] = id;
    }
    // sc: 64-bit scratch (the staged seeds or the BWT rows, no longer read)
    for (int k = lane; k < nf; k += 64) sc[k] = (int64_t)ch[ord[k]].w << 32 | (uint32_t)ord[k];
    wave_sync();
    stamp(3);
    c_introsort(nf, sc, ByW{});
    wave_sync();
    stamp(4);
    for (int k = lane; k < nf; k += 64) ord[k] = (int32_t)(uint32_t)sc[k];
    wave_sync();
    nout = 0;
    if (nf > 0) {
      // the kept list, one packed entry per kept chain: sorted index (the
      // list's own element) | chain beg | end | w | is_alt, in sc
      auto kept_entry = [&](int i) -> int64_t {
        const int c = ord[i];
        return (int64_t)i | (int64_t)(uint16_t)ch[c].s0_qbeg << 20 |
               (int64_t)(uint16_t)(ch[c].last_qbeg + ch[c].last_len) << 34 | (int64_t)(uint16_t)ch[c].w << 48 |
               (int64_t)(ch[c].is_alt != 0) << 63;
      };
      int nk = 0;
      ch[ord[0]].kept = 3;
      sc[nk++] = kept_entry(0);
      // the pairwise loop (bwamem.c:355-375): chain i against the kept list,
      // 64 entries at a time — each lane tests one; the scan stops at the
      // first entry whose break condition holds (ballot), and every entry up
      // to it applies its large_ovlp / first updates (distinct chains)
      for (int i = 1; i < nf; ++i) {
        const int ci = ord[i];
        const int bi = ch[ci].s0_qbeg, ei = ch[ci].last_qbeg + ch[ci].last_len;
        const int wi = ch[ci].w, ai = ch[ci].is_alt;
        bool large = false, brk = false;
        for (int k0 = 0; k0 < nk && !brk; k0 += 64) {
          const int k = k0 + lane;
          bool sig = false, drop = false;
          int j = 0;
          if (k < nk) {
            const int64_t e = sc[k];
            j = (int)(e & 0xfffff);
            const int bj = (int)((e >> 20) & 0x3fff), ej = (int)((e >> 34) & 0x3fff), wj = (int)((e >> 48) & 0x7fff);
            const bool aj = e < 0;
            const int b_max = bj > bi ? bj : bi, e_min = ej < ei ? ej : ei;
            if (e_min > b_max && (!aj || ai)) {
              const int li = ei - bi, lj = ej - bj;
              const int min_l = li < lj ? li : lj;
              if (e_min - b_max >= min_l * a.mask_level && min_l < a.max_chain_gap) {
                sig = true;
                drop = wi < wj * a.drop_ratio && wj - wi >= a.min_seed_len << 1;
              }
            }
          }
          const uint64_t dm = __builtin_amdgcn_ballot_w64(drop);
          const int lim = dm ? __builtin_ctzll(dm) : 64;  // lanes <= lim take part
          brk = dm != 0;
          const bool act = sig && lane <= lim;
          if (__builtin_amdgcn_ballot_w64(act)) large = true;
          if (act) {
            const int cj = ord[j];
            if (ch[cj].first < 0) ch[cj].first = i;
          }
          wave_sync();
        }
        if (!brk) {
          sc[nk++] = kept_entry(i);
          ch[ci].kept = (int8_t)(large ? 2 : 3);
        }
      }
      for (int i = lane; i < nk; i += 64) {
        const int f = ch[ord[(int)(sc[i] & 0xfffff)]].first;
        if (f >= 0) ch[ord[f]].kept = 1;
      }
      __threadfence_block();
      int i, k;
      for (i = k = 0; i < nf; ++i) {
        const int kp = ch[ord[i]].kept;
        if (kp == 0 || kp == 3) continue;
        if (++k >= a.max_chain_extend) break;
      }
      for (; i < nf; ++i)
        if (ch[ord[i]].kept < 3) ch[ord[i]].kept = 0;
      for (i = 0; i < nf; ++i)
        if (ch[ord[i]].kept != 0) ord[nout++] = ord[i];
    }
  }
  stamp(5);
  // the chains out and their seeds, lane-parallel
  DChain* oc = a.ochains + base;
  int32_t* os = a.oslist + base;
  int ns = 0;
  for (int k = 0; k < nout; ++k) {
    const int id = ord[k];
    const int n = ch[id].n, s0 = ch[id].soff;
    if (lane == 0) {
      DChain d;
      d.pos = ch[id].s0_rbeg;
      d.rid = ch[id].rid;
      d.n = n;
      d.w = a.raw ? 0 : ch[id].w;
      d.kept = a.raw ? 0 : ch[id].kept;
      d.first = a.raw ? -1 : ch[id].first;
      d.is_alt = ch[id].is_alt;
      d.soff = ns;
      d.pad_ = 0;
      oc[k] = d;
    }
    for (int j = lane; j < n; j += 64) os[ns + j] = slist[s0 + j];
    ns += n;
  }
  if (lane == 0) {
    a.n_out[r] = nout;
    a.n_oseed[r] = ns;
    int nsw = 0;
    if (!a.raw && nout) {
      const int len = (int)(a.seq_off[r + 1] - a.seq_off[r]);
      if (a.sw_tab[len] >= 0) nsw = ns;  // mem_flt_chained_seeds runs (bwamem.c:609-611)
    }
    a.n_sw[r] = nsw;
  }
  if (dbg && lane == 0) {
    dbg[6] = __builtin_amdgcn_s_memrealtime();
    dbg[7] = (uint64_t)np | (uint64_t)no << 32;
  }
}

// reads into bins by their position count (the last bin: global memory);
// one atomic per wave and bin
__global__ void __launch_bounds__(256) chain_bin_kernel(ChainArgs a) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  const int lane = (int)(threadIdx.x & 63);
  int b = -1;
  if (r < a.n_reads) {
    const int np = a.n_pos[r];
    if (np == 0) {
      a.n_out[r] = 0;
      a.n_oseed[r] = 0;
      a.n_sw[r] = 0;
    } else {
      b = 0;
      while (b < kLdsBins && np > kBinCap[b]) ++b;
    }
  }
  const uint64_t below = lane ? ~0ull >> (64 - lane) : 0ull;
  for (int k = 0; k <= kLdsBins; ++k) {
    const uint64_t m = __builtin_amdgcn_ballot_w64(b == k);
    if (!m) continue;
    const int leader = __builtin_ctzll(m);
    int at = 0;
    if (lane == leader) at = atomicAdd(a.bin_count + k, __builtin_popcountll(m));
    at = __shfl(at, leader, 64);
    if (b == k) a.bin_list[(int64_t)k * a.n_reads + at + __builtin_popcountll(m & below)] = r;
  }
}

typedef __attribute__((address_space(3))) LChain LdsChain;
typedef __attribute__((address_space(3))) BNode16 LdsNode;
typedef __attribute__((address_space(3))) int32_t LdsI32;
typedef __attribute__((address_space(3))) int64_t LdsI64;


// one wave per read of bin B, its arena in LDS
template <int B>
__global__ void __launch_bounds__(64) chain_build_lds_kernel(ChainArgs a) {
  extern __shared__ __align__(16) char smem[];
  constexpr int cap = kBinCap[B];
  LdsChain* ch = (LdsChain*)(smem);
  LdsNode* nd = (LdsNode*)(smem + (size_t)cap * sizeof(LChain));
  char* tail = smem + (size_t)cap * sizeof(LChain) + lds_nodes_bytes(cap);
  LdsI64* rb = (LdsI64*)tail;
  LdsI64* qi = (LdsI64*)(tail + 8 * (size_t)cap);
  LdsI32* label = (LdsI32*)(tail + 16 * (size_t)cap);
  LdsI32* slist = label + cap;
  LdsI32* ord = slist + cap;
  const int n = a.bin_count[B];
  const int32_t* list = a.bin_list + (int64_t)B * a.n_reads;
  for (int i = (int)blockIdx.x; i < n; i += (int)gridDim.x) chain_read<true>(a, list[i], ch, nd, label, slist, ord, rb, qi, rb);
}

// one wave per read past the largest bin, its arena in global memory
__global__ void __launch_bounds__(64) chain_build_glb_kernel(ChainArgs a) {
  const int n = a.bin_count[kLdsBins];
  const int32_t* list = a.bin_list + (int64_t)kLdsBins * a.n_reads;
  for (int i = (int)blockIdx.x; i < n; i += (int)gridDim.x) {
    const int r = list[i];
    const int64_t base = a.pos_off[r];
    chain_read<false>(a, r, a.lchains + base, a.lnodes + node_base(base, r), a.label + base, a.slist + base, a.ord + base,
               a.rbeg + base, reinterpret_cast<const int64_t*>(a.qinfo) + base,
               reinterpret_cast<int64_t*>(a.kpos) + base);
  }
}

// ---- mem_seed_sw (bwamem.c:580-605) as ksw_align2 tasks, one lane per read
__global__ void __launch_bounds__(256) chain_sw_prep_kernel(ChainArgs a, ChainSw s) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads || a.n_sw[r] == 0) return;
  const int64_t base = a.pos_off[r], q0 = a.seq_off[r];
  const int l_query = (int)(a.seq_off[r + 1] - q0);
  const int64_t l_pac = a.l_pac;
  int64_t t = s.sw_off[r];
  for (int k = 0; k < a.n_out[r]; ++k) {
    const DChain& c = a.ochains[base + k];
    for (int j = 0; j < c.n; ++j, ++t) {
      const int p = a.oslist[base + c.soff + j];
      const int2 qi = a.qinfo[base + p];
      const int64_t sr = (int64_t)a.rbeg[base + p];
      bwagpu_align2_task_t task;
      task.qoff = q0;
      task.toff = t * kSwWin;
      task.qlen = task.tlen = 1;  // a placeholder when the seed is not realigned
      task.xtra = 0;
      task.pad_ = 0;
      int skip = 1;
      if (qi.y < kSwWin) {
        int qb = qi.x, qe = qi.x + qi.y;
        int64_t rb = sr, re = sr + qi.y;
        const int64_t mid = (rb + re) >> 1;
        qb = qb - 50 > 0 ? qb - 50 : 0;  // MEM_SHORT_EXT
        qe = qe + 50 < l_query ? qe + 50 : l_query;
        rb = rb - 50 > 0 ? rb - 50 : 0;
        re = re + 50 < (l_pac << 1) ? re + 50 : (l_pac << 1);
        if (rb < l_pac && l_pac < re) {
          if (mid < l_pac) re = l_pac;
          else rb = l_pac;
        }
        if (qe - qb < kSwWin && re - rb < kSwWin) {
          // bns_fetch_seq (bntseq.c:421-446): clipped to the contig holding mid
          const bool rev = mid >= l_pac;
          const int rid = pos2rid(a, depos(l_pac, mid));
          int64_t fb = a.ann_off[rid], fe = fb + a.ann_len[rid];
          if (rev) {
            const int64_t x = fb;
            fb = (l_pac << 1) - fe;
            fe = (l_pac << 1) - x;
          }
          rb = rb > fb ? rb : fb;
          re = re < fe ? re : fe;
          uint8_t* dst = s.tpool + t * kSwWin;
          for (int64_t x = rb; x < re; ++x) {
            int b;
            if (x < l_pac) {
              b = (a.pac[x >> 2] >> ((~x & 3) << 1)) & 3;
            } else {
              const int64_t f = (l_pac << 1) - 1 - x;
              b = 3 - ((a.pac[f >> 2] >> ((~f & 3) << 1)) & 3);
            }
            dst[x - rb] = (uint8_t)b;
          }
          task.qoff = q0 + qb;
          task.qlen = qe - qb;
          task.tlen = (int32_t)(re - rb);
          task.xtra = BWAGPU_KSW_XSTART;
          skip = 0;
        }
      }
      if (skip) s.tpool[t * kSwWin] = 0;
      s.tasks[t] = task;
      s.skip[t] = skip;
    }
  }
}

// mem_flt_chained_seeds' filter (bwamem.c:612-622)
__global__ void __launch_bounds__(256) chain_sw_apply_kernel(ChainArgs a, ChainSw s) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads || a.n_sw[r] == 0) return;
  const int64_t base = a.pos_off[r];
  const int min_hsp = a.sw_tab[a.seq_off[r + 1] - a.seq_off[r]];
  int64_t t = s.sw_off[r];
  int ns = 0;
  for (int k = 0; k < a.n_out[r]; ++k) {
    DChain& c = a.ochains[base + k];
    const int s0 = c.soff;
    int kk = 0;
    for (int j = 0; j < c.n; ++j, ++t) {
      const int p = a.oslist[base + s0 + j];
      const int sc = s.skip[t] ? -1 : s.res[t].score;
      if (sc < 0 || sc >= min_hsp) {
        a.score[base + p] = sc < 0 ? a.qinfo[base + p].y * a.a : sc;
        a.oslist[base + ns + kk++] = p;  // compacted in place (ns + kk <= s0 + j)
      }
    }
    c.soff = ns;
    c.n = kk;
    ns += kk;
  }
  a.n_oseed[r] = ns;
}

// ---- the chains out, in bwagpu_batch_t's layout (one lane per read)
// one wave per read, a lane per chain (64 at a time): the chains' seed offsets
// by a wave scan of their seed counts, then each lane copies its chain's seeds.
// (A lane per read left the repeat reads' hundreds of chains to one lane: a
// 470 us tail per C2 batch.)
__global__ void __launch_bounds__(256) chain_pack_kernel(ChainArgs a, ChainPack p) {
  const int r = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = (int)(threadIdx.x & 63);
  if (r >= a.n_reads) return;
  const int64_t base = a.pos_off[r];
  const int64_t co0 = p.oc_off[r];
  int64_t carry = p.os_off[r];
  if (lane == 0) {
    p.read_chain_off[r] = (int32_t)co0;
    if (r == a.n_reads - 1) {
      p.read_chain_off[a.n_reads] = (int32_t)p.oc_off[a.n_reads];
      p.chain_seed_off[p.oc_off[a.n_reads]] = (int32_t)p.os_off[a.n_reads];
    }
  }
  const float fr = a.frac_rep[r];
  const int nout = a.n_out[r];
  for (int k0 = 0; k0 < nout; k0 += 64) {
    const int k = k0 + lane;
    const bool valid = k < nout;
    DChain c{};
    if (valid) c = a.ochains[base + k];
    int incl = valid ? c.n : 0;  // inclusive scan of the seed counts
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int y = __shfl_up(incl, o, 64);
      incl += lane >= o ? y : 0;
    }
    if (valid) {
      const int64_t co = co0 + k;
      int64_t so = carry + incl - c.n;
      bwagpu_chain_t out;
      out.pos = c.pos;
      out.rid = c.rid;
      out.n = c.n;
      out.w = c.w;
      out.kept = c.kept;
      out.first = c.first;
      out.is_alt = c.is_alt;
      out.frac_rep = fr;
      out.pad_ = 0;
      p.chains[co] = out;
      p.chain_rid[co] = c.rid;
      p.chain_frac[co] = fr;
      p.chain_seed_off[co] = (int32_t)so;
      for (int j = 0; j < c.n; ++j, ++so) {
        const int q = a.oslist[base + c.soff + j];
        bwagpu_seed_t sd;
        sd.rbeg = (int64_t)a.rbeg[base + q];
        sd.qbeg = a.qinfo[base + q].x;
        sd.len = a.qinfo[base + q].y;
        sd.score = a.score[base + q];
        sd.pad_ = 0;
        p.seeds[so] = sd;
      }
    }
    carry += __shfl(incl, 63, 64);
  }
}

// exclusive scan, one workgroup: each thread sums a contiguous run, eight
// independent loads at a time (one load per iteration left every thread
// waiting on each of its ~65 scattered loads in turn: 110 us per C2 batch)
__global__ void __launch_bounds__(1024) scan_i32_kernel(const int32_t* __restrict__ in, int64_t* __restrict__ out,
                                                        int32_t n) {
  __shared__ int64_t part[1024];
  const int t = (int)threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int b = t * per, e = min(n, b + per);
  int64_t s = 0;
  int i = b;
  for (; i + 8 <= e; i += 8) {
    int v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = in[i + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[k];
  }
  for (; i < e; ++i) s += in[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  i = b;
  for (; i + 8 <= e; i += 8) {
    int v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = in[i + k];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      out[i + k] = run;
      run += v[k];
    }
  }
  for (; i < e; ++i) {
    out[i] = run;
    run += in[i];
  }
  if (t == 1023) out[n] = part[1023];
}

__global__ void __launch_bounds__(256) reg_compact_kernel(int32_t n_reads, const int32_t* __restrict__ rco,
                                                          const int32_t* __restrict__ cso,
                                                          const bwagpu_alnreg_t* __restrict__ regs,
                                                          const int64_t* __restrict__ off,
                                                          bwagpu_alnreg_t* __restrict__ dst) {
  const int r = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const int lane = (int)(threadIdx.x & 63);
  if (r >= n_reads) return;
  const int64_t n = off[r + 1] - off[r];
  if (n == 0) return;
  const bwagpu_alnreg_t* src = regs + cso[rco[r]];
  for (int64_t i = lane; i < n; i += 64) dst[off[r] + i] = src[i];
}

}  // namespace

hipError_t launch_scan_i32(const int32_t* in, int64_t* out, int32_t n, hipStream_t st) {
  hipLaunchKernelGGL(scan_i32_kernel, dim3(1), dim3(1024), 0, st, in, out, n);
  return hipGetLastError();
}

static inline dim3 lanes(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

hipError_t launch_chain_count(const ChainArgs& a, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_count_kernel, lanes(a.n_reads), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_chain_emit(const ChainArgs& a, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_emit_kernel, lanes(64 * (int64_t)a.n_reads), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_chain_build(const ChainArgs& a, hipStream_t st, const ChainStreams& cs) {
  if (a.n_reads <= 0) return hipSuccess;
  hipError_t e = hipMemsetAsync(a.bin_count, 0, sizeof(int32_t) * (kLdsBins + 1), st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(chain_bin_kernel, lanes(a.n_reads), dim3(256), 0, st, a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  // the bins run side by side (the heavy reads' bins are long, serial walks):
  // bin 3 (the longest) on st, bins 2, 0, 1 and the global bin after one
  // another on ONE side stream (with more streams than the process's hardware
  // queues, a second side stream shared st's queue and waited behind bin 3);
  // bin counts stay on the device: each launch's workgroups stride over its
  // bin's list (a resident-size grid for the small bins, fewer for the big)
  if ((e = hipEventRecord(cs.fork, st)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(cs.side[0], cs.fork, 0)) != hipSuccess) return e;
  const int grid[kLdsBins + 1] = {8192, 2048, 512, 256, 256};
  const hipStream_t on[kLdsBins] = {cs.side[0], cs.side[0], cs.side[0], st};
#define BUILD_BIN(B)                                                                                         \
  hipLaunchKernelGGL(chain_build_lds_kernel<B>, dim3(grid[B]), dim3(64), lds_arena(kBinCap[B]), on[B], a); \
  if ((e = hipGetLastError()) != hipSuccess) return e;
  BUILD_BIN(3) BUILD_BIN(2) BUILD_BIN(0) BUILD_BIN(1)
#undef BUILD_BIN
  hipLaunchKernelGGL(chain_build_glb_kernel, dim3(grid[kLdsBins]), dim3(64), 0, cs.side[0], a);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  if ((e = hipEventRecord(cs.join[0], cs.side[0])) != hipSuccess) return e;
  return hipStreamWaitEvent(st, cs.join[0], 0);
}

hipError_t launch_chain_sw_prep(const ChainArgs& a, const ChainSw& s, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_sw_prep_kernel, lanes(a.n_reads), dim3(256), 0, st, a, s);
  return hipGetLastError();
}

hipError_t launch_chain_sw_apply(const ChainArgs& a, const ChainSw& s, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_sw_apply_kernel, lanes(a.n_reads), dim3(256), 0, st, a, s);
  return hipGetLastError();
}

hipError_t launch_chain_pack(const ChainArgs& a, const ChainPack& p, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_pack_kernel, lanes(64 * (int64_t)a.n_reads), dim3(256), 0, st, a, p);
  return hipGetLastError();
}

hipError_t launch_reg_compact(int32_t n_reads, const int32_t* rco, const int32_t* cso, const bwagpu_alnreg_t* regs,
                              const int64_t* off, bwagpu_alnreg_t* dst, hipStream_t st) {
  if (n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(reg_compact_kernel, lanes(64 * (int64_t)n_reads), dim3(256), 0, st, n_reads, rco, cso, regs, off,
                     dst);
  return hipGetLastError();
}

}  // namespace bwagpu
