// chain.hip — seeding's chaining on the device (bwa-flow SeqsToChains after
// the interval search, src/bwa_wrapper.cpp:105-115): mem_chain's body
// (bwa/bwamem.c:260-330), test_and_merge (199-221), mem_chain_flt (336-396)
// and mem_flt_chained_seeds (607-624; mem_seed_sw 580-605 becomes a batch of
// ksw_align2 tasks for align2.hip).  Layout: chain.h.
//
// The work of one read is a strictly sequential walk — every seed either
// joins the chain kb_intervalp finds for it or opens a new one, and the
// chain's last seed decides the next merge — so a read runs on one lane,
// with its kbtree in global memory (a few KB per read, L1/L2 resident while
// the lane works on it).  The kbtree is restated as a B-tree of chain ids with
// the reference's node search, split and in-order traversal (t = 5): chains
// with EQUAL positions exist (tandem repeats), and their order — and which of
// them kb_intervalp returns — follows the tree's shape.  Positions are
// expanded by a wave per read and resolved by bwt_sa (seed.hip) in between.
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

// ---- the kbtree (kbtree.h:54-197, 336-358) over one read's node arena
struct Tree {
  BNode* nd;
  int root, n_nodes, n_keys;

  // first key >= pos (r = 0 if equal, else -1 after stepping back to the last
  // key < pos); past the end the last key with r = 1 (kbtree.h:100-113)
  __device__ int find(int x, int64_t pos, int& r) const {
    const int n = nd[x].n;
    if (n == 0) {
      r = -1;
      return -1;
    }
    int b = 0, e = n;
    while (b < e) {
      const int m = (b + e) >> 1;
      if (nd[x].pos[m] < pos) b = m + 1;
      else e = m;
    }
    if (b == n) {
      r = 1;
      return n - 1;
    }
    r = pcmp(pos, nd[x].pos[b]);
    return r < 0 ? b - 1 : b;
  }

  __device__ int lower(int64_t pos) const {  // kb_intervalp's lower (kbtree.h:130-147)
    int lo = -1, r = 0;
    for (int x = root;;) {
      const int i = find(x, pos, r);
      if (i >= 0 && r == 0) return nd[x].key[i];
      if (i >= 0) lo = nd[x].key[i];
      if (!nd[x].internal) return lo;
      x = nd[x].child[i + 1];
    }
  }

  __device__ void split(int x, int i, int y) {  // __kb_split (kbtree.h:152-167)
    const int z = n_nodes++;
    BNode& Z = nd[z];
    BNode& Y = nd[y];
    BNode& X = nd[x];
    Z.internal = Y.internal;
    Z.n = kBT - 1;
    for (int k = 0; k < kBT - 1; ++k) {
      Z.key[k] = Y.key[kBT + k];
      Z.pos[k] = Y.pos[kBT + k];
    }
    if (Y.internal)
      for (int k = 0; k < kBT; ++k) Z.child[k] = Y.child[kBT + k];
    Y.n = kBT - 1;
    for (int k = X.n; k > i; --k) X.child[k + 1] = X.child[k];
    X.child[i + 1] = z;
    for (int k = X.n; k > i; --k) {
      X.key[k] = X.key[k - 1];
      X.pos[k] = X.pos[k - 1];
    }
    X.key[i] = Y.key[kBT - 1];
    X.pos[i] = Y.pos[kBT - 1];
    ++X.n;
  }

  __device__ void put(int k, int64_t pos) {  // kb_putp (kbtree.h:168-197)
    int r;
    ++n_keys;
    if (nd[root].n == kBN) {
      const int s = n_nodes++;
      nd[s].internal = 1;
      nd[s].n = 0;
      nd[s].child[0] = root;
      split(s, 0, root);
      root = s;
    }
    for (int x = root;;) {
      if (!nd[x].internal) {
        const int i = find(x, pos, r);
        for (int j = nd[x].n - 1; j > i; --j) {
          nd[x].key[j + 1] = nd[x].key[j];
          nd[x].pos[j + 1] = nd[x].pos[j];
        }
        nd[x].key[i + 1] = k;
        nd[x].pos[i + 1] = pos;
        ++nd[x].n;
        return;
      }
      int i = find(x, pos, r) + 1;
      if (nd[nd[x].child[i]].n == kBN) {
        split(x, i, nd[x].child[i]);
        if (pos > nd[x].pos[i]) ++i;
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

// klib introsort (ksort.h:146-226) of chain ids by weight, greater first
// (mem_flt's flt_lt, bwamem.c:333-334), step for step: it is not stable
struct ByW {
  const DChain* c;
  __device__ bool operator()(int x, int y) const { return c[x].w > c[y].w; }
};
__device__ void c_insert(int* s, int* t, ByW lt) {
  for (int* i = s + 1; i < t; ++i)
    for (int* j = i; j > s && lt(*j, *(j - 1)); --j) {
      const int x = *j;
      *j = *(j - 1);
      *(j - 1) = x;
    }
}
__device__ void c_comb(int n, int* a, ByW lt) {
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
        const int x = a[i];
        a[i] = a[i + gap];
        a[i + gap] = x;
        swapped = true;
      }
  } while (swapped || gap > 2);
  if (gap != 1) c_insert(a, a + n, lt);
}
__device__ void c_introsort(int n, int* a, ByW lt) {
  if (n < 1) return;
  if (n == 2) {
    if (lt(a[1], a[0])) {
      const int x = a[0];
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
        c_comb(t - s + 1, a + s, lt);
        t = s;
        continue;
      }
      int i = s, j = t, k = i + ((j - i) >> 1) + 1;
      if (lt(a[k], a[i])) {
        if (lt(a[k], a[j])) k = j;
      } else {
        k = lt(a[j], a[i]) ? i : j;
      }
      const int rp = a[k];
      if (k != t) {
        a[k] = a[t];
        a[t] = rp;
      }
      for (;;) {
        do ++i; while (lt(a[i], rp));
        do --j; while (i <= j && lt(rp, a[j]));
        if (j <= i) break;
        const int x = a[i];
        a[i] = a[j];
        a[j] = x;
      }
      {
        const int x = a[i];
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
        c_insert(a, a + n, lt);
        return;
      }
      --top;
      s = stack[top].l;
      t = stack[top].r;
      d = stack[top].d;
    }
  }
}

// ---- one lane per read: mem_chain's loop, the traversal, mem_chain_flt
__global__ void __launch_bounds__(256) chain_build_kernel(ChainArgs a) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads) return;
  const int np = a.n_pos[r];
  a.n_out[r] = 0;
  a.n_oseed[r] = 0;
  a.n_sw[r] = 0;
  if (np == 0) return;
  const int64_t base = a.pos_off[r];
  DChain* ch = a.chains + base;
  int32_t* label = a.label + base;
  int32_t* slist = a.slist + base;
  int32_t* ord = a.ord + base;
  const uint64_t* rbeg = a.rbeg + base;
  const int2* qi = a.qinfo + base;
  Tree t{a.nodes + node_base(base, r), 0, 1, 0};
  t.nd[0].n = 0;
  t.nd[0].internal = 0;
  int n_ch = 0;
  for (int p = 0; p < np; ++p) {  // bwamem.c:286-311
    const int64_t sr = (int64_t)rbeg[p];
    const int qb = qi[p].x, sl = qi[p].y;
    const int rid = intv2rid(a, sr, sr + sl);
    int lab = -1;
    if (rid >= 0) {
      bool add = true;
      if (t.n_keys) {
        const int lo = t.lower(sr);
        if (lo >= 0) {
          DChain& c = ch[lo];
          // test_and_merge (bwamem.c:199-221)
          const int64_t qend = c.last_qbeg + c.last_len, rend = c.last_rbeg + c.last_len;
          if (rid == c.rid) {
            if (qb >= c.s0_qbeg && qb + sl <= qend && sr >= c.s0_rbeg && sr + sl <= rend) {
              add = false;  // contained: dropped
            } else if (!((c.last_rbeg < a.l_pac || c.s0_rbeg < a.l_pac) && sr >= a.l_pac)) {
              const int64_t x = qb - c.last_qbeg, y = sr - c.last_rbeg;
              if (y >= 0 && x - y <= a.w && y - x <= a.w && x - c.last_len < a.max_chain_gap &&
                  y - c.last_len < a.max_chain_gap) {
                c.last_qbeg = qb;
                c.last_rbeg = sr;
                c.last_len = sl;
                ++c.n;
                lab = lo;
                add = false;
              }
            }
          }
        }
      }
      if (add) {
        DChain& c = ch[n_ch];
        c.pos = c.s0_rbeg = c.last_rbeg = sr;
        c.s0_qbeg = c.last_qbeg = qb;
        c.last_len = sl;
        c.rid = rid;
        c.n = 1;
        c.is_alt = a.is_alt ? (a.is_alt[rid] != 0) : 0;
        c.w = 0;
        c.kept = 0;
        c.first = -1;
        lab = n_ch;
        t.put(n_ch++, sr);
      }
    }
    label[p] = lab;
  }
  // in-order traversal (__kb_traverse, kbtree.h:336-358): the chain order
  int no = 0;
  {
    int sn[32], si[32], top = -1;
    for (int x = t.root;;) {  // the leftmost path
      sn[++top] = x;
      si[top] = 0;
      if (!t.nd[x].internal) break;
      x = t.nd[x].child[0];
    }
    while (top >= 0) {
      const int x = sn[top], i = si[top];
      if (i < t.nd[x].n) {
        ord[no++] = t.nd[x].key[i];
        si[top] = i + 1;
        if (t.nd[x].internal)
          for (int y = t.nd[x].child[i + 1];;) {
            sn[++top] = y;
            si[top] = 0;
            if (!t.nd[y].internal) break;
            y = t.nd[y].child[0];
          }
      } else {
        --top;
      }
    }
  }
  {  // seed lists in kbtree order, each in merge (= processing) order
    int s = 0;
    for (int k = 0; k < no; ++k) {
      DChain& c = ch[ord[k]];
      c.soff = s;
      c.cur = 0;
      s += c.n;
    }
    for (int p = 0; p < np; ++p) {
      const int l = label[p];
      if (l >= 0) slist[ch[l].soff + ch[l].cur++] = p;
    }
  }
  int nout = no;
  if (!a.raw) {  // mem_chain_flt (bwamem.c:336-396)
    int nf = 0;
    for (int k = 0; k < no; ++k) {
      DChain& c = ch[ord[k]];
      // mem_chain_weight (bwamem.c:223-244)
      int64_t end = 0;
      int wq = 0, wr = 0;
      for (int j = 0; j < c.n; ++j) {
        const int2 s = qi[slist[c.soff + j]];
        if (s.x >= end) wq += s.y;
        else if (s.x + s.y > end) wq += (int)(s.x + s.y - end);
        end = end > s.x + s.y ? end : s.x + s.y;
      }
      end = 0;
      for (int j = 0; j < c.n; ++j) {
        const int p = slist[c.soff + j];
        const int64_t rb = (int64_t)rbeg[p];
        const int ln = qi[p].y;
        if (rb >= end) wr += ln;
        else if (rb + ln > end) wr += (int)(rb + ln - end);
        end = end > rb + ln ? end : rb + ln;
      }
      int w = wr < wq ? wr : wq;
      w = w < (1 << 30) ? w : (1 << 30) - 1;
      c.w = w & ((1 << 29) - 1);  // the 29-bit field of mem_chain_t
      c.first = -1;
      c.kept = 0;
      if (c.w >= a.min_chain_weight) ord[nf++] = ord[k];
    }
    c_introsort(nf, ord, ByW{ch});
    nout = 0;
    if (nf > 0) {
      int32_t* kl = label;  // the kept list (label is no longer needed)
      int nk = 0;
      ch[ord[0]].kept = 3;
      kl[nk++] = 0;
      for (int i = 1; i < nf; ++i) {
        DChain& ci = ch[ord[i]];
        const int bi = ci.s0_qbeg, ei = ci.last_qbeg + ci.last_len;
        bool large = false;
        int k;
        for (k = 0; k < nk; ++k) {
          const int j = kl[k];
          DChain& cj = ch[ord[j]];
          const int bj = cj.s0_qbeg, ej = cj.last_qbeg + cj.last_len;
          const int b_max = bj > bi ? bj : bi, e_min = ej < ei ? ej : ei;
          if (e_min > b_max && (!cj.is_alt || ci.is_alt)) {
            const int li = ei - bi, lj = ej - bj;
            const int min_l = li < lj ? li : lj;
            if (e_min - b_max >= min_l * a.mask_level && min_l < a.max_chain_gap) {
              large = true;
              if (cj.first < 0) cj.first = i;
              if (ci.w < cj.w * a.drop_ratio && cj.w - ci.w >= a.min_seed_len << 1) break;
            }
          }
        }
        if (k == nk) {
          kl[nk++] = i;
          ci.kept = large ? 2 : 3;
        }
      }
      for (int i = 0; i < nk; ++i) {
        const DChain& c = ch[ord[kl[i]]];
        if (c.first >= 0) ch[ord[c.first]].kept = 1;
      }
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
  int ns = 0;
  for (int k = 0; k < nout; ++k) ns += ch[ord[k]].n;
  a.n_out[r] = nout;
  a.n_oseed[r] = ns;
  if (!a.raw && nout) {
    const int len = (int)(a.seq_off[r + 1] - a.seq_off[r]);
    if (a.sw_tab[len] >= 0) a.n_sw[r] = ns;  // mem_flt_chained_seeds runs (bwamem.c:609-611)
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
    const DChain& c = a.chains[base + a.ord[base + k]];
    for (int j = 0; j < c.n; ++j, ++t) {
      const int p = a.slist[base + c.soff + j];
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
    DChain& c = a.chains[base + a.ord[base + k]];
    int kk = 0;
    for (int j = 0; j < c.n; ++j, ++t) {
      const int p = a.slist[base + c.soff + j];
      const int sc = s.skip[t] ? -1 : s.res[t].score;
      if (sc < 0 || sc >= min_hsp) {
        a.score[base + p] = sc < 0 ? a.qinfo[base + p].y * a.a : sc;
        a.slist[base + c.soff + kk++] = p;
      }
    }
    c.n = kk;
    ns += kk;
  }
  a.n_oseed[r] = ns;
}

// ---- the chains out, in bwagpu_batch_t's layout (one lane per read)
__global__ void __launch_bounds__(256) chain_pack_kernel(ChainArgs a, ChainPack p) {
  const int r = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (r >= a.n_reads) return;
  const int64_t base = a.pos_off[r];
  int64_t co = p.oc_off[r], so = p.os_off[r];
  p.read_chain_off[r] = (int32_t)co;
  if (r == a.n_reads - 1) {
    p.read_chain_off[a.n_reads] = (int32_t)p.oc_off[a.n_reads];
    p.chain_seed_off[p.oc_off[a.n_reads]] = (int32_t)p.os_off[a.n_reads];
  }
  const float fr = a.frac_rep[r];
  for (int k = 0; k < a.n_out[r]; ++k, ++co) {
    const DChain& c = a.chains[base + a.ord[base + k]];
    bwagpu_chain_t o;
    o.pos = c.pos;
    o.rid = c.rid;
    o.n = c.n;
    o.w = a.raw ? 0 : c.w;
    o.kept = a.raw ? 0 : c.kept;
    o.first = a.raw ? -1 : c.first;
    o.is_alt = c.is_alt;
    o.frac_rep = fr;
    o.pad_ = 0;
    p.chains[co] = o;
    p.chain_rid[co] = c.rid;
    p.chain_frac[co] = fr;
    p.chain_seed_off[co] = (int32_t)so;
    for (int j = 0; j < c.n; ++j, ++so) {
      const int q = a.slist[base + c.soff + j];
      bwagpu_seed_t sd;
      sd.rbeg = (int64_t)a.rbeg[base + q];
      sd.qbeg = a.qinfo[base + q].x;
      sd.len = a.qinfo[base + q].y;
      sd.score = a.score[base + q];
      sd.pad_ = 0;
      p.seeds[so] = sd;
    }
  }
}

// exclusive scan, one workgroup: each thread sums a contiguous run
__global__ void __launch_bounds__(1024) scan_i32_kernel(const int32_t* __restrict__ in, int64_t* __restrict__ out,
                                                        int32_t n) {
  __shared__ int64_t part[1024];
  const int t = (int)threadIdx.x;
  const int per = (n + 1023) / 1024;
  const int b = t * per, e = min(n, b + per);
  int64_t s = 0;
  for (int i = b; i < e; ++i) s += in[i];
  part[t] = s;
  __syncthreads();
  for (int off = 1; off < 1024; off <<= 1) {
    const int64_t v = t >= off ? part[t - off] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int64_t run = t ? part[t - 1] : 0;
  for (int i = b; i < e; ++i) {
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

hipError_t launch_chain_build(const ChainArgs& a, hipStream_t st) {
  if (a.n_reads <= 0) return hipSuccess;
  hipLaunchKernelGGL(chain_build_kernel, lanes(a.n_reads), dim3(256), 0, st, a);
  return hipGetLastError();
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
  hipLaunchKernelGGL(chain_pack_kernel, lanes(a.n_reads), dim3(256), 0, st, a, p);
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
