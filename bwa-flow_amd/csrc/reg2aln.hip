// reg2aln.hip — MI355X (gfx950) CIGAR generation of bwa-flow's SAM stage:
// mem_reg2aln (bwa/bwamem.c:1104-1174) per output region, i.e. infer_bw
// (801-808), the band-doubling loop (1123-1134) over bwa_gen_cigar2
// (bwa/bwa.c:121-207) and its banded global DP with backtrack ksw_global2
// (bwa/ksw.c:504-606), NM and the MD string, the deletion squeeze, soft clips
// and the contig position (bwamem.c:1137-1166, bntseq.h:87-90,
// bntseq.c:349-363).  Called from src/bwa_wrapper.cpp:611/728/736/774.
//
// One wave per region (job):
//  * the query slice and the reference window (2-bit pac gather, reverse
//    strand = complement of the mirrored forward strand; both sequences
//    reversed for reverse-strand regions, bwa.c:136-141) go to LDS once and
//    serve every band try;
//  * DP rows over the target; query columns STRIDED over the lanes (lane r
//    holds eh[] slots j = 64c + r, c < CD), exactly the reference's eh[]
//    update per row: M from the slot's own H(i-1, j-1), E from the slot, F as
//    an exclusive max-plus scan (F_j = max(NEG - (j-lo)e, max_{lo<=k<j}
//    (M_k - oe_ins + k e) - (j-1) e)), the slot's new H(i, j-1) by a one-lane
//    shift; every in-band cell writes its direction byte (h source | E flag
//    << 2 | F flag << 4, ksw.c:552-566) to a row-major ncol-stride matrix in
//    LDS (or, for jobs whose matrix exceeds the LDS bins, in a per-wave HBM
//    slice);
//  * the backtrack (ksw.c:578-590) walks that matrix with the reference's
//    state-dependent bit shift; runs are merged as push_cigar does;
//  * MD/NM: matched runs compared 64 bases per step, mismatches from a ballot.
#include <hip/hip_runtime.h>

#include "engine.h"
#include "reg2aln.h"
#include "wave_ops.h"

namespace bwagpu {

namespace {

constexpr int R2_NEG = -0x40000000;        // ksw.c:489 MINUS_INF
constexpr int R2_SENT = -(3 << 29);        // below every reachable scan value

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ int64_t uni64(int64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)v >> 32));
  return (int64_t)((uint64_t)hi << 32 | lo);
}
__device__ __forceinline__ int wave_sum(int v) {
  v += __shfl_xor(v, 32);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 1);
  return uni(v);
}
// query profile of base q: byte t = mat[t*5 + q] (t = reference base 0..3)
__device__ __forceinline__ uint32_t prof_word(const DevOpt& o, int q) {
  uint32_t p0 = o.qprof[0], p1 = o.qprof[1], p2 = o.qprof[2], p3 = o.qprof[3], p4 = o.qprof[4];
  asm volatile("" : "+s"(p0), "+s"(p1), "+s"(p2), "+s"(p3), "+s"(p4));
  uint32_t v = p0;
  v = q == 1 ? p1 : v;
  v = q == 2 ? p2 : v;
  v = q == 3 ? p3 : v;
  v = q == 4 ? p4 : v;
  return v;
}
__device__ __forceinline__ void wave_sync_lds() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// infer_bw, bwamem.c:801-808
__device__ int infer_bw_dev(int l1, int l2, int score, int a, int q, int r) {
  if (l1 == l2 && l1 * a - score < (q + r - a) << 1) return 0;
  int w = (int)((double)((l1 < l2 ? l1 : l2) * a - score - q) / r + 2.);
  const int d = l1 > l2 ? l1 - l2 : l2 - l1;
  return w < d ? d : w;
}

// ksw_global2's DP over the wave (see the file comment); returns eh[qlen].h
template <int CD>
__device__ int global_dp(const DevOpt& o, int ql, const uint8_t* q, int tl, const uint8_t* r, int w, int ncol,
                         uint8_t* z, int64_t& cells) {
  const int lane = (int)(threadIdx.x & 63);
  const int e_del = o.e_del, e_ins = o.e_ins, oe_del = o.oe_del, oe_ins = o.oe_ins;
  int Hs[CD], Es[CD];
  uint32_t pf[CD];
#pragma unroll
  for (int c = 0; c < CD; ++c) {
    const int j = 64 * c + lane;
    pf[c] = prof_word(o, j < ql ? q[j] : 0);
    Hs[c] = j == 0 ? 0 : (j <= ql && j <= w ? -(o.o_ins + e_ins * j) : R2_NEG);
    Es[c] = R2_NEG;
  }
  int64_t ncells = 0;
  for (int i = 0; i < tl; ++i) {
    const int lo = i > w ? i - w : 0, hi = i + w + 1 < ql ? i + w + 1 : ql;
    const int sh = (r[i] & 3) << 3;
    const int h1init = lo == 0 ? -(o.o_del + e_del * (i + 1)) : R2_NEG;
    const int fdecay = R2_NEG + lo * e_ins;  // + (-j e_ins): F's start value decayed to column j
    uint8_t* zi = z + (size_t)i * ncol - lo;
    int M[CD], EX[CD];
    bool inb[CD];
    int carry = R2_SENT;
#pragma unroll
    for (int c = 0; c < CD; ++c) {
      const int j = 64 * c + lane;
      inb[c] = j >= lo && j < hi;
      M[c] = Hs[c] + __builtin_amdgcn_sbfe((int)pf[c], sh, 8);
      const int u = inb[c] ? M[c] - oe_ins + j * e_ins : R2_SENT;
      int x = c == 0 ? u : max(u, carry);
      x = max_bc31(max_bc15(max_shr8(max_shr4(max_shr2(max_shr1(x))))));
      EX[c] = dpp<DPP_WAVE_SHR1>(carry, x);
      if (c + 1 < CD) carry = __builtin_amdgcn_readlane(x, 63);
    }
    int prev63 = h1init;
#pragma unroll
    for (int c = 0; c < CD; ++c) {
      const int j = 64 * c + lane;
      const int m = M[c], e = Es[c];
      const int f = max(fdecay - j * e_ins, EX[c] - (j - 1) * e_ins);
      uint32_t d = m >= e ? 0u : 1u;
      int h = m >= e ? m : e;
      d = h >= f ? d : 2u;
      h = h >= f ? h : f;
      const int te = m - oe_del, ed = e - e_del;
      d |= ed > te ? 4u : 0u;
      const int tf = m - oe_ins, fd = f - e_ins;
      d |= fd > tf ? 32u : 0u;
      if (inb[c]) zi[j] = (uint8_t)d;
      // H(i, j-1) into slot j: lane 0 of segment 0 (and slot lo) takes h1init
      const int hsh = dpp<DPP_WAVE_SHR1>(prev63, h);
      if (c + 1 < CD) prev63 = __builtin_amdgcn_readlane(h, 63);
      const bool upd = (j >= lo && j <= hi) || j == hi;
      Hs[c] = upd ? (j <= lo ? h1init : hsh) : Hs[c];
      Es[c] = inb[c] ? (ed > te ? ed : te) : (j == hi ? R2_NEG : Es[c]);
    }
    ncells += hi > lo ? hi - lo : 0;
  }
  cells += ncells;
  // eh[qlen].h: slot ql lives in lane ql & 63 of segment ql >> 6
  int s = 0;
#pragma unroll
  for (int c = 0; c < CD; ++c) s = (ql >> 6) == c ? Hs[c] : s;
  return __builtin_amdgcn_readlane(s, ql & 63);
}

// The same DP in the BAND frame, for bands of 2w+1 <= 64 CDB columns: lane
// position p (segment c, p = 64c + lane) holds column j = i - w + p of row
// i, so the band never moves relative to the lanes.  Per row:
//  * M(i,j) needs H(i-1, j-1), which sits at the same position p of the
//    previous row: no shift; the query base of a position changes every row
//    (one LDS byte per lane);
//  * E(i,j) is the E written at column j by row i-1, one position up (p+1):
//    a one-lane shift down of the new E values, NEG entering at the top
//    (eh[end].e = MINUS_INF, ksw.c:569);
//  * eh[j+1].h for the next row is H(i, j) at the same position, except the
//    row's first slot, which takes h1 (ksw.c:533-534);
//  * eh[qlen].h, the score, is followed as a uniform value.
template <int CDB>
__device__ int band_dp(const DevOpt& o, int ql, const uint8_t* q, int tl, const uint8_t* r, int w, int ncol,
                       uint8_t* z, int64_t& cells) {
  const int lane = (int)(threadIdx.x & 63);
  const int e_del = o.e_del, e_ins = o.e_ins, oe_del = o.oe_del, oe_ins = o.oe_ins;
  int EH[CDB], EE[CDB];
#pragma unroll
  for (int c = 0; c < CDB; ++c) {
    const int j = 64 * c + lane - w;  // row 0
    EH[c] = j == 0 ? 0 : (j >= 1 && j <= ql && j <= w ? -(o.o_ins + e_ins * j) : R2_NEG);
    EE[c] = R2_NEG;
  }
  int sc = ql == 0 ? 0 : (ql <= w ? -(o.o_ins + e_ins * ql) : R2_NEG);  // eh[qlen].h
  int64_t ncells = 0;
  for (int i = 0; i < tl; ++i) {
    const int lo = i > w ? i - w : 0, hi = i + w + 1 < ql ? i + w + 1 : ql;
    const int sh = (r[i] & 3) << 3;
    const int h1init = lo == 0 ? -(o.o_del + e_del * (i + 1)) : R2_NEG;
    const int fdecay = R2_NEG + lo * e_ins;
    uint8_t* zi = z + (size_t)i * ncol - lo;
    int M[CDB], EX[CDB], J[CDB];
    bool inb[CDB];
    int carry = R2_SENT;
#pragma unroll
    for (int c = 0; c < CDB; ++c) {
      const int j = i - w + 64 * c + lane;
      J[c] = j;
      inb[c] = j >= lo && j < hi;
      const int qb = inb[c] ? q[j] : 0;
      M[c] = EH[c] + __builtin_amdgcn_sbfe((int)prof_word(o, qb), sh, 8);
      const int u = inb[c] ? M[c] - oe_ins + j * e_ins : R2_SENT;
      int x = c == 0 ? u : max(u, carry);
      x = max_bc31(max_bc15(max_shr8(max_shr4(max_shr2(max_shr1(x))))));
      EX[c] = dpp<DPP_WAVE_SHR1>(carry, x);
      if (c + 1 < CDB) carry = __builtin_amdgcn_readlane(x, 63);
    }
    int En[CDB], Hn[CDB];
#pragma unroll
    for (int c = 0; c < CDB; ++c) {
      const int j = J[c];
      const int m = M[c], e = EE[c];
      const int f = max(fdecay - j * e_ins, EX[c] - (j - 1) * e_ins);
      uint32_t d = m >= e ? 0u : 1u;
      int h = m >= e ? m : e;
      d = h >= f ? d : 2u;
      h = h >= f ? h : f;
      const int te = m - oe_del, ed = e - e_del;
      d |= ed > te ? 4u : 0u;
      const int tf = m - oe_ins, fd = f - e_ins;
      d |= fd > tf ? 32u : 0u;
      if (inb[c]) zi[j] = (uint8_t)d;
      Hn[c] = h;
      En[c] = inb[c] ? (ed > te ? ed : te) : R2_NEG;
    }
    // eh[qlen].h after this row (ksw.c:568): H(i, ql-1), or h1 when the band is empty
    if (hi == ql) {
      const int pq = ql - 1 - i + w;  // position of column ql-1
      int v = 0;
#pragma unroll
      for (int c = 0; c < CDB; ++c) v = (pq >> 6) == c ? Hn[c] : v;
      sc = lo < hi ? __builtin_amdgcn_readlane(v, pq & 63) : h1init;
    }
    // next row's frame: EH at the same position (h1 at column lo-1), EE one position down
    int nxt = R2_NEG;
#pragma unroll
    for (int c = CDB - 1; c >= 0; --c) {
      EH[c] = J[c] == lo - 1 ? h1init : Hn[c];
      const int dn = __builtin_amdgcn_mov_dpp(En[c], 0x130, 0xF, 0xF, false);  // wave_shl:1 (lane l <- l+1)
      EE[c] = lane == 63 ? nxt : dn;
      if (c > 0) nxt = __builtin_amdgcn_readlane(En[c], 0);
    }
    ncells += hi > lo ? hi - lo : 0;
  }
  cells += ncells;
  return sc;
}

__device__ __forceinline__ void put_md_int(char* md, int& ml, int cap, int v, bool& ovf) {
  char b[12];
  int n = 0;
  do {
    b[n++] = (char)('0' + v % 10);
    v /= 10;
  } while (v);
  if (ml + n >= cap) {
    ovf = true;
    return;
  }
  while (n) md[ml++] = b[--n];
}
__device__ __forceinline__ void put_md_chr(char* md, int& ml, int cap, char ch, bool& ovf) {
  if (ml + 1 >= cap) {
    ovf = true;
    return;
  }
  md[ml++] = ch;
}

}  // namespace

template <int CD>
__global__ void __launch_bounds__(256) reg2aln_kernel(DevOpt o, DevRef ref, R2AArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = (int)(threadIdx.x & 63);
  const int wib = uni((int)(threadIdx.x >> 6)), wpb = (int)(blockDim.x >> 6);
  const int wave = (int)blockIdx.x * wpb + wib, nwaves = (int)gridDim.x * wpb;
  uint8_t* const wl = lds + (size_t)wib * a.lds_per_wave;
  uint8_t* const q = wl;                                               // qcap bytes
  uint8_t* const r = wl + a.qcap;                                      // rcap bytes
  uint32_t* const ops = reinterpret_cast<uint32_t*>(wl + a.qcap + a.rcap);  // ocap words
  uint8_t* const z = a.zglob ? a.zglob + (int64_t)wave * a.zstride : wl + a.qcap + a.rcap + 4 * a.ocap;
  const int64_t l_pac = ref.l_pac, two = l_pac << 1;
  const int wmax = o.w << 2;
  int64_t t_cells = 0, t_rows = 0, t_calls = 0;
  for (int li = wave; li < a.n; li += nwaves) {
    const int k = uni(a.list[li]);
    const bwagpu_reg2aln_task_t* tp = a.tasks + k;
    const int64_t rb = uni64(tp->rb), re = uni64(tp->re), qoff = uni64(tp->qoff);
    const int l_seq = uni(tp->l_seq), qb = uni(tp->qb), qe = uni(tp->qe), truesc = uni(tp->truesc),
              wreg = uni(tp->w);
    bwagpu_aln_t res{};
    if (rb < 0 || re < 0) {  // bwamem.c:1112-1115
      res.rid = -1;
      res.pos = -1;
      res.status = BWAGPU_ALN_UNMAPPED;
      if (lane == 0) a.out[k] = res;
      continue;
    }
    const int lq = qe - qb;
    const int64_t rl64 = re - rb;
    // bwa_gen_cigar2's rejections (bwa.c:133-135): none depends on the band
    const int64_t beg = rb < 0 ? 0 : rb, end = re > two ? two : re;
    if (lq <= 0 || rb >= re || (rb < l_pac && re > l_pac) || !(beg >= l_pac || end <= l_pac) || end - beg != rl64) {
      int w2 = max(infer_bw_dev(lq, (int)rl64, truesc, o.a, o.o_del, o.e_del),
                   infer_bw_dev(lq, (int)rl64, truesc, o.a, o.o_ins, o.e_ins));
      if (w2 > o.w) w2 = min(w2, wreg);
      res.w = min(w2, wmax);
      res.NM = -1;
      res.status = BWAGPU_ALN_NO_CIGAR;
      t_calls += 1;
      if (lane == 0) a.out[k] = res;
      continue;
    }
    const int rl = (int)rl64;
    const bool rev = rb >= l_pac;
    // query slice and reference window into LDS (reversed for the reverse strand)
    for (int x = lane; x < lq; x += 64) q[x] = a.qpool[qoff + qb + (rev ? lq - 1 - x : x)];
    for (int x = lane; x < rl; x += 64) {
      const int64_t p = rev ? re - 1 - x : rb + x;
      const int64_t f = p >= l_pac ? two - 1 - p : p;
      const int b = (ref.pac[f >> 2] >> ((~f & 3) << 1)) & 3;
      r[x] = (uint8_t)(p >= l_pac ? 3 - b : b);
    }
    wave_sync_lds();
    // the band loop (bwamem.c:1122-1134)
    int w2 = max(infer_bw_dev(lq, rl, truesc, o.a, o.o_del, o.e_del),
                 infer_bw_dev(lq, rl, truesc, o.a, o.o_ins, o.e_ins));
    if (w2 > o.w) w2 = min(w2, wreg);
    int last = -(1 << 30), score = 0, wcall = 0, tries = 0, wdp = 0, ncol = 0;
    bool ungapped = false;
    for (;;) {
      w2 = min(w2, wmax);
      wcall = w2;
      t_calls += 1;
      if (lq == rl && w2 == 0) {  // bwa.c:142-150
        int s = 0;
        for (int x = lane; x < lq; x += 64) s += o.mat[r[x] * 5 + q[x]];
        score = wave_sum(s);
        ungapped = true;
      } else {  // bwa.c:152-165
        const int half = (lq + 1) >> 1;
        const int mi = (int)((double)(half * o.mat[0] - o.o_ins) / o.e_ins + 1.);
        const int md = (int)((double)(half * o.mat[0] - o.o_del) / o.e_del + 1.);
        int mg = max(max(mi, md), 1);
        const int dl = lq > rl ? lq - rl : rl - lq;
        int w = min((mg + dl + 1) >> 1, w2);
        w = max(w, dl + 3);
        wdp = w;
        ncol = lq < 2 * w + 1 ? lq : 2 * w + 1;
        ungapped = false;
        if (2 * w + 1 <= 64)
          score = uni(band_dp<1>(o, lq, q, rl, r, w, ncol, z, t_cells));
        else if (2 * w + 1 <= 128 && CD >= 2)
          score = uni(band_dp<(CD >= 2 ? 2 : 1)>(o, lq, q, rl, r, w, ncol, z, t_cells));
        else
          score = uni(global_dp<CD>(o, lq, q, rl, r, w, ncol, z, t_cells));
        t_rows += rl;
      }
      if (score == last || w2 == wmax) break;
      last = score;
      w2 <<= 1;
      if (!(++tries < 3 && score < truesc - o.a)) break;
    }
    res.score = score;
    res.w = wcall;
    // ---- CIGAR of the last try: backtrack (ksw.c:578-590), reversed runs in ops[]
    int nops = 0;
    if (ungapped) {
      if (lane == 0) ops[0] = (uint32_t)lq << 4;
      nops = 1;
    } else {
      wave_sync_lds();  // direction bytes of every lane visible
      // Runs of one state are taken 64 cells at a time: in state s the walk
      // moves diagonally (s = 0, M), up (1, D) or left (2, I) and stays in s
      // while the cell's bits for s (>> 2s) read s again; lane l looks at the
      // l-th cell of the run, a ballot finds where it ends.  Cells outside the
      // row's band end a run (the serial step then reads what the reference
      // reads).
      int i = rl - 1, kk = min(i + wdp + 1, lq) - 1, st = 0, cop = -1, clen = 0;
      auto emit = [&](int op, int len) {
        if (op == cop) {
          clen += len;
        } else {
          if (clen && lane == 0) ops[nops] = (uint32_t)clen << 4 | (uint32_t)cop;
          nops += clen ? 1 : 0;
          cop = op;
          clen = len;
        }
      };
      while (i >= 0 && kk >= 0) {
        const int di = st != 2, dk = st != 1;
        const int il = i - lane * di, kl = kk - lane * dk;
        const int lol = il > wdp ? il - wdp : 0, hil = min(il + wdp + 1, lq);
        const bool valid = il >= 0 && kl >= lol && kl < hil;
        const int d = valid ? (int)z[(size_t)il * ncol + (kl - lol)] : 0;
        const bool stop = !valid || ((d >> (st << 1)) & 3) != st;
        const uint64_t sb = __builtin_amdgcn_ballot_w64(stop);
        const int f = sb ? __builtin_ctzll(sb) : 64;
        if (f) {
          emit(st == 0 ? 0 : (st == 1 ? 2 : 1), f);
          i -= f * di;
          kk -= f * dk;
        }
        if (f < 64 && i >= 0 && kk >= 0) {  // one serial step at the run's end (reference addressing)
          const int lo_i = i > wdp ? i - wdp : 0;
          // a walk that leaves the band reads outside the row in the reference
          // (undefined there); here the index stays inside the matrix
          int64_t zi = (int64_t)i * ncol + (kk - lo_i);
          zi = zi < 0 ? 0 : (zi >= (int64_t)ncol * rl ? (int64_t)ncol * rl - 1 : zi);
          const int dd = uni((int)z[zi]);
          st = (dd >> (st << 1)) & 3;
          emit(st == 0 ? 0 : (st == 1 ? 2 : 1), 1);
          i -= st != 2;
          kk -= st != 1;
        }
      }
      auto push = emit;
      // the ends (ksw.c:591-592), then the last run
      if (i >= 0) push(2, i + 1);
      if (kk >= 0) push(1, kk + 1);
      if (clen && lane == 0) ops[nops] = (uint32_t)clen << 4 | (uint32_t)cop;
      nops += clen ? 1 : 0;
      // forward order
      for (int x = lane; x < nops >> 1; x += 64) {
        const uint32_t t0 = ops[x];
        ops[x] = ops[nops - 1 - x];
        ops[nops - 1 - x] = t0;
      }
    }
    wave_sync_lds();
    // ---- NM and MD (bwa.c:167-199), MD written straight to the job's slot
    char* const mdo = a.md + (int64_t)k * a.max_md;
    const bool fwd = rb < l_pac;
    int x = 0, y = 0, u = 0, nmm = 0, ngap = 0, ml = 0;
    bool ovf = false;
    for (int kop = 0; kop < nops; ++kop) {
      const uint32_t cv = uni((int)ops[kop]);
      const int op = (int)(cv & 0xf), len = (int)(cv >> 4);
      if (op == 0) {
        for (int s0 = 0; s0 < len; s0 += 64) {
          const int n = min(64, len - s0);
          const bool mm = lane < n && q[x + s0 + lane] != r[y + s0 + lane];
          uint64_t bits = __builtin_amdgcn_ballot_w64(mm);
          int cur = 0;
          while (bits) {
            const int b = __builtin_ctzll(bits);
            bits &= bits - 1;
            u += b - cur;
            const int rbse = uni((int)r[y + s0 + b]);
            if (lane == 0) {
              put_md_int(mdo, ml, a.max_md, u, ovf);
              put_md_chr(mdo, ml, a.max_md, "ACGTN"[fwd ? rbse : (rbse < 4 ? 3 - rbse : 4)], ovf);
            }
            ++nmm;
            u = 0;
            cur = b + 1;
          }
          u += n - cur;
        }
        x += len;
        y += len;
      } else if (op == 2) {
        if (kop > 0 && kop < nops - 1) {
          if (lane == 0) {
            put_md_int(mdo, ml, a.max_md, u, ovf);
            put_md_chr(mdo, ml, a.max_md, '^', ovf);
            for (int b = 0; b < len; ++b) {
              const int rbse = r[y + b];
              put_md_chr(mdo, ml, a.max_md, "ACGTN"[fwd ? rbse : (rbse < 4 ? 3 - rbse : 4)], ovf);
            }
          }
          u = 0;
          ngap += len;
        }
        y += len;
      } else if (op == 1) {
        x += len;
        ngap += len;
      }
    }
    if (lane == 0) {
      put_md_int(mdo, ml, a.max_md, u, ovf);
      if (!ovf) mdo[ml] = 0;
    }
    ovf = uni(ovf ? 1 : 0) != 0;
    ml = uni(ml);
    res.NM = nmm + ngap;
    // ---- squeeze / clip / position (bwamem.c:1137-1166)
    int64_t pos = rb < l_pac ? rb : re - 1;
    const int is_rev = pos >= l_pac;
    if (is_rev) pos = two - 1 - pos;
    int s0 = 0, n = nops;
    if (n > 0) {
      const uint32_t f0 = uni((int)ops[0]), fl = uni((int)ops[n - 1]);
      if ((f0 & 0xf) == 2) {
        pos += f0 >> 4;
        s0 = 1;
        --n;
      } else if ((fl & 0xf) == 2) {
        --n;
      }
    }
    int clip5 = 0, clip3 = 0;
    if (qb != 0 || qe != l_seq) {
      clip5 = is_rev ? l_seq - qe : qb;
      clip3 = is_rev ? qb : l_seq - qe;
    }
    const int total = n + (clip5 != 0) + (clip3 != 0);
    if (ovf || total > a.max_ops) {
      res.status = BWAGPU_ALN_OVERFLOW;
      if (lane == 0) a.out[k] = res;
      continue;
    }
    uint32_t* const co = a.cigar + (int64_t)k * a.max_ops;
    const int c0 = clip5 != 0;
    for (int e = lane; e < n; e += 64) co[c0 + e] = ops[s0 + e];
    if (lane == 0) {
      if (clip5) co[0] = (uint32_t)clip5 << 4 | 3;
      if (clip3) co[c0 + n] = (uint32_t)clip3 << 4 | 3;
    }
    // bns_pos2rid (bntseq.c:349-363)
    int left = 0, mid = 0, right = ref.n_seqs;
    if (pos >= l_pac) {
      mid = -1;
    } else {
      while (left < right) {
        mid = (left + right) >> 1;
        if (pos >= ref.ann_offset[mid]) {
          if (mid == ref.n_seqs - 1) break;
          if (pos < ref.ann_offset[mid + 1]) break;
          left = mid + 1;
        } else {
          right = mid;
        }
      }
    }
    res.rid = mid;
    res.pos = mid >= 0 ? pos - ref.ann_offset[mid] : pos;
    res.is_rev = is_rev;
    res.n_cigar = total;
    res.md_len = ml;
    res.status = BWAGPU_ALN_OK;
    if (lane == 0) a.out[k] = res;
  }
  if (a.stats && lane == 0) {
    if (t_cells) atomicAdd((unsigned long long*)&a.stats[ST_CELLS], (unsigned long long)t_cells);
    if (t_rows) atomicAdd((unsigned long long*)&a.stats[ST_ROWS], (unsigned long long)t_rows);
    if (t_calls) atomicAdd((unsigned long long*)&a.stats[ST_CALLS], (unsigned long long)t_calls);
  }
}

const int kR2CD[kR2Buckets] = {1, 2, 3, 4, 8, 16};

int r2_resident_waves(int cd, size_t lds_per_block, int wpb) {
  int dev = 0, ncu = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 4096;
  if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 4096;
  hipError_t e = hipErrorInvalidValue;
  switch (cd) {
#define R2_OCC(C) \
  case C: e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reg2aln_kernel<C>, 64 * wpb, lds_per_block); break;
    R2_OCC(1) R2_OCC(2) R2_OCC(3) R2_OCC(4) R2_OCC(8) R2_OCC(16)
#undef R2_OCC
  }
  if (e != hipSuccess || per < 1) per = 1;
  return per * ncu * wpb;
}

hipError_t launch_reg2aln(int cd, const DevOpt& o, const DevRef& ref, const R2AArgs& a, int n_blocks, int wpb,
                          hipStream_t st) {
  const size_t lds = (size_t)wpb * a.lds_per_wave;
  switch (cd) {
#define R2_LAUNCH(C)                                                                                   \
  case C:                                                                                              \
    hipLaunchKernelGGL((reg2aln_kernel<C>), dim3(n_blocks), dim3(64 * wpb), lds, st, o, ref, a);            \
    return hipGetLastError();
    R2_LAUNCH(1) R2_LAUNCH(2) R2_LAUNCH(3) R2_LAUNCH(4) R2_LAUNCH(8) R2_LAUNCH(16)
#undef R2_LAUNCH
  }
  return hipErrorInvalidValue;
}

}  // namespace bwagpu
