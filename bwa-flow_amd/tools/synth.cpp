// synth.cpp — synthetic workload generator for bench.py (lib/libsynth.so).
//
// There is no network and no GRCh38/chr21 in this environment, so the
// benchmark configurations of BASELINE.json are reproduced with seeded
// synthetic data of the same shape:
//   * a reference of the requested length in bwa's forward 2-bit pac layout
//     (bntseq.c:225, l_pac/4+1 bytes) split into contigs, iid ACGT plus
//     diverged interspersed repeats and tandem repeats;
//   * read pairs (~N(400,40) fragments, 0.8% substitutions, 0.1% 1-3 bp
//     indels, 0.05% N) of 100/150/250 bp or a mix;
//   * per read, the chains bwa's SeqsToChains would hand to ChainsToRegions
//     on a unique reference: every maximal exact match of >= min_seed_len bases
//     between the read and its true origin becomes a seed {rbeg in the 2-strand
//     coordinate, qbeg, len, score=len} (bwamem.c:294 sets score = len), all
//     seeds of a read form one chain on the origin contig; a fraction of reads
//     additionally get a repeat chain (a seed copied to another locus), and
//     chimeric reads get two chains.
// This is input generation only; the stage under test is libbwagpu.so.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <thread>
#include <vector>

#include "bwagpu.h"

namespace {

struct Rng {
  uint64_t s;
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  double u() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  int i(int n) { return (int)(u() * n); }
  double n() {
    double a = u() + 1e-300, b = u();
    return sqrt(-2 * log(a)) * cos(2 * M_PI * b);
  }
};

inline int get2(const uint8_t* pac, int64_t k) { return pac[k >> 2] >> ((~k & 3) << 1) & 3; }
inline void set2(uint8_t* pac, int64_t k, int c) { pac[k >> 2] |= (uint8_t)(c << ((~k & 3) << 1)); }
inline void put2(uint8_t* pac, int64_t k, int c) {  // overwrite
  const int sh = (~k & 3) << 1;
  pac[k >> 2] = (uint8_t)((pac[k >> 2] & ~(3 << sh)) | (c << sh));
}

// GRCh38 primary assembly: chr1..chr22, chrX, chrY, chrM lengths (the
// no-alt analysis set has these 25 plus 170 unlocalized/unplaced contigs,
// 195 sequences, l_pac = 3,099,734,149).
constexpr int kG38Primary = 25, kG38Contigs = 195;
constexpr int64_t kG38Len = 3099734149LL;
const int64_t kG38PrimaryLen[kG38Primary] = {
    248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636, 138394717,
    133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345,  83257441,  80373285,
    58617616,  64444167,  46709983,  50818468,  156040895, 57227415,  16569};

}  // namespace

extern "C" {

// The genome of the reference-seeded workloads (oracle/gen_golden.c
// make_genome, the bench's C2 fixture tests/golden/c2_refseed.npz): total_len
// bases in three contigs (1 Mb: 500k/300k/200k; otherwise 50/30/20 %), iid ACGT
// from splitmix64(seed), then per Mb 10 repeat families x 4 copies (1 %
// diverged), 30 tandem repeats and 12 N runs — and the pac bwa builds from it:
// each N becomes lrand48() & 3 after srand48(11) (bntseq.c:261,290-291; the
// drand48 generator is X' = 0x5DEECE66D X + 11 mod 2^48, lrand48 = X >> 17).
// pac: total_len/4+1 bytes; ann_off/ann_len: 3 entries.
int golden_genome(uint64_t seed, int64_t total_len, uint8_t* pac, int64_t* ann_off, int32_t* ann_len) {
  if (total_len < 1000 || !pac) return -1;
  int64_t ctg[3] = {500000, 300000, 200000};
  if (total_len != 1000000) {
    ctg[0] = total_len / 2;
    ctg[1] = total_len * 3 / 10;
    ctg[2] = total_len - ctg[0] - ctg[1];
  }
  const int64_t L = total_len;
  static const char kB[4] = {0, 1, 2, 3};
  Rng g{seed};
  std::vector<uint8_t> s((size_t)L);  // 0..3, 4 = N
  for (auto& b : s) b = kB[g.next() & 3];
  auto per_mb = [L](int k) { return (int)(k * (double)L / 1e6 + 0.5); };
  const int n_fam = per_mb(10), n_tan = per_mb(30), n_nrun = per_mb(12);
  for (int fam = 0; fam < n_fam; ++fam) {
    const int len = 300 + g.i(2700);
    const int64_t src = (int64_t)(g.u() * (double)(L - len));
    for (int c = 0; c < 4; ++c) {
      const int64_t dst = (int64_t)(g.u() * (double)(L - len));
      for (int k = 0; k < len; ++k) s[dst + k] = g.u() < 0.01 ? kB[g.next() & 3] : s[src + k];
    }
  }
  for (int t = 0; t < n_tan; ++t) {
    const int per = 2 + g.i(49);
    const int len = 200 + g.i(800);
    const int64_t dst = (int64_t)(g.u() * (double)(L - len));
    for (int k = per; k < len; ++k) s[dst + k] = g.u() < 0.005 ? kB[g.next() & 3] : s[dst + k - per];
  }
  for (int t = 0; t < n_nrun; ++t) {
    const int len = 10 + g.i(300);
    const int64_t dst = (int64_t)(g.u() * (double)(L - len));
    memset(s.data() + dst, 4, (size_t)len);
  }
  uint64_t x = (11ull << 16) | 0x330Eull;  // srand48(11)
  memset(pac, 0, (size_t)(L / 4 + 1));
  for (int64_t k = 0; k < L; ++k) {
    int c = s[k];
    if (c >= 4) {
      x = (0x5DEECE66Dull * x + 0xBull) & ((1ull << 48) - 1);
      c = (int)(x >> 17) & 3;
    }
    set2(pac, k, c);
  }
  int64_t off = 0;
  for (int i = 0; i < 3; ++i) {
    if (ann_off) ann_off[i] = off;
    if (ann_len) ann_len[i] = (int32_t)ctg[i];
    off += ctg[i];
  }
  return 0;
}

// Build a reference of total_len bases in n_ctg contigs.  pac must hold
// total_len/4+1 zeroed bytes; ann_off/ann_len get n_ctg entries.
int synth_ref(uint64_t seed, int64_t total_len, int n_ctg, uint8_t* pac, int64_t* ann_off, int32_t* ann_len) {
  if (total_len <= 0 || n_ctg <= 0 || !pac) return -1;
  Rng g{seed};
  std::vector<uint8_t> s((size_t)total_len);
  for (auto& b : s) b = (uint8_t)(g.next() & 3);
  // interspersed repeats (~2% of the genome), 1% diverged
  int64_t rep = total_len / 50;
  for (int64_t done = 0; done < rep;) {
    int len = 300 + g.i(2700);
    if (len >= total_len / 4) break;
    int64_t src = (int64_t)(g.u() * (double)(total_len - len));
    for (int c = 0; c < 3; ++c) {
      int64_t dst = (int64_t)(g.u() * (double)(total_len - len));
      for (int k = 0; k < len; ++k) s[dst + k] = g.u() < 0.01 ? (uint8_t)(g.next() & 3) : s[src + k];
      done += len;
    }
  }
  // tandem repeats
  for (int64_t t = 0; t < total_len / 100000 + 1; ++t) {
    int per = 2 + g.i(49), len = 200 + g.i(800);
    if (len >= total_len) break;
    int64_t dst = (int64_t)(g.u() * (double)(total_len - len));
    for (int k = per; k < len; ++k) s[dst + k] = g.u() < 0.005 ? (uint8_t)(g.next() & 3) : s[dst + k - per];
  }
  memset(pac, 0, (size_t)(total_len / 4 + 1));
  for (int64_t k = 0; k < total_len; ++k) set2(pac, k, s[k]);
  int64_t off = 0;
  for (int c = 0; c < n_ctg; ++c) {
    int64_t len = total_len / n_ctg + (c == n_ctg - 1 ? total_len % n_ctg : 0);
    ann_off[c] = off;
    ann_len[c] = (int32_t)len;
    off += len;
  }
  return 0;
}

// The C3 regime's reference (BASELINE.json configs[2]): a GRCh38-shaped
// genome.  grch38_layout fills the 195-entry contig table (the 25 primary
// chromosomes at their real lengths, then 170 small contigs of seeded lengths
// that bring the total to GRCh38's l_pac) and returns the contig count;
// grch38_genome fills pac (l_pac/4+1 bytes) with seeded content: iid bases
// (a counter-based splitmix64 per 32-base word, so threads do not change the
// result), then interspersed repeat families (4 copies, 1 % diverged) and
// tandem repeats.  Forward coordinates reach 3.1e9 (> 2^31) and 2-strand
// coordinates 6.2e9 (> 2^32); the pac is 0.78 GB (outside the MALL).
int grch38_layout(int64_t* ann_off, int32_t* ann_len, int64_t* l_pac) {
  int64_t len[kG38Contigs];
  int64_t prim = 0;
  for (int i = 0; i < kG38Primary; ++i) prim += (len[i] = kG38PrimaryLen[i]);
  Rng g{195};
  int64_t raw = 0;
  for (int i = kG38Primary; i < kG38Contigs; ++i) raw += (len[i] = 1000 + g.i(300000));
  const int64_t want = kG38Len - prim;  // 11,447,748
  int64_t acc = 0;
  for (int i = kG38Primary; i < kG38Contigs; ++i) {
    len[i] = i + 1 < kG38Contigs ? std::max<int64_t>(1000, len[i] * want / raw) : want - acc;
    acc += len[i];
  }
  int64_t off = 0;
  for (int i = 0; i < kG38Contigs; ++i) {
    if (ann_off) ann_off[i] = off;
    if (ann_len) ann_len[i] = (int32_t)len[i];
    off += len[i];
  }
  if (l_pac) *l_pac = off;
  return kG38Contigs;
}

int grch38_genome(uint64_t seed, uint8_t* pac, int n_threads) {
  if (!pac) return -1;
  const int64_t L = kG38Len, nbytes = L / 4 + 1, nwords = (nbytes + 7) / 8;
  n_threads = std::max(1, std::min(n_threads, 64));
  std::vector<std::thread> th;
  for (int t = 0; t < n_threads; ++t)
    th.emplace_back([=] {
      for (int64_t w = nwords * t / n_threads; w < nwords * (t + 1) / n_threads; ++w) {
        Rng r{seed * 0x2545F4914F6CDD1DULL + (uint64_t)w * 0x9E3779B97F4A7C15ULL};
        const uint64_t v = r.next();
        const int64_t b0 = w * 8, nb = std::min<int64_t>(8, nbytes - b0);
        memcpy(pac + b0, &v, (size_t)nb);
      }
    });
  for (auto& x : th) x.join();
  // bits past the last base are zero, as in the pac bwa builds
  const int rem = (int)(L & 3);
  pac[L >> 2] &= (uint8_t)(rem ? 0xff00 >> (2 * rem) : 0);
  Rng g{seed ^ 0xC3C3C3C3ULL};
  for (int fam = 0; fam < 3000; ++fam) {  // ~20 Mb of interspersed repeats
    const int len = 300 + g.i(2700);
    const int64_t src = (int64_t)(g.u() * (double)(L - len));
    for (int c = 0; c < 4; ++c) {
      const int64_t dst = (int64_t)(g.u() * (double)(L - len));
      for (int k = 0; k < len; ++k) put2(pac, dst + k, g.u() < 0.01 ? (int)(g.next() & 3) : get2(pac, src + k));
    }
  }
  for (int t = 0; t < 10000; ++t) {  // tandem repeats
    const int per = 2 + g.i(49), len = 200 + g.i(800);
    const int64_t dst = (int64_t)(g.u() * (double)(L - len));
    for (int k = per; k < len; ++k) put2(pac, dst + k, g.u() < 0.005 ? (int)(g.next() & 3) : get2(pac, dst + k - per));
  }
  return 0;
}

// Upper bounds for synth_reads outputs.
void synth_bounds(int n_pairs, int len_mode, int64_t* max_seq, int32_t* max_chains, int32_t* max_seeds) {
  const int L = len_mode == 0 ? 250 : len_mode;
  *max_seq = (int64_t)2 * n_pairs * L;
  *max_chains = 2 * n_pairs * 3;
  *max_seeds = 2 * n_pairs * (L / 19 + 4) * 2;
}

}  // extern "C"

namespace {

// placement 0: a uniform contig, then a uniform fragment inside it (the
// synth workload); 1: genome-wide (contigs weighted by length, fragments may
// run off a contig) with one pair in ten straddling a contig junction (C3).
int reads_core(const uint8_t* pac, int64_t l_pac, const int64_t* ann_off, const int32_t* ann_len, int n_ctg,
               uint64_t seed, int n_pairs, int len_mode, int min_seed_len, int placement, int64_t* seq_off,
               uint8_t* seq, int32_t* read_chain_off, int32_t* chain_seed_off, int32_t* chain_rid,
               float* chain_frac_rep, bwagpu_seed_t* seeds, int32_t* n_reads_out, int32_t* n_chains_out,
               int32_t* n_seeds_out) {
  Rng g{seed ^ 0x5eedULL};
  int64_t so = 0;
  int32_t nr = 0, nc = 0, ns = 0;
  seq_off[0] = 0;
  read_chain_off[0] = 0;
  chain_seed_off[0] = 0;
  std::vector<uint8_t> frag, rd, fwdr;
  std::vector<int64_t> pos;  // per read base: 2-strand ref coordinate, or -1
  auto ctg_of = [&](int64_t f) {
    int lo = 0, hi = n_ctg - 1;
    while (lo < hi) {
      int m = (lo + hi + 1) >> 1;
      if (ann_off[m] <= f) lo = m;
      else hi = m - 1;
    }
    return lo;
  };
  for (int p = 0; p < n_pairs; ++p) {
    const int L = len_mode == 0 ? (p % 3 == 0 ? 100 : p % 3 == 1 ? 150 : 250) : len_mode;
    int fl = (int)(400 + 40 * g.n());
    fl = std::max(fl, L + 10);
    fl = std::min<int64_t>(fl, l_pac - 1);
    int64_t start;
    if (placement == 0) {
      const int ctg = g.i(n_ctg);
      if (ann_len[ctg] <= fl + 1) continue;
      start = ann_off[ctg] + (int64_t)(g.u() * (double)(ann_len[ctg] - fl));
    } else if (n_ctg > 1 && g.u() < 0.1) {  // the fragment straddles the start of contig k
      const int k = 1 + g.i(n_ctg - 1);
      start = std::max<int64_t>(0, ann_off[k] - 1 - g.i(fl - 1));
      if (start + fl > l_pac) continue;
    } else {
      start = (int64_t)(g.u() * (double)(l_pac - fl));
    }
    const int strand = (int)(g.next() & 1);
    for (int e = 0; e < 2; ++e) {
      const bool fwd = ((e == 0) ^ strand) != 0;
      // the read before errors, with the 2-strand coordinate of each base
      fwdr.assign(L, 0);
      std::vector<int64_t> p0(L);
      for (int i = 0; i < L; ++i) {
        if (fwd) {
          int64_t f = start + i;
          fwdr[i] = (uint8_t)get2(pac, f);
          p0[i] = f;
        } else {
          int64_t f = start + fl - 1 - i;
          fwdr[i] = (uint8_t)(3 - get2(pac, f));
          p0[i] = (l_pac << 1) - 1 - f;
        }
      }
      // errors
      rd.clear();
      pos.clear();
      for (int i = 0; i < L && (int)rd.size() < L; ++i) {
        double u = g.u();
        if (u < 0.0005) {
          rd.push_back(4);
          pos.push_back(-1);
        } else if (u < 0.0085) {
          rd.push_back((uint8_t)((fwdr[i] + 1 + g.i(3)) & 3));
          pos.push_back(-1);
        } else if (u < 0.009) {
          i += g.i(3);
        } else if (u < 0.0095) {
          int k = 1 + g.i(3);
          while (k-- && (int)rd.size() < L) {
            rd.push_back((uint8_t)(g.next() & 3));
            pos.push_back(-1);
          }
          if ((int)rd.size() < L) {
            rd.push_back(fwdr[i]);
            pos.push_back(p0[i]);
          }
        } else {
          rd.push_back(fwdr[i]);
          pos.push_back(p0[i]);
        }
      }
      const bool chimera = g.u() < 0.01;
      if (chimera) {  // second half from a random locus (forward)
        int64_t q = (int64_t)(g.u() * (double)(l_pac - L));
        for (int i = L / 2; i < (int)rd.size(); ++i) {
          rd[i] = (uint8_t)get2(pac, q + i);
          pos[i] = q + i;
        }
      }
      const int n = (int)rd.size();
      memcpy(seq + so, rd.data(), n);
      so += n;
      seq_off[nr + 1] = so;
      // maximal exact matches along the true alignment -> seeds
      auto emit_chain = [&](int a_begin, int a_end) {
        int32_t s0 = ns;
        int i = a_begin;
        int rid = -1;
        while (i < a_end) {
          if (pos[i] < 0) { ++i; continue; }
          int j = i + 1;
          while (j < a_end && pos[j] == pos[j - 1] + 1 &&
                 ((pos[j] < l_pac) == (pos[i] < l_pac)))
            ++j;
          const int len = j - i;
          if (len >= min_seed_len) {
            int64_t f = pos[i] < l_pac ? pos[i] : (l_pac << 1) - 1 - (pos[i] + len - 1);
            int64_t fe = f + len - 1;
            int c0 = ctg_of(f), c1 = ctg_of(fe);
            if (c0 == c1 && (rid < 0 || rid == c0)) {
              rid = c0;
              bwagpu_seed_t s;
              s.rbeg = pos[i];
              s.qbeg = i;
              s.len = len;
              s.score = len;
              s.pad_ = 0;
              seeds[ns++] = s;
            }
          }
          i = j;
        }
        if (ns > s0) {
          chain_rid[nc] = rid;
          chain_frac_rep[nc] = 0.f;
          chain_seed_off[++nc] = ns;
        }
      };
      if (chimera) {
        emit_chain(0, L / 2);
        emit_chain(L / 2, n);
      } else {
        emit_chain(0, n);
      }
      // a repeat copy of the longest seed elsewhere (secondary chain)
      if (nc > read_chain_off[nr] && g.u() < 0.1) {
        const int32_t c = nc - 1;
        int best = chain_seed_off[c];
        for (int k = chain_seed_off[c]; k < chain_seed_off[c + 1]; ++k)
          if (seeds[k].len > seeds[best].len) best = k;
        bwagpu_seed_t s = seeds[best];
        const int64_t f = (int64_t)(g.u() * (double)(l_pac - s.len - 1));
        const int cc = ctg_of(f);
        if (ctg_of(f + s.len - 1) == cc) {
          s.rbeg = f;
          s.score = s.len;
          seeds[ns++] = s;
          chain_rid[nc] = cc;
          chain_frac_rep[nc] = 0.25f;
          chain_seed_off[++nc] = ns;
        }
      }
      read_chain_off[++nr] = nc;
    }
  }
  *n_reads_out = nr;
  *n_chains_out = nc;
  *n_seeds_out = ns;
  return 0;
}

}  // namespace

extern "C" {

// Simulate n_pairs read pairs and their chains.  len_mode: 100/150/250, or 0
// for equal thirds of 100/150/250 (BASELINE config 5).  Outputs follow
// bwagpu_batch_t; sizes are returned through *n_*.  Returns 0 or -1.
int synth_reads(const uint8_t* pac, int64_t l_pac, const int64_t* ann_off, const int32_t* ann_len, int n_ctg,
                uint64_t seed, int n_pairs, int len_mode, int min_seed_len, int64_t* seq_off, uint8_t* seq,
                int32_t* read_chain_off, int32_t* chain_seed_off, int32_t* chain_rid, float* chain_frac_rep,
                bwagpu_seed_t* seeds, int32_t* n_reads_out, int32_t* n_chains_out, int32_t* n_seeds_out) {
  return reads_core(pac, l_pac, ann_off, ann_len, n_ctg, seed, n_pairs, len_mode, min_seed_len, 0, seq_off, seq,
                    read_chain_off, chain_seed_off, chain_rid, chain_frac_rep, seeds, n_reads_out, n_chains_out,
                    n_seeds_out);
}

// The same generator with C3's placement (reads_core placement 1).
int synth_reads_genome(const uint8_t* pac, int64_t l_pac, const int64_t* ann_off, const int32_t* ann_len, int n_ctg,
                       uint64_t seed, int n_pairs, int len_mode, int min_seed_len, int64_t* seq_off, uint8_t* seq,
                       int32_t* read_chain_off, int32_t* chain_seed_off, int32_t* chain_rid, float* chain_frac_rep,
                       bwagpu_seed_t* seeds, int32_t* n_reads_out, int32_t* n_chains_out, int32_t* n_seeds_out) {
  return reads_core(pac, l_pac, ann_off, ann_len, n_ctg, seed, n_pairs, len_mode, min_seed_len, 1, seq_off, seq,
                    read_chain_off, chain_seed_off, chain_rid, chain_frac_rep, seeds, n_reads_out, n_chains_out,
                    n_seeds_out);
}

}  // extern "C"
