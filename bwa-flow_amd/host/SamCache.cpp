// SamCache.cpp — the SAM-stage call cache of include/bwagpu_sam.h
// (lib/libgpusam.so): ksw_align2 calls of mate rescue (bwa/bwamem_pair.c:154)
// and mem_reg2aln CIGAR jobs (bwa/bwamem.c:1104-1174), keyed by content,
// queued on a miss and computed in one device batch per kind on flush
// (bwagpu_align2_batch / bwagpu_reg2aln_batch).
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <memory>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

#include "bwagpu.h"
#include "bwagpu_sam.h"

namespace {

// 64-bit content hash (multiply-xorshift over 8-byte words); collisions are
// resolved by comparing the stored bytes, so the hash only has to spread keys
inline uint64_t mix(uint64_t h, uint64_t v) {
  h ^= v + 0x9e3779b97f4a7c15ULL + (h << 6) + (h >> 2);
  h *= 0xbf58476d1ce4e5b9ULL;
  return h ^ (h >> 31);
}
uint64_t hash_bytes(uint64_t h, const uint8_t* p, int64_t n) {
  int64_t i = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t v;
    memcpy(&v, p + i, 8);
    h = mix(h, v);
  }
  uint64_t t = 0;
  for (int k = 0; i < n; ++i, ++k) t |= (uint64_t)p[i] << (8 * k);
  return mix(h, t ^ (uint64_t)n);
}

struct A2Entry {
  int64_t qoff, toff;
  int32_t qlen, tlen, xtra;
  bool ready;
  bwagpu_kswr_t r;
};

struct R2Entry {
  int64_t rb, re, qoff;
  int32_t l_seq, qb, qe, truesc, w;
  bool ready;
  bwagpu_aln_t a;
  int64_t cig_off, md_off;  // into the result pools once ready
};

// Calls are spread over kShards shards by hash, each with its own lock, so the
// stage's worker threads (16 on the reference's pipeline) rarely contend.
constexpr int kShards = 64;

struct Shard {
  std::mutex mu;
  std::vector<uint8_t> a2q, a2t, r2q;  // bases of the calls (nt4)
  std::vector<A2Entry> a2;
  std::vector<R2Entry> r2;
  std::unordered_multimap<uint64_t, int32_t> a2map, r2map;
  std::vector<int32_t> a2pend, r2pend;
  std::vector<uint32_t> cig;  // CIGAR ops of the ready reg2aln jobs
  std::vector<char> md;       // their MD strings, NUL-terminated
  int64_t st[4] = {};         // align2 hits / misses, reg2aln hits / misses
  void clear() {
    a2q.clear(); a2t.clear(); r2q.clear(); a2.clear(); r2.clear(); a2map.clear(); r2map.clear();
    a2pend.clear(); r2pend.clear(); cig.clear(); md.clear();
  }
};

}  // namespace

struct bwagpu_samcache {
  bwagpu_ctx_t* ctx;
  int32_t max_ops, max_md;
  Shard sh[kShards];
  int64_t st[4] = {};  // align2 computed, reg2aln computed, flushes, flush microseconds
};

namespace {

inline Shard& shard_of(bwagpu_samcache_t* c, uint64_t h) { return c->sh[h >> 58]; }

// f(t, nt) on nt threads (the flush runs with the stage's workers joined, so
// their cores are free)
template <typename F>
void on_threads(F f) {
  const int nt = (int)std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (int t = 1; t < nt; ++t) th.emplace_back(f, t, nt);
  f(0, nt);
  for (auto& x : th) x.join();
}

uint32_t* empty_block() { return (uint32_t*)calloc(1, sizeof(uint32_t)); }

// every shard's queued ksw_align2 calls in one bwagpu_align2_batch (their
// bases gathered into one query / target pool)
int flush_align2(bwagpu_samcache_t* c) {
  std::vector<bwagpu_align2_task_t> tasks;
  std::vector<std::pair<int, int32_t>> who;  // (shard, entry)
  std::vector<uint8_t> qp, tp;
  for (int s = 0; s < kShards; ++s)
    for (int32_t id : c->sh[s].a2pend) {
      const A2Entry& e = c->sh[s].a2[(size_t)id];
      tasks.push_back(bwagpu_align2_task_t{(int64_t)qp.size(), (int64_t)tp.size(), e.qlen, e.tlen, e.xtra, 0});
      qp.insert(qp.end(), c->sh[s].a2q.begin() + e.qoff, c->sh[s].a2q.begin() + e.qoff + e.qlen);
      tp.insert(tp.end(), c->sh[s].a2t.begin() + e.toff, c->sh[s].a2t.begin() + e.toff + e.tlen);
      who.emplace_back(s, id);
    }
  const int32_t n = (int32_t)tasks.size();
  if (n == 0) return 0;
  std::vector<bwagpu_kswr_t> res((size_t)n);
  const int rc = bwagpu_align2_batch(c->ctx, n, tasks.data(), qp.data(), (int64_t)qp.size(), tp.data(),
                                     (int64_t)tp.size(), res.data());
  if (rc) return rc;
  for (int32_t k = 0; k < n; ++k) {
    A2Entry& e = c->sh[who[(size_t)k].first].a2[(size_t)who[(size_t)k].second];
    e.r = res[(size_t)k];
    e.ready = true;
  }
  for (auto& sh : c->sh) sh.a2pend.clear();
  c->st[0] += n;
  return 0;
}

// one bwagpu_reg2aln_batch over `ids` (shard, entry; in shard order); jobs
// whose CIGAR or MD overflowed the launch's capacity are returned in `over`.
// Packing and the result copy-back run on several threads (the result copy
// split at shard boundaries, so each shard's pools have one writer).
int run_reg2aln(bwagpu_samcache_t* c, const std::vector<std::pair<int, int32_t>>& ids, int32_t max_ops,
                int32_t max_md, std::vector<std::pair<int, int32_t>>& over) {
  const int32_t n = (int32_t)ids.size();
  if (n == 0) return 0;
  std::vector<bwagpu_reg2aln_task_t> tasks((size_t)n);
  std::vector<int64_t> qoff((size_t)n + 1, 0);
  for (int32_t k = 0; k < n; ++k)
    qoff[(size_t)k + 1] = qoff[(size_t)k] + c->sh[ids[(size_t)k].first].r2[(size_t)ids[(size_t)k].second].l_seq;
  std::unique_ptr<uint8_t[]> qpp(new uint8_t[(size_t)qoff[(size_t)n] + 1]);
  uint8_t* const qp = qpp.get();
  on_threads([&](int t, int nt) {
    for (int32_t k = (int32_t)((int64_t)n * t / nt); k < (int32_t)((int64_t)n * (t + 1) / nt); ++k) {
      const Shard& sh = c->sh[ids[(size_t)k].first];
      const R2Entry& e = sh.r2[(size_t)ids[(size_t)k].second];
      tasks[(size_t)k] = bwagpu_reg2aln_task_t{e.rb, e.re, qoff[(size_t)k], e.l_seq, e.qb, e.qe, e.truesc, e.w, 0};
      memcpy(qp + qoff[(size_t)k], sh.r2q.data() + e.qoff, (size_t)e.l_seq);
    }
  });
  std::vector<bwagpu_aln_t> out((size_t)n);
  // the device fills every slot it reports; no zero fill of the n x (max_ops,
  // max_md) blocks (tens of MB per flush at C2 batch size)
  std::unique_ptr<uint32_t[]> cgp(new uint32_t[(size_t)n * (size_t)max_ops]);
  std::unique_ptr<char[]> mdp(new char[(size_t)n * (size_t)max_md]);
  uint32_t* const cg = cgp.get();
  char* const mdb = mdp.get();
  const int rc = bwagpu_reg2aln_batch(c->ctx, n, tasks.data(), qp, qoff[(size_t)n], max_ops, max_md, out.data(), cg,
                                      mdb);
  if (rc) return rc;
  // shard boundaries in ids
  std::vector<int32_t> sb(kShards + 1, n);
  for (int32_t k = n - 1; k >= 0; --k) sb[(size_t)ids[(size_t)k].first] = k;
  for (int s = kShards - 1; s >= 0; --s) sb[(size_t)s] = std::min(sb[(size_t)s], sb[(size_t)s + 1]);
  std::vector<std::vector<std::pair<int, int32_t>>> over_t(16);
  std::vector<int64_t> done_t(16, 0);
  on_threads([&](int t, int nt) {
    for (int s = t; s < kShards; s += nt) {
      Shard& sh = c->sh[s];
      for (int32_t k = sb[(size_t)s]; k < sb[(size_t)s + 1]; ++k) {
        R2Entry& e = sh.r2[(size_t)ids[(size_t)k].second];
        const bwagpu_aln_t& a = out[(size_t)k];
        if (a.status == BWAGPU_ALN_OVERFLOW) {
          over_t[(size_t)t].push_back(ids[(size_t)k]);
          continue;
        }
        e.a = a;
        e.cig_off = (int64_t)sh.cig.size();
        e.md_off = (int64_t)sh.md.size();
        if (a.status == BWAGPU_ALN_OK) {
          const uint32_t* src = cg + (size_t)k * max_ops;
          sh.cig.insert(sh.cig.end(), src, src + a.n_cigar);
          const char* m = mdb + (size_t)k * max_md;
          sh.md.insert(sh.md.end(), m, m + a.md_len);
        }
        sh.md.push_back(0);
        e.ready = true;
        ++done_t[(size_t)t];
      }
    }
  });
  for (int t = 0; t < 16; ++t) {
    over.insert(over.end(), over_t[(size_t)t].begin(), over_t[(size_t)t].end());
    c->st[1] += done_t[(size_t)t];
  }
  return 0;
}

int flush_reg2aln(bwagpu_samcache_t* c) {
  std::vector<std::pair<int, int32_t>> ids, over, over2;
  for (int s = 0; s < kShards; ++s)
    for (int32_t id : c->sh[s].r2pend) ids.emplace_back(s, id);
  if (ids.empty()) return 0;
  int rc = run_reg2aln(c, ids, c->max_ops, c->max_md, over);
  if (rc) return rc;
  if (!over.empty()) {
    // room for any alignment of the longest read among them: one op per base
    // and indel run, MD at most a few bytes per base
    std::sort(over.begin(), over.end());  // run_reg2aln wants shard order
    int32_t lmax = 0;
    for (auto& w : over) lmax = std::max(lmax, c->sh[w.first].r2[(size_t)w.second].l_seq);
    rc = run_reg2aln(c, over, 2 * lmax + 8, 8 * lmax + 64, over2);
    if (rc) return rc;
    if (!over2.empty()) return BWAGPU_E_RESULTS;
  }
  for (auto& sh : c->sh) sh.r2pend.clear();
  return 0;
}

}  // namespace

extern "C" {

int bwagpu_samcache_create(bwagpu_ctx_t* ctx, int32_t max_ops, int32_t max_md, bwagpu_samcache_t** out) {
  if (!ctx || !out || max_ops < 1 || max_md < 1) return BWAGPU_E_INVAL;
  auto* c = new bwagpu_samcache;
  c->ctx = ctx;
  c->max_ops = max_ops;
  c->max_md = max_md;
  *out = c;
  return BWAGPU_OK;
}

int bwagpu_samcache_destroy(bwagpu_samcache_t* c) {
  delete c;
  return BWAGPU_OK;
}

int bwagpu_samcache_clear(bwagpu_samcache_t* c) {
  if (!c) return BWAGPU_E_INVAL;
  on_threads([&](int t, int nt) {
    for (int s = t; s < kShards; s += nt) {
      std::lock_guard<std::mutex> g(c->sh[s].mu);
      c->sh[s].clear();
    }
  });
  return BWAGPU_OK;
}

int bwagpu_samcache_align2(bwagpu_samcache_t* c, int32_t qlen, const uint8_t* query, int32_t tlen,
                           const uint8_t* target, int32_t xtra, bwagpu_kswr_t* out) {
  if (!c || !out || qlen < 0 || tlen < 0 || (qlen && !query) || (tlen && !target)) return -BWAGPU_E_INVAL;
  uint64_t h = mix(mix(0x243f6a8885a308d3ULL, (uint64_t)(uint32_t)qlen << 32 | (uint32_t)tlen), (uint64_t)(uint32_t)xtra);
  h = hash_bytes(hash_bytes(h, query, qlen), target, tlen);
  Shard& sh = shard_of(c, h);
  std::lock_guard<std::mutex> g(sh.mu);
  auto range = sh.a2map.equal_range(h);
  for (auto it = range.first; it != range.second; ++it) {
    const A2Entry& e = sh.a2[(size_t)it->second];
    if (e.qlen != qlen || e.tlen != tlen || e.xtra != xtra || memcmp(sh.a2q.data() + e.qoff, query, (size_t)qlen) ||
        memcmp(sh.a2t.data() + e.toff, target, (size_t)tlen))
      continue;
    if (e.ready) {
      *out = e.r;
      ++sh.st[0];
      return 0;
    }
    *out = bwagpu_kswr_t{0, -1, -1, -1, -1, -1, -1};
    ++sh.st[1];
    return 1;  // queued by an earlier miss of this pass
  }
  A2Entry e{(int64_t)sh.a2q.size(), (int64_t)sh.a2t.size(), qlen, tlen, xtra, false, {}};
  sh.a2q.insert(sh.a2q.end(), query, query + qlen);
  sh.a2t.insert(sh.a2t.end(), target, target + tlen);
  sh.a2map.emplace(h, (int32_t)sh.a2.size());
  sh.a2pend.push_back((int32_t)sh.a2.size());
  sh.a2.push_back(e);
  *out = bwagpu_kswr_t{0, -1, -1, -1, -1, -1, -1};
  ++sh.st[1];
  return 1;
}

int bwagpu_samcache_reg2aln(bwagpu_samcache_t* c, int32_t l_seq, const uint8_t* read, int64_t rb, int64_t re,
                            int32_t qb, int32_t qe, int32_t truesc, int32_t w, bwagpu_aln_t* out, uint32_t** cigar) {
  if (!c || !out || !cigar || l_seq < 0 || (l_seq && !read) || rb < 0 || re < 0) return -BWAGPU_E_INVAL;
  uint64_t h = mix(mix(mix(0x13198a2e03707344ULL, (uint64_t)rb), (uint64_t)re),
                   (uint64_t)(uint32_t)qb << 32 | (uint32_t)qe);
  h = mix(mix(h, (uint64_t)(uint32_t)truesc << 32 | (uint32_t)w), (uint64_t)(uint32_t)l_seq);
  h = hash_bytes(h, read, l_seq);
  Shard& sh = shard_of(c, h);
  std::lock_guard<std::mutex> g(sh.mu);
  auto range = sh.r2map.equal_range(h);
  bool queued = false;
  for (auto it = range.first; it != range.second; ++it) {
    const R2Entry& e = sh.r2[(size_t)it->second];
    if (e.rb != rb || e.re != re || e.qb != qb || e.qe != qe || e.truesc != truesc || e.w != w || e.l_seq != l_seq ||
        memcmp(sh.r2q.data() + e.qoff, read, (size_t)l_seq))
      continue;
    if (!e.ready) {
      queued = true;
      break;
    }
    *out = e.a;
    const int32_t nc = e.a.status == BWAGPU_ALN_OK ? e.a.n_cigar : 0;
    const int32_t ml = e.a.status == BWAGPU_ALN_OK ? e.a.md_len : 0;
    uint32_t* blk = (uint32_t*)malloc(sizeof(uint32_t) * (size_t)nc + (size_t)ml + 1);
    if (!blk) return -BWAGPU_E_NOMEM;
    memcpy(blk, sh.cig.data() + e.cig_off, sizeof(uint32_t) * (size_t)nc);
    memcpy((char*)(blk + nc), sh.md.data() + e.md_off, (size_t)ml + 1);
    *cigar = blk;
    ++sh.st[2];
    return 0;
  }
  if (!queued) {
    R2Entry e{rb, re, (int64_t)sh.r2q.size(), l_seq, qb, qe, truesc, w, false, {}, 0, 0};
    sh.r2q.insert(sh.r2q.end(), read, read + l_seq);
    sh.r2map.emplace(h, (int32_t)sh.r2.size());
    sh.r2pend.push_back((int32_t)sh.r2.size());
    sh.r2.push_back(e);
  }
  memset(out, 0, sizeof *out);
  out->status = -1;
  *cigar = empty_block();
  ++sh.st[3];
  return *cigar ? 1 : -BWAGPU_E_NOMEM;
}

int64_t bwagpu_samcache_flush(bwagpu_samcache_t* c) {
  if (!c) return -BWAGPU_E_INVAL;
  const auto t0 = std::chrono::steady_clock::now();
  int64_t n = 0;
  for (auto& sh : c->sh) n += (int64_t)sh.a2pend.size() + (int64_t)sh.r2pend.size();
  if (n == 0) return 0;
  int rc = flush_align2(c);
  if (!rc) rc = flush_reg2aln(c);
  ++c->st[2];
  c->st[3] += (int64_t)std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  return rc ? -(int64_t)rc : n;
}

int bwagpu_samcache_stats(const bwagpu_samcache_t* c, int64_t out[8]) {
  if (!c || !out) return BWAGPU_E_INVAL;
  for (int i = 0; i < 4; ++i) out[i] = 0;
  for (const auto& sh : c->sh)
    for (int i = 0; i < 4; ++i) out[i] += sh.st[i];
  for (int i = 0; i < 4; ++i) out[4 + i] = c->st[i];
  return BWAGPU_OK;
}

}  // extern "C"
