// GPUPipeline.cpp — see GPUPipeline.h.
#include "GPUPipeline.h"

#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <functional>
#include <memory>
#include <stdexcept>
#include <thread>

#ifdef BWAFLOW_NATIVE_HEADERS
#include "Pipeline.h"
#else
#include "cpu_stage.h"
#endif

// ------------------------------------------------------------------ GPUEnv
namespace {

// the few RCCL entry points GPUEnv needs, resolved at run time
struct Rccl {
  void* h = nullptr;
  ncclResult_t (*init_all)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*bcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  bool load() {
    const char* names[] = {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"};
    for (const char* n : names)
      if ((h = dlopen(n, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
    if (!h) return false;
    init_all = (decltype(init_all))dlsym(h, "ncclCommInitAll");
    bcast = (decltype(bcast))dlsym(h, "ncclBroadcast");
    group_start = (decltype(group_start))dlsym(h, "ncclGroupStart");
    group_end = (decltype(group_end))dlsym(h, "ncclGroupEnd");
    destroy = (decltype(destroy))dlsym(h, "ncclCommDestroy");
    return init_all && bcast && group_start && group_end && destroy;
  }
};

}  // namespace

static bool force_rccl_env() {
  const char* e = getenv("BWAGPU_FORCE_RCCL");
  return e && e[0] == '1';
}

GPUEnv::GPUEnv(const bwagpu_opt_t& opt, const bwagpu_bns_t& bns, const uint8_t* pac, int max_devices,
               int watchdog_ms, int per_device, int force_rccl) {
  int n = 0;
  const int rc = bwagpu_device_count(&n);
  if (rc != BWAGPU_OK) {
    status_ = "no GPU device (bwagpu_device_count rc=" + std::to_string(rc) + ")";
    return;
  }
  n = std::min(n, max_devices);
  const size_t pac_bytes = (size_t)(bns.l_pac / 4 + 1);
  // the reference on every device: H2D to the first, RCCL broadcast to the rest
  for (int d = 0; d < n; ++d) {
    void* p = nullptr;
    if (hipSetDevice(d) != hipSuccess || hipMalloc(&p, pac_bytes) != hipSuccess) {
      status_ += "device " + std::to_string(d) + ": no memory for the reference; ";
      continue;
    }
    pac_dev_.push_back(p);
    pac_devid_.push_back(d);
  }
  if (pac_dev_.empty()) return;
  auto drop = [&](size_t i) {  // device i keeps no reference and gets no context
    (void)hipSetDevice(pac_devid_[i]);
    (void)hipFree(pac_dev_[i]);
    pac_dev_.erase(pac_dev_.begin() + (long)i);
    pac_devid_.erase(pac_devid_.begin() + (long)i);
  };
  // With one device the broadcast is normally skipped.  force_rccl (or
  // BWAGPU_FORCE_RCCL=1) runs it anyway on a one-rank communicator: the host
  // copy goes to a staging buffer and ncclBroadcast fills the context's
  // reference from it, so the path the 8-GPU node takes is exercised (and its
  // result checked by every alignment) on a one-GPU box.
  const bool force = (force_rccl < 0 ? force_rccl_env() : force_rccl > 0) && pac_dev_.size() == 1;
  void* root = pac_dev_[0];
  (void)hipSetDevice(pac_devid_[0]);
  if (force && hipMalloc(&root, pac_bytes) != hipSuccess) {
    status_ += "no memory for the broadcast staging buffer; ";
    root = pac_dev_[0];
  }
  const bool staged = root != pac_dev_[0];
  if (hipMemcpy(root, pac, pac_bytes, hipMemcpyHostToDevice) != hipSuccess) {
    status_ += "H2D of the reference failed; ";
    if (staged) (void)hipFree(root);
    while (!pac_dev_.empty()) drop(pac_dev_.size() - 1);
    return;
  }
  if (pac_dev_.size() > 1 || staged) {
    Rccl r;
    bool ok = r.load();
    const int nd = (int)pac_dev_.size();
    std::vector<ncclComm_t> comms((size_t)nd, nullptr);
    std::vector<hipStream_t> st((size_t)nd, nullptr);
    if (ok) ok = r.init_all(comms.data(), nd, pac_devid_.data()) == ncclSuccess;
    if (ok) {
      for (int i = 0; i < nd; ++i) {
        (void)hipSetDevice(pac_devid_[i]);
        (void)hipStreamCreate(&st[i]);
      }
      ok = r.group_start() == ncclSuccess;
      for (int i = 0; ok && i < nd; ++i)
        ok = r.bcast(root, pac_dev_[i], pac_bytes, ncclUint8, 0, comms[i], st[i]) == ncclSuccess;
      ok = (r.group_end() == ncclSuccess) && ok;
      for (int i = 0; i < nd; ++i) {
        (void)hipSetDevice(pac_devid_[i]);
        ok = (hipStreamSynchronize(st[i]) == hipSuccess) && ok;
        (void)hipStreamDestroy(st[i]);
      }
    }
    for (auto c : comms)
      if (c) r.destroy(c);
    rccl_ = ok;
    if (!ok) {  // per-device host copies instead; a device whose copy fails is dropped
      for (size_t i = staged ? 0 : 1; i < pac_dev_.size();) {
        (void)hipSetDevice(pac_devid_[i]);
        if (hipMemcpy(pac_dev_[i], pac, pac_bytes, hipMemcpyHostToDevice) != hipSuccess) {
          status_ += "device " + std::to_string(pac_devid_[i]) + ": H2D of the reference failed; ";
          drop(i);
          continue;
        }
        ++i;
      }
      status_ += "RCCL unavailable: host copies; ";
    }
  }
  if (staged) {
    (void)hipSetDevice(pac_devid_.empty() ? 0 : pac_devid_[0]);
    (void)hipFree(root);
  }
  for (size_t i = 0; i < pac_dev_.size(); ++i) {
    for (int k = 0; k < per_device; ++k) {
      bwagpu_ctx_t* c = nullptr;
      const int r = bwagpu_create_resident(pac_devid_[i], &opt, &bns, pac_dev_[i], &c);
      if (r != BWAGPU_OK) {
        status_ += "device " + std::to_string(pac_devid_[i]) + ": " + (c ? bwagpu_last_error(c) : "create failed") + "; ";
        if (c) bwagpu_destroy(c);
        continue;
      }
      bwagpu_set_watchdog_ms(c, watchdog_ms);  // fpgaHangError's 10 s watchdog (SWTask.cpp:116-122)
      ctx_.push_back(c);
    }
  }
  status_ += std::to_string(ctx_.size()) + " context(s) on " + std::to_string(pac_dev_.size()) + " device(s)" +
             (rccl_ ? ", reference broadcast over RCCL" : "");
}

GPUEnv::~GPUEnv() {
  for (auto* c : ctx_) bwagpu_destroy(c);  // synchronizes each context's streams
  for (size_t i = 0; i < pac_dev_.size(); ++i) {
    (void)hipSetDevice(pac_devid_[i]);
    (void)hipFree(pac_dev_[i]);
  }
}

// --------------------------------------------------------------- FlatBatch
// Host-side packing and unpacking run over read ranges on a few threads: at
// C2 batch size (66.7k reads, 300k seeds) one thread needs ~10 ms for each
// direction, twice the batch's GPU time (bench.py end_to_end phases).
int host_threads() {
  static const int n = [] {
    const char* e = getenv("BWAGPU_HOST_THREADS");
    int v = e ? atoi(e) : (int)std::thread::hardware_concurrency();
    return std::max(1, std::min(v, 8));
  }();
  return n;
}

// One persistent pool for every stage worker's pack/unpack ranges (threads are
// not created per record; with several workers per device their pieces queue
// on the same host_threads() - 1 threads).
namespace {
class HostPool {
 public:
  static HostPool& get() {
    static HostPool p(host_threads() - 1);
    return p;
  }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  explicit HostPool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  void loop() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  std::vector<std::thread> th_;
  bool stop_ = false;
};
}  // namespace

// threads that malloc the records' mem_alnreg_v (unpack_dense):
// BWAGPU_UNPACK_THREADS, default host_threads().  Every region array is freed
// later by another stage's threads (RegionsToSam), so each malloc takes a chunk
// a remote free put back into its arena; more threads are not always faster
int unpack_threads() {
  static const int n = [] {
    const char* e = getenv("BWAGPU_UNPACK_THREADS");
    return std::max(1, std::min(e ? atoi(e) : host_threads(), host_threads()));
  }();
  return n;
}

template <typename F>
static void parallel_ranges(int n, F f, int max_t = 0) {  // f(begin, end) over [0, n) in <= max_t pieces
  const int t = std::min(max_t > 0 ? max_t : host_threads(), std::max(1, n / 2048));
  if (t <= 1) {
    f(0, n);
    return;
  }
  // the count is decremented under the lock: a task touches m / done only while
  // holding m, and the caller cannot see left == 0 (and unwind this frame)
  // before the last task has released it
  int left = t - 1;
  std::mutex m;
  std::condition_variable done;
  for (int k = 1; k < t; ++k)
    HostPool::get().post([&, k] {
      f((int)((int64_t)n * k / t), (int)((int64_t)n * (k + 1) / t));
      std::lock_guard<std::mutex> g(m);
      if (--left == 0) done.notify_all();
    });
  f(0, (int)((int64_t)n / t));
  std::unique_lock<std::mutex> g(m);
  done.wait(g, [&] { return left == 0; });
}

void FlatBatch::pack(const ChainsRecord& rec) {
  const int nr = rec.batch_num;
  // pass 1: per-read counts -> offsets
  seq_off.assign((size_t)nr + 1, 0);
  read_chain_off.assign((size_t)nr + 1, 0);
  std::vector<int64_t> seed_base((size_t)nr + 1, 0);
  for (int i = 0; i < nr; ++i) {
    const mem_chain_v& cv = rec.chains[i];
    int64_t ns = 0;
    for (size_t j = 0; j < cv.n; ++j) ns += cv.a[j].n;
    seq_off[i + 1] = seq_off[i] + rec.seqs[i].l_seq;
    read_chain_off[i + 1] = read_chain_off[i] + (int32_t)cv.n;
    seed_base[i + 1] = seed_base[i] + ns;
  }
  const size_t nc = (size_t)read_chain_off[nr], ns = (size_t)seed_base[nr];
  seq.resize((size_t)seq_off[nr]);
  chain_rid.resize(nc);
  chain_frac_rep.resize(nc);
  chain_seed_off.resize(nc + 1);
  seeds.resize(ns);
  chain_seed_off[0] = 0;
  // pass 2: every read's bases, chains and seeds in place
  parallel_ranges(nr, [&](int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
      const bseq1_t& s = rec.seqs[i];
      memcpy(seq.data() + seq_off[i], s.seq, (size_t)s.l_seq);
      const mem_chain_v& cv = rec.chains[i];
      int64_t so = seed_base[i];
      for (size_t j = 0; j < cv.n; ++j) {
        const mem_chain_t& c = cv.a[j];
        const size_t ci = (size_t)read_chain_off[i] + j;
        chain_rid[ci] = c.rid;
        chain_frac_rep[ci] = c.frac_rep;
        for (int k = 0; k < c.n; ++k) {
          bwagpu_seed_t& t = seeds[(size_t)so + k];
          t.rbeg = c.seeds[k].rbeg;
          t.qbeg = c.seeds[k].qbeg;
          t.len = c.seeds[k].len;
          t.score = c.seeds[k].score;
          t.pad_ = 0;
        }
        so += c.n;
        chain_seed_off[ci + 1] = (int32_t)so;
      }
    }
  });
  regs.resize(ns ? ns : 1);
  n.assign(nr ? nr : 1, 0);
  c = bwagpu_batch_t{};
  c.n_reads = nr;
  c.n_chains = (int32_t)nc;
  c.n_seeds = (int32_t)ns;
  c.seq_bytes = seq_off.back();
  c.seq_off = seq_off.data();
  c.seq = seq.data();
  c.read_chain_off = read_chain_off.data();
  c.chain_seed_off = chain_seed_off.data();
  c.chain_rid = chain_rid.data();
  c.chain_frac_rep = chain_frac_rep.data();
  c.seeds = seeds.data();
}

int FlatBatch::pack_staged(bwagpu_ctx_t* ctx, int slot, const ChainsRecord& rec) {
  const int nr = rec.batch_num;
  // pass 1, on the pool: per-read counts (bases, chains, seeds) in place, then
  // their prefix sums -> offsets (kept here: unpack needs them).  Reading every
  // chain's seed count is a pointer chase per read; serial it cost ~1 ms a record
  seq_off.assign((size_t)nr + 1, 0);
  read_chain_off.assign((size_t)nr + 1, 0);
  seed_base.assign((size_t)nr + 1, 0);
  parallel_ranges(nr, [&](int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
      const mem_chain_v& cv = rec.chains[i];
      int64_t ns = 0;
      for (size_t j = 0; j < cv.n; ++j) ns += cv.a[j].n;
      seq_off[i + 1] = rec.seqs[i].l_seq;
      read_chain_off[i + 1] = (int32_t)cv.n;
      seed_base[i + 1] = ns;
    }
  });
  for (int i = 0; i < nr; ++i) {
    seq_off[i + 1] += seq_off[i];
    read_chain_off[i + 1] += read_chain_off[i];
    seed_base[i + 1] += seed_base[i];
  }
  const int32_t nc = read_chain_off[nr];
  const int64_t ns = seed_base[nr];
  if (ns > INT32_MAX) return BWAGPU_E_UNSUPPORTED;
  const int rc = bwagpu_chain2aln_stage(ctx, slot, nr, nc, (int32_t)ns, seq_off[nr], &c);
  if (rc != BWAGPU_OK) return rc;
  int64_t* v_so = const_cast<int64_t*>(c.seq_off);
  uint8_t* v_seq = const_cast<uint8_t*>(c.seq);
  int32_t* v_rco = const_cast<int32_t*>(c.read_chain_off);
  int32_t* v_cso = const_cast<int32_t*>(c.chain_seed_off);
  int32_t* v_rid = const_cast<int32_t*>(c.chain_rid);
  float* v_fr = const_cast<float*>(c.chain_frac_rep);
  bwagpu_seed_t* v_sd = const_cast<bwagpu_seed_t*>(c.seeds);
  memcpy(v_so, seq_off.data(), sizeof(int64_t) * ((size_t)nr + 1));
  memcpy(v_rco, read_chain_off.data(), sizeof(int32_t) * ((size_t)nr + 1));
  v_cso[0] = 0;
  // pass 2: every read's bases, chains and seeds, in place in pinned memory;
  // mem_seed_t and bwagpu_seed_t are the same 24 bytes (records.h), so a
  // chain's seeds go in one copy
  parallel_ranges(nr, [&](int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
      const bseq1_t& s = rec.seqs[i];
      memcpy(v_seq + seq_off[i], s.seq, (size_t)s.l_seq);
      const mem_chain_v& cv = rec.chains[i];
      int64_t so = seed_base[i];
      for (size_t j = 0; j < cv.n; ++j) {
        const mem_chain_t& ch = cv.a[j];
        const size_t ci = (size_t)read_chain_off[i] + j;
        v_rid[ci] = ch.rid;
        v_fr[ci] = ch.frac_rep;
        if (ch.n > 0) memcpy(v_sd + so, ch.seeds, sizeof(bwagpu_seed_t) * (size_t)ch.n);
        so += ch.n;
        v_cso[ci + 1] = (int32_t)so;
      }
    }
  });
  return BWAGPU_OK;
}

mem_alnreg_v* FlatBatch::unpack_dense(const bwagpu_alnreg_t* rg, const int32_t* nn, const int32_t* off,
                                      int batch_num) {
  mem_alnreg_v* av = (mem_alnreg_v*)malloc(sizeof(mem_alnreg_v) * (size_t)(batch_num > 0 ? batch_num : 1));
  if (!av) throw std::runtime_error("Memory allocation failed");
  std::atomic<bool> oom{false};
  parallel_ranges(batch_num, [&](int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
      const size_t k = (size_t)nn[i];
      av[i].n = av[i].m = k;
      av[i].a = nullptr;
      if (k) {
        av[i].a = (mem_alnreg_t*)malloc(sizeof(mem_alnreg_t) * k);
        if (!av[i].a) {
          oom = true;
          continue;
        }
        memcpy(av[i].a, &rg[off[i]], sizeof(mem_alnreg_t) * k);
      }
    }
  }, unpack_threads());
  if (oom) throw std::runtime_error("Memory allocation failed");
  return av;
}

mem_alnreg_v* FlatBatch::unpack(int batch_num) const {
  mem_alnreg_v* av = (mem_alnreg_v*)malloc(sizeof(mem_alnreg_v) * (size_t)(batch_num > 0 ? batch_num : 1));
  if (!av) throw std::runtime_error("Memory allocation failed");
  std::atomic<bool> oom{false};
  parallel_ranges(batch_num, [&](int r0, int r1) {
    for (int i = r0; i < r1; ++i) {
      const size_t k = (size_t)n[i];
      av[i].n = av[i].m = k;
      av[i].a = nullptr;
      if (k) {
        av[i].a = (mem_alnreg_t*)malloc(sizeof(mem_alnreg_t) * k);
        if (!av[i].a) {
          oom = true;
          continue;
        }
        memcpy(av[i].a, &regs[chain_seed_off[read_chain_off[i]]], sizeof(mem_alnreg_t) * k);
      }
    }
  });
  if (oom) throw std::runtime_error("Memory allocation failed");
  return av;
}

// serial: the chains were malloc'd by the upstream stage's threads, and frees
// from several threads into one glibc arena contend for its lock (measured:
// 2x slower on 8 threads than on one)
void freeChainsRecordChains(mem_chain_v* chains, int batch_num) {
  if (!chains) return;
  for (int i = 0; i < batch_num; ++i) {
    for (size_t j = 0; j < chains[i].n; ++j) free(chains[i].a[j].seeds);
    free(chains[i].a);
  }
  free(chains);
}

// ------------------------------------------------------------ ChainReaper
static bool reaper_enabled() {
  static const bool on = [] {
    const char* e = getenv("BWAGPU_CHAIN_REAPER");
    return !(e && e[0] == '0');
  }();
  return on;
}

int ChainReaper::threads() {
  static const int n = [] {
    const char* e = getenv("BWAGPU_REAPER_THREADS");
    // 4: a record's ~170 k chain frees cost ~8-14 ms of CPU (remote frees into
    // the producers' arenas); with 2 threads they capped the stage
    return std::max(1, std::min(e ? atoi(e) : 4, 16));
  }();
  return n;
}

ChainReaper::~ChainReaper() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_)
    if (t.joinable()) t.join();  // run() frees what is left before it returns
}

void ChainReaper::release(mem_chain_v* chains, int batch_num) {
  if (!chains) return;
  if (!reaper_enabled()) {
    freeChainsRecordChains(chains, batch_num);
    return;
  }
  bool queued = false;
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!started_) {
      started_ = true;
      for (int k = 0; k < threads(); ++k) th_.emplace_back([this] { run(); });
    }
    // bounded: when the reaper falls behind, the releasing worker frees this
    // record itself (chain memory cannot grow without limit)
    if (q_.size() < kMaxQueued) {
      q_.emplace_back(chains, batch_num);
      queued = true;
    }
  }
  if (!queued) {
    n_inline_.fetch_add(1);
    freeChainsRecordChains(chains, batch_num);
    return;
  }
  cv_.notify_one();
}

void ChainReaper::hold(bool on) {
  {
    std::lock_guard<std::mutex> g(mu_);
    held_ = on;
  }
  cv_.notify_all();
}

void ChainReaper::drain() {
  std::unique_lock<std::mutex> g(mu_);
  idle_.wait(g, [this] { return q_.empty() && busy_ == 0; });
}

void ChainReaper::run() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    cv_.wait(g, [this] { return stop_ || (!q_.empty() && !held_); });
    if (q_.empty()) return;  // stop_ and nothing left
    auto job = q_.front();
    q_.pop_front();
    ++busy_;
    g.unlock();
    freeChainsRecordChains(job.first, job.second);
    g.lock();
    --busy_;
    if (q_.empty() && busy_ == 0) idle_.notify_all();
  }
}

// ----------------------------------------------------------------- PostPool
int PostPool::threads() {
  static const int n = [] {
    const char* e = getenv("BWAGPU_POST_THREADS");
    // default 0: on the box's 16 cores the measured gain was within the
    // host's run-to-run noise (tools_dev/e2e_sweep.py, gpurun_out/r06c)
    return std::max(0, std::min(e ? atoi(e) : 0, 16));
  }();
  return n;
}

PostPool::~PostPool() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : th_)
    if (t.joinable()) t.join();  // run() finishes what is queued before it returns
}

void PostPool::post(std::function<void()> f) {
  {
    std::lock_guard<std::mutex> g(mu_);
    if (!started_) {
      started_ = true;
      for (int k = 0; k < threads(); ++k) th_.emplace_back([this] { run(); });
    }
    q_.push_back(std::move(f));
  }
  cv_.notify_one();
}

void PostPool::run() {
  std::unique_lock<std::mutex> g(mu_);
  for (;;) {
    cv_.wait(g, [this] { return stop_ || !q_.empty(); });
    if (q_.empty()) return;
    auto f = std::move(q_.front());
    q_.pop_front();
    g.unlock();
    f();
    g.lock();
  }
}

// ------------------------------------------------------- ChainsToRegionsGPU
// records a worker keeps in flight (its context's slots in use): every slot
// is a stream of its own, and with its selection side stream each takes a
// hardware queue (GPU_MAX_HW_QUEUES = 4 by default); BWAGPU_STAGE_SLOTS
// (1..BWAGPU_NUM_SLOTS, default 3 with a PostPool, else 2)
int stage_slots() {
  static const int n = [] {
    const char* e = getenv("BWAGPU_STAGE_SLOTS");
    // with a PostPool a third slot keeps the device fed while a finished
    // record is being posted from another
    return std::max(1, std::min(e ? atoi(e) : (PostPool::threads() > 0 ? 3 : 2), BWAGPU_NUM_SLOTS));
  }();
  return n;
}

RegionsRecord ChainsToRegionsGPU::on_cpu(const ChainsRecord& rec) {
  // finishUpOnCPU (FPGAPipeline.cpp:526-551): the whole record goes through
  // the CPU stage's body; a GPU batch is all-or-nothing, so start_seq = 0
  if (!cpu_stage_) throw std::runtime_error("GPU SW stage failed and no CPU stage to fall back to");
  n_cpu_.fetch_add(1);
  return cpu_stage_->compute(rec);
}

void ChainsToRegionsGPU::retire() {
  // the last accelerator worker switches the CPU stage's accx dispatch off
  // (FPGAPipeline.cpp:402-405, 528-529): queued records drain back to the CPU
  if (--n_active_ == 0) {
    reaper_.drain();  // the stage is done when its chains are freed
    if (cpu_stage_) cpu_stage_->setUseAccx(false);
  }
}

void ChainsToRegionsGPU::post_record(int wid, const ChainsRecord& rec, const bwagpu_alnreg_t* rg,
                                     const int32_t* nn, const int32_t* off) {
  const auto t0 = std::chrono::steady_clock::now();
  RegionsRecord out;
  out.start_idx = rec.start_idx;
  out.batch_num = rec.batch_num;
  out.seqs = rec.seqs;
  out.alnreg = FlatBatch::unpack_dense(rg, nn, off, rec.batch_num);
  if (own_ == ChainOwnership::kForward) {
    out.chains = rec.chains;  // RegionsToSam frees them (Pipeline.cpp:559)
  } else {
    reaper_.release(rec.chains, rec.batch_num);
    out.chains = nullptr;
  }
  ns_[3] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
  n_gpu_.fetch_add(1);
  if (wid < kMaxWorkers) per_worker_[wid].fetch_add(1);
  pushOutput(out);
}

void ChainsToRegionsGPU::compute(int wid) {
  bwagpu_ctx_t* ctx = env_ ? env_->ctx(wid) : nullptr;
  if (!ctx) {  // no device for this worker: leave every record to the CPU
    retire();
    return;
  }
  // up to BWAGPU_NUM_SLOTS records in flight (the SWTask ping-pong,
  // FPGAPipeline.cpp:374-386, widened: a batch's serial tail — the last
  // extension round and the redo pass — overlaps the next batches' kernels):
  // record k uses slot k % BWAGPU_NUM_SLOTS; waits are FIFO, so that slot is
  // free again
  // one FlatBatch per slot, reused record after record: its vectors keep their
  // capacity, so packing and the region copy-back write into pages already
  // faulted in (a fresh 40-MB set per record cost page faults on every byte)
  struct Job {
    ChainsRecord rec;
    FlatBatch* flat;
    int slot;
  };
  const int nslots = stage_slots();
  std::vector<FlatBatch> flats(nslots);
  std::deque<Job> inflight;
  long long submitted = 0;
  bool more = true;
  // slots whose finished record a PostPool thread is still turning into
  // regions (its results are read from the slot's pinned buffers)
  const bool async_post = PostPool::threads() > 0;
  std::unique_ptr<std::atomic<int>[]> posting(new std::atomic<int>[nslots]);
  for (int k = 0; k < nslots; ++k) posting[k].store(0);
  auto settle = [&](int k) {  // slot k's record posted
    while (posting[k].load(std::memory_order_acquire)) std::this_thread::sleep_for(std::chrono::microseconds(10));
  };
  auto settle_all = [&] {
    for (int k = 0; k < nslots; ++k) settle(k);
  };
  auto fail_all = [&](const char* what, int rc) {
    // fpgaHangError / fpgaResultsError path: recompute what is in flight on
    // the CPU, push it, retire this worker
    (void)what;
    (void)rc;
    for (auto& j : inflight) pushOutput(on_cpu(j.rec));
    inflight.clear();
    settle_all();
    retire();
  };
  for (;;) {
    if (more && inflight.size() < (size_t)nslots) {
      ChainsRecord rec;
      bool ready = getInput(rec);
      if (!ready && inflight.empty()) {
        while (!ready && !isFinal()) {  // poll like FPGAPipeline.cpp:394-399
          std::this_thread::sleep_for(std::chrono::microseconds(10));
          ready = getInput(rec);
        }
      }
      if (!ready && isFinal()) {
        ready = getInput(rec);  // a record may have landed just before the final flag
        if (!ready) more = false;
      }
      if (ready) {
        const int sl = (int)(submitted % nslots);
        settle(sl);
        inflight.push_back(Job{rec, &flats[sl], sl});
        Job& j = inflight.back();
        auto t0 = std::chrono::steady_clock::now();
        int rc = j.flat->pack_staged(ctx, j.slot, j.rec);
        auto t1 = std::chrono::steady_clock::now();
        if (rc == BWAGPU_OK) rc = bwagpu_chain2aln_submit(ctx, j.slot, &j.flat->c);
        ns_[0] += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
        ns_[1] += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t1).count();
        if (rc == BWAGPU_E_UNSUPPORTED || rc == BWAGPU_E_INVAL) {
          // this record only (e.g. a read longer than BWAGPU_MAX_READ_LEN):
          // CPU path for it, the device stays in service
          ChainsRecord r = j.rec;
          inflight.pop_back();
          pushOutput(on_cpu(r));
          continue;
        }
        if (rc != BWAGPU_OK) {
          fail_all("submit", rc);
          return;
        }
        ++submitted;
        continue;  // fill both slots before waiting
      }
    }
    if (inflight.empty()) {
      if (!more) break;
      continue;
    }
    Job& j = inflight.front();
    auto t0 = std::chrono::steady_clock::now();
    const int rc = bwagpu_chain2aln_wait(ctx, j.slot, nullptr, nullptr);  // results stay in pinned memory
    auto t1 = std::chrono::steady_clock::now();
    ns_[2] += std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
    if (rc == BWAGPU_E_RESULTS) {
      // a malformed record (a chain outside its contig: bwa would assert,
      // bwamem.c:669): the error path — reported, emitted with that chain
      // skipped; the CPU stage never sees it and the device stays in service
      n_failed_.fetch_add(1);
      fprintf(stderr, "[ChainsToRegionsGPU] record %llu: %s; its flagged chains are skipped\n",
              (unsigned long long)j.rec.start_idx, bwagpu_last_error(ctx));
    } else if (rc != BWAGPU_OK) {
      fail_all("wait", rc);
      return;
    }
    const bwagpu_alnreg_t* rg = nullptr;
    const int32_t* nn = nullptr;
    const int32_t* off = nullptr;
    if (bwagpu_chain2aln_results_dense(ctx, j.slot, &rg, &nn, &off) != BWAGPU_OK) {
      fail_all("results", BWAGPU_E_INVAL);
      return;
    }
    bwagpu_stats_t ds{};
    if (bwagpu_last_stats(ctx, j.slot, &ds) == BWAGPU_OK) {
      dev_ns_[0] += (long long)(ds.kernel_ms * 1e6);
      dev_ns_[1] += (long long)((ds.total_ms - ds.kernel_ms) * 1e6);
    }
    if (async_post) {
      const int sl = j.slot;
      posting[sl].store(1, std::memory_order_release);
      std::atomic<int>* flag = &posting[sl];
      poster_.post([this, wid, rec = j.rec, rg, nn, off, flag] {
        post_record(wid, rec, rg, nn, off);
        flag->store(0, std::memory_order_release);
      });
    } else {
      post_record(wid, j.rec, rg, nn, off);
    }
    inflight.pop_front();
  }
  settle_all();  // every record of this worker is downstream before it retires
  retire();
}
