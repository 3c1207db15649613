// capi.hip — implementation of the C ABI declared in include/bwagpu.h.
//
// One context = one device.  It owns the HBM-resident reference (pac +
// contig table), the scoring options, and BWAGPU_NUM_SLOTS independent
// submission slots, each with its own HIP stream, device buffers, pinned
// host staging and events — the MI355X form of the reference's two
// ping-ponged SWTask objects (src/fpga/FPGAPipeline.cpp:373-386,
// SWTask.cpp:40-104).  No C++ exception crosses the ABI.
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <functional>
#include <cstdio>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "align2.h"
#include "reg2aln.h"
#include "seed.h"
#include "chain.h"
#include "engine.h"

using namespace bwagpu;

namespace {

// A persistent pool for the host-side passes over a batch (the staging copy
// and check of bwagpu_chain2aln_submit, seeding's validation and staging):
// creating threads per call cost 20-50 us each, and far more when several
// stage workers submit at once.  host_parallel(nt, f) runs f(1..nt-1) on the
// pool and f(0) on the caller, and returns when all are done; pool tasks never
// wait on the pool, so concurrent callers cannot deadlock.
class PassPool {
 public:
  static PassPool& get() {
    static PassPool p(7);
    return p;
  }
  void post(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  ~PassPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }

 private:
  explicit PassPool(int n) {
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

template <typename F>
void host_parallel(int nt, F f) {
  if (nt <= 1) {
    f(0);
    return;
  }
  int left = nt - 1;  // decremented under m: the caller cannot unwind before the last task released it
  std::mutex m;
  std::condition_variable done;
  for (int t = 1; t < nt; ++t)
    PassPool::get().post([&, t] {
      f(t);
      std::lock_guard<std::mutex> g(m);
      if (--left == 0) done.notify_all();
    });
  f(0);
  std::unique_lock<std::mutex> g(m);
  done.wait(g, [&] { return left == 0; });
}


struct DevBuf {  // grow-only device buffer
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n + n / 4, 4096);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

struct HostBuf {  // grow-only pinned host buffer
  void* p = nullptr;
  size_t cap = 0;
  unsigned flags = hipHostMallocDefault;
  hipError_t ensure(size_t n) {
    if (n <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n + n / 4, 4096);
    hipError_t e = hipHostMalloc(&p, want, flags);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return (T*)p; }
};

// layout of one batch inside a slot's single input allocation
struct InLayout {
  size_t seq_off, seq, rco, cso, rid, frac, seeds, total;
  void make(const bwagpu_batch_t& b) {
    size_t o = 0;
    auto take = [&](size_t n) {
      size_t at = o;
      o += (n + 255) & ~(size_t)255;
      return at;
    };
    seq_off = take(sizeof(int64_t) * (size_t)(b.n_reads + 1));
    rco = take(sizeof(int32_t) * (size_t)(b.n_reads + 1));
    cso = take(sizeof(int32_t) * (size_t)(b.n_chains + 1));
    rid = take(sizeof(int32_t) * (size_t)b.n_chains);
    frac = take(sizeof(float) * (size_t)b.n_chains);
    seeds = take(sizeof(bwagpu_seed_t) * (size_t)b.n_seeds);
    seq = take((size_t)b.seq_bytes);
    total = o;
  }
};

struct Slot {
  // created on first use (lazy_stream): the device entry runs on the caller's
  // streams, and every stream a context creates takes a place on one of the
  // process's hardware queues (GPU_MAX_HW_QUEUES) the caller's streams and
  // the selection side streams share
  hipStream_t stream = nullptr;
  std::once_flag stream_once;
  hipError_t stream_err = hipSuccess;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev2 = nullptr, ev3 = nullptr;
  DevBuf d_in, d_win, d_srt, d_prog, d_desc, d_out, d_n, d_stats, d_lists, d_counts;
  DevBuf d_cread, d_ext, d_tasks, d_ctr, d_regpos, d_skipf, d_heavy, d_redo, d_rbits;  // speculative path
  DevBuf d_schain, d_hinfo, d_mat, d_cov, d_colent, d_qh, d_longc, d_sorth, d_stasks, d_ftask, d_ftaskR;
  SpecStreams spec;  // created on first use (choose_side)
  bool side_chosen = false;
  void release_scratch() {
    d_win.release(); d_srt.release(); d_prog.release(); d_desc.release(); d_lists.release(); d_counts.release();
    d_cread.release(); d_ext.release(); d_tasks.release(); d_ctr.release(); d_regpos.release(); d_skipf.release();
    d_heavy.release(); d_redo.release(); d_rbits.release(); d_schain.release(); d_hinfo.release(); d_mat.release(); d_cov.release(); d_colent.release(); d_longc.release();
    d_qh.release();
    d_sorth.release();
    d_stasks.release();
    d_ftask.release();
    d_ftaskR.release();
    if (spec.side) (void)hipStreamSynchronize(spec.side);
    if (spec.side) (void)hipStreamDestroy(spec.side);
    if (spec.fork) (void)hipEventDestroy(spec.fork);
    if (spec.join) (void)hipEventDestroy(spec.join);
    spec = SpecStreams{};
    side_chosen = false;
  }
  HostBuf h_in, h_out, h_n, h_stats;
  // the submit/wait path's results: regions written densely (read r's at
  // h_dense[h_off[r] ..]) by dense_copy_kernel straight into pinned memory;
  // h_out (the slot layout) is filled from them only when asked for
  HostBuf h_dense, h_off;
  DevBuf d_off;
  size_t in_rco = 0, in_cso = 0;  // where the batch's offsets sit in h_in
  bool slot_view = false;         // h_out holds the last batch's slot layout
  bool busy = false;
  // the last submitted batch finished and its results are in h_dense / h_n /
  // h_off (set by _wait; cleared by the next _submit, and never set when a
  // submit fails)
  bool has_results = false;
  // the finished batch's offsets, copied out of h_in by a _stage of the next
  // batch (which overwrites h_in) so that a later _results can still build
  // the slot layout
  bool kept = false;
  std::vector<int32_t> keep_rco, keep_cso;
  int32_t n_reads = 0, n_chains = 0, n_seeds = 0;
  std::chrono::steady_clock::time_point t_submit;
  bwagpu_stats_t last{};
  int64_t h2d = 0, d2h = 0;
};

hipError_t lazy_stream(Slot& s, hipStream_t* st) {
  std::call_once(s.stream_once, [&s] { s.stream_err = hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking); });
  *st = s.stream;
  return s.stream_err;
}

// Side-stream probes.  HIP maps every stream of the process onto one of
// GPU_MAX_HW_QUEUES hardware queues (4 on the pool's boxes), and work on two
// streams that share a queue runs in submission order: a selection side
// stream on the same queue as a caller stream serializes the two (the GRCh38
// regime leg of round 4: 2.56 against 1.75 ms per batch).
// Whether two streams share a queue is measured: a ~150 us spin on `a`, then
// an empty kernel on `b`; b done while a still spins = separate queues.
__global__ void side_probe_spin(uint64_t ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}
__global__ void side_probe_nop() {}

bool streams_concurrent(hipStream_t a, hipStream_t b) {
  hipEvent_t ea = nullptr, eb = nullptr;
  if (hipEventCreateWithFlags(&ea, hipEventDisableTiming) != hipSuccess) return false;
  if (hipEventCreateWithFlags(&eb, hipEventDisableTiming) != hipSuccess) {
    (void)hipEventDestroy(ea);
    return false;
  }
  hipLaunchKernelGGL(side_probe_spin, dim3(1), dim3(64), 0, a, (uint64_t)15000);
  bool conc = false;
  if (hipGetLastError() == hipSuccess && hipEventRecord(ea, a) == hipSuccess) {
    hipLaunchKernelGGL(side_probe_nop, dim3(1), dim3(64), 0, b);
    if (hipGetLastError() == hipSuccess && hipEventRecord(eb, b) == hipSuccess &&
        hipEventSynchronize(eb) == hipSuccess)
      conc = hipEventQuery(ea) == hipErrorNotReady;
  }
  (void)hipEventSynchronize(ea);
  (void)hipEventDestroy(ea);
  (void)hipEventDestroy(eb);
  return conc;
}

// Per-read offsets of the dense result layout: off[r] = n[0] + ... + n[r-1]
// (one workgroup; a batch has < 2^31 regions), written to the device (for the
// copy) and to pinned host memory (for the caller).
constexpr int kDenseScanBlock = 1024;
__global__ void __launch_bounds__(kDenseScanBlock) dense_scan_kernel(const int32_t* __restrict__ n, int nr,
                                                                     int32_t* __restrict__ off,
                                                                     int32_t* __restrict__ h_off) {
  __shared__ int32_t part[kDenseScanBlock];
  const int t = (int)threadIdx.x;
  const int per = (nr + kDenseScanBlock - 1) / kDenseScanBlock;
  const int r0 = min(t * per, nr), r1 = min(r0 + per, nr);
  int sum = 0;
  for (int r = r0; r < r1; ++r) sum += n[r];
  part[t] = sum;
  __syncthreads();
  for (int d = 1; d < kDenseScanBlock; d <<= 1) {  // inclusive scan of the parts
    const int v = t >= d ? part[t - d] : 0;
    __syncthreads();
    part[t] += v;
    __syncthreads();
  }
  int run = part[t] - sum;
  for (int r = r0; r < r1; ++r) {
    off[r] = run;
    h_off[r] = run;
    run += n[r];
  }
  if (t == kDenseScanBlock - 1) {
    off[nr] = part[t];
    h_off[nr] = part[t];
  }
}

// Regions of read r from its slots (chain_seed_off[read_chain_off[r]], the
// ABI's layout) to dense[off[r] ..], 16 lanes per read, 8-byte words: the
// D2H moves the sum of n (~1.8 regions per read on C2) instead of every seed slot.
__global__ void __launch_bounds__(256) dense_copy_kernel(const bwagpu_alnreg_t* __restrict__ out,
                                                         const int32_t* __restrict__ n,
                                                         const int32_t* __restrict__ off,
                                                         const int32_t* __restrict__ rco,
                                                         const int32_t* __restrict__ cso, int nr,
                                                         bwagpu_alnreg_t* __restrict__ dense) {
  constexpr int kW = (int)(sizeof(bwagpu_alnreg_t) / 8);
  const int r = (int)((blockIdx.x * 256u + threadIdx.x) >> 4), l = (int)(threadIdx.x & 15);
  if (r >= nr) return;
  const int words = n[r] * kW;
  const uint2* src = reinterpret_cast<const uint2*>(out + cso[rco[r]]);
  uint2* dst = reinterpret_cast<uint2*>(dense + off[r]);
  for (int w = l; w < words; w += 16) dst[w] = src[w];
}

}  // namespace

struct bwagpu_ctx {
  int device = 0;
  // caller streams seen by the spec path, and side streams retired after a
  // later caller turned out to share their hardware queue (choose_side)
  std::mutex side_mu;
  std::vector<hipStream_t> callers, side_graveyard;
  DevOpt opt{};
  DevRef ref{};
  bool own_pac = false;
  void* d_pac = nullptr;
  int64_t* d_ann_off = nullptr;
  int32_t* d_ann_len = nullptr;
  int watchdog_ms = 10000;
  int ext_form = 0;  // bwagpu_ctx_ext_form (the process default when made)
  Slot slot[BWAGPU_NUM_SLOTS];
  // bwagpu_chain2aln_device: the caller's streams, one per slot's scratch (a
  // stream always reuses the same scratch, so its launches never race)
  hipStream_t dev_stream[BWAGPU_NUM_SLOTS] = {};
  // ... and its own scratch (only the Dev buffers of these are used): the
  // submit/wait path's slots never share scratch with the device entry, so the
  // two entry points may run concurrently on one context
  Slot dev_scratch[BWAGPU_NUM_SLOTS];
  // ksw_align2 batches (bwagpu_align2_*): grow-only, reused across calls
  DevBuf a2_tasks, a2_q, a2_t, a2_out, a2_scratch, a2_lists, a2_counts, a2_boff;
  // mem_reg2aln batches (bwagpu_reg2aln_batch)
  DevBuf r2_tasks, r2_q, r2_out, r2_cig, r2_md, r2_lists, r2_z, r2_stats;
  // bins run concurrently on these (fork/join with events from the caller's stream)
  static constexpr int kA2Streams = 4;
  hipStream_t a2_st[kA2Streams] = {};
  hipEvent_t a2_fork = nullptr, a2_join[kA2Streams] = {};
  // seeding (bwagpu_set_bwt / bwagpu_collect_intv): the resident FM-index and
  // the batch buffers
  DevBuf bwt_words, sa_d, sa_in, sa_out, occ_d, sup_d, sa_full;
  DevBwt bwt{};
  bool has_bwt = false;
  DevBuf sd_off, sd_seq, sd_out, sd_n, sd_scratch, sd_poff, sd_pack, sd_heavy, sd_dbg;
  // seeding's chaining (bwagpu_seqs2chains / bwagpu_seqs2regions): per read,
  // per SA position, the kbtree arenas, mem_seed_sw tasks, the packed chains
  DevBuf ch_npos, ch_posoff, ch_frac, ch_nout, ch_noseed, ch_nsw, ch_need, ch_swtab, ch_alt;
  DevBuf ch_kpos, ch_rbeg, ch_qinfo, ch_label, ch_score, ch_slist, ch_ord, ch_chains, ch_nodes;
  DevBuf ch_ochains, ch_oslist, ch_bins, ch_dbg;
  DevBuf ch_swoff, ch_swtasks, ch_swt, ch_swskip, ch_swres, ch_swscr;
  DevBuf ch_ocoff, ch_osoff, ch_rco, ch_cso, ch_rid, ch_cfrac, ch_out, ch_seeds;
  DevBuf ch_regoff, ch_regc;
  HostBuf chh_tot, chh_rco, chh_cso, chh_chains, chh_seeds, chh_regs, chh_n;
  HostBuf sdh_in;  // the reads of a seeding call, staged for the H2D
  hipEvent_t sdh_done = nullptr;  // recorded after the H2D out of sdh_in
  Slot ch_slot;  // chain2aln scratch of bwagpu_seqs2regions
  ChainStreams ch_cs{};  // created on first use
  bool has_alt = false;
  // the FPGA wire format (bwagpu_sw_stream)
  DevBuf st_buf, st_start, st_q, st_tasks, st_lists, st_seen, st_ctr, st_out;
  // bwt_extend calls tier 1 spends on a read before tier 2 (one wave per read)
  // takes it: ~p90 of the C2 batch's per-read counts (mean 666, p90 975)
  int seed_budget = 1024;
  int sup_shift = 32;  // bwagpu_debug_sup_shift: superblock size of the next set_bwt
  int dev_read_len = BWAGPU_MAX_READ_LEN;  // bwagpu_set_device_read_len
  // bwagpu_debug_fail_wait: after fail_after more successful waits, _wait
  // returns fail_code once (tests of the stage's recovery path)
  int fail_after = -1, fail_code = 0;
  // bwagpu_prof_*: event pairs around the dominant extension launches
  std::vector<hipEvent_t> prof_ev;
  int prof_used = 0;
  std::string err;
};

namespace {

int fail(bwagpu_ctx_t* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

int hip_fail(bwagpu_ctx_t* c, hipError_t e, const char* what) {
  std::string m = std::string(what) + ": " + hipGetErrorString(e);
  if (e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation) return fail(c, BWAGPU_E_NOMEM, m);
  return fail(c, BWAGPU_E_DEVICE, m);
}

#define HIPC(call, what)                             \
  do {                                               \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) return hip_fail(ctx, e_, what); \
  } while (0)

bool make_opt(const bwagpu_opt_t* o, DevOpt* d, std::string* why) {
  if (!o) { *why = "opt is NULL"; return false; }
  if (o->e_del <= 0 || o->e_ins <= 0) { *why = "gap extension penalties must be > 0"; return false; }
  if (o->w < 0 || o->a < 0) { *why = "negative band width or match score"; return false; }
  // bounds under which the kernels' integer forms of the reference's double
  // expressions (cal_max_gap, the ksw_extend2 band clamp) are exact
  if (o->a > 127 || o->e_del > 65535 || o->e_ins > 65535 || o->o_del < 0 || o->o_del > 65535 || o->o_ins < 0 ||
      o->o_ins > 65535 || o->pen_clip5 < 0 || o->pen_clip5 >= (1 << 20) || o->pen_clip3 < 0 ||
      o->pen_clip3 >= (1 << 20) || o->w > (1 << 20)) {
    *why = "scoring option out of range";
    return false;
  }
  memset(d, 0, sizeof(*d));
  d->a = o->a;
  d->o_del = o->o_del;
  d->e_del = o->e_del;
  d->o_ins = o->o_ins;
  d->e_ins = o->e_ins;
  d->oe_del = o->o_del + o->e_del;
  d->oe_ins = o->o_ins + o->e_ins;
  d->pen_clip5 = o->pen_clip5;
  d->pen_clip3 = o->pen_clip3;
  d->w = o->w;
  d->zdrop = o->zdrop;
  int mx = 0;  // ksw.c:397-398 — max over the m*m matrix, starting from 0
  for (int i = 0; i < 25; ++i) mx = std::max<int>(mx, o->mat[i]);
  d->max_mat = mx;
  d->row_bound = 1;
  memcpy(d->mat, o->mat, 25);
  for (int q = 0; q < 5; ++q) {
    uint32_t w = 0;
    for (int t = 0; t < 4; ++t) w |= (uint32_t)(uint8_t)o->mat[t * 5 + q] << (8 * t);
    d->qprof[q] = w;
    d->qprof4[q] = o->mat[20 + q];
  }
  return true;
}

// ksw_qinit's profile (ksw.c:69-108) as v_perm byte pools, see A2Prof
A2Prof make_a2prof(const DevOpt& o, bool u8) {
  A2Prof P{};
  int mn = 127, mx = 0;
  for (int i = 0; i < 25; ++i) {
    mn = std::min<int>(mn, o.mat[i]);
    mx = std::max<int>(mx, o.mat[i]);
  }
  const int shift = (256 - (mn & 0xff)) & 0xff;
  const int bias = u8 ? shift : 128;
  for (int t = 0; t < 5; ++t) {
    uint32_t lo = 0;
    for (int q = 0; q < 4; ++q) lo |= (uint32_t)(uint8_t)(o.mat[t * 5 + q] + bias) << (8 * q);
    P.lo[t] = lo;
    P.hi[t] = (uint32_t)(uint8_t)(o.mat[t * 5 + 4] + bias) | (uint32_t)(uint8_t)bias << 8;
  }
  P.shift = shift;
  P.qmax = mx;
  P.e_del = o.e_del;
  P.oe_del = o.oe_del;
  P.e_ins = o.e_ins;
  P.oe_ins = o.oe_ins;
  return P;
}

// scoring limits of the align2 kernels (reasons are the E_UNSUPPORTED text)
const char* align2_opt_unsupported(const DevOpt& o) {
  if (o.o_ins <= 0)
    return "ksw_align2 with o_ins == 0: the reference's lazy-F early exit (ksw.c:180) then depends on "
           "its SIMD lane order; run it on the CPU";
  if (o.max_mat <= 0) return "ksw_align2 needs a positive match score (ksw.c:216 divides by it)";
  if (o.o_ins > 65535 || o.e_ins > 65535 || o.o_del > 65535 || o.e_del > 65535) return "gap penalty > 65535";
  return nullptr;
}

// Launch the given bins concurrently: fork the align2 streams off `st`,
// deal the bins (in the given order) round-robin over them, join back.
// counts_host: task count per bin when known (0 = unknown -> grid = capacity).
int launch_align2_concurrent(bwagpu_ctx_t* ctx, hipStream_t st, const std::vector<int>& bins, const A2Args& base,
                             const int32_t* list_off, const int32_t* counts_host, int32_t* d_counts,
                             int32_t* d_cursors, size_t list_stride);

int create_common(int device, const bwagpu_opt_t* opt, const bwagpu_bns_t* bns, bwagpu_ctx_t** out,
                  bwagpu_ctx_t** made) {
  if (!out || !bns || bns->l_pac <= 0 || bns->n_seqs <= 0 || !bns->ann_offset || !bns->ann_len)
    return BWAGPU_E_INVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return BWAGPU_E_NODEVICE;
  if (device < 0 || device >= n) return BWAGPU_E_NODEVICE;
  bwagpu_ctx_t* ctx = new (std::nothrow) bwagpu_ctx_t();
  if (!ctx) return BWAGPU_E_NOMEM;
  std::string why;
  if (!make_opt(opt, &ctx->opt, &why)) {
    delete ctx;
    return BWAGPU_E_INVAL;
  }
  ctx->device = device;
  ctx->ext_form = set_ext_form(-1);
  *made = ctx;
  HIPC(hipSetDevice(device), "hipSetDevice");
  HIPC(hipMalloc(&ctx->d_ann_off, sizeof(int64_t) * bns->n_seqs), "hipMalloc(ann_offset)");
  HIPC(hipMalloc(&ctx->d_ann_len, sizeof(int32_t) * bns->n_seqs), "hipMalloc(ann_len)");
  HIPC(hipMemcpy(ctx->d_ann_off, bns->ann_offset, sizeof(int64_t) * bns->n_seqs, hipMemcpyHostToDevice),
       "upload ann_offset");
  HIPC(hipMemcpy(ctx->d_ann_len, bns->ann_len, sizeof(int32_t) * bns->n_seqs, hipMemcpyHostToDevice),
       "upload ann_len");
  for (auto& s : ctx->slot) {
    HIPC(hipEventCreate(&s.ev0), "hipEventCreate");
    HIPC(hipEventCreate(&s.ev1), "hipEventCreate");
    HIPC(hipEventCreate(&s.ev2), "hipEventCreate");
    HIPC(hipEventCreate(&s.ev3), "hipEventCreate");
  }
  ctx->ref.l_pac = bns->l_pac;
  ctx->ref.n_seqs = bns->n_seqs;
  ctx->ref.ann_offset = ctx->d_ann_off;
  ctx->ref.ann_len = ctx->d_ann_len;
  return BWAGPU_OK;
}

// every Slot of a context whose spec path may hold a side stream
std::vector<Slot*> all_slots(bwagpu_ctx_t* ctx) {
  std::vector<Slot*> v;
  for (auto& x : ctx->slot) v.push_back(&x);
  for (auto& x : ctx->dev_scratch) v.push_back(&x);
  v.push_back(&ctx->ch_slot);
  return v;
}

void destroy_ctx(bwagpu_ctx_t* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (auto& s : ctx->slot) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    s.d_in.release(); s.release_scratch();
    s.d_out.release(); s.d_n.release(); s.d_stats.release();
    s.h_in.release(); s.h_out.release(); s.h_n.release(); s.h_stats.release();
    s.h_dense.release(); s.h_off.release(); s.d_off.release();
    if (s.ev0) (void)hipEventDestroy(s.ev0);
    if (s.ev1) (void)hipEventDestroy(s.ev1);
    if (s.ev2) (void)hipEventDestroy(s.ev2);
    if (s.ev3) (void)hipEventDestroy(s.ev3);
    if (s.stream) (void)hipStreamDestroy(s.stream);
  }
  for (int k = 0; k < BWAGPU_NUM_SLOTS; ++k) {
    if (ctx->dev_stream[k]) (void)hipStreamSynchronize(ctx->dev_stream[k]);
    Slot& s = ctx->dev_scratch[k];
    s.release_scratch();
    s.d_stats.release();
  }
  if (ctx->sdh_done) {
    (void)hipEventSynchronize(ctx->sdh_done);
    (void)hipEventDestroy(ctx->sdh_done);
  }
  for (hipStream_t x : ctx->side_graveyard) {
    (void)hipStreamSynchronize(x);
    (void)hipStreamDestroy(x);
  }
  ctx->side_graveyard.clear();
  for (hipEvent_t e : ctx->prof_ev) (void)hipEventDestroy(e);
  ctx->prof_ev.clear();
  for (int i = 0; i < bwagpu_ctx::kA2Streams; ++i) {
    if (ctx->a2_st[i]) (void)hipStreamSynchronize(ctx->a2_st[i]);
    if (ctx->a2_st[i]) (void)hipStreamDestroy(ctx->a2_st[i]);
    if (ctx->a2_join[i]) (void)hipEventDestroy(ctx->a2_join[i]);
  }
  if (ctx->a2_fork) (void)hipEventDestroy(ctx->a2_fork);
  ctx->a2_tasks.release(); ctx->a2_q.release(); ctx->a2_t.release(); ctx->a2_out.release();
  ctx->a2_scratch.release(); ctx->a2_lists.release(); ctx->a2_counts.release(); ctx->a2_boff.release();
  ctx->ch_slot.release_scratch();
  for (int k = 0; k < 2; ++k) {
    if (ctx->ch_cs.side[k]) (void)hipStreamSynchronize(ctx->ch_cs.side[k]);
    if (ctx->ch_cs.side[k]) (void)hipStreamDestroy(ctx->ch_cs.side[k]);
    if (ctx->ch_cs.join[k]) (void)hipEventDestroy(ctx->ch_cs.join[k]);
  }
  if (ctx->ch_cs.fork) (void)hipEventDestroy(ctx->ch_cs.fork);
  ctx->ch_slot.d_out.release(); ctx->ch_slot.d_n.release(); ctx->ch_slot.d_stats.release();
  for (DevBuf* b : {&ctx->r2_tasks, &ctx->r2_q, &ctx->r2_out, &ctx->r2_cig, &ctx->r2_md, &ctx->r2_lists, &ctx->r2_z,
                    &ctx->r2_stats, &ctx->bwt_words, &ctx->sa_d, &ctx->sa_in, &ctx->sa_out, &ctx->occ_d, &ctx->sup_d, &ctx->sa_full, &ctx->sd_off,
                    &ctx->sd_seq, &ctx->sd_out, &ctx->sd_n, &ctx->sd_scratch, &ctx->sd_poff, &ctx->sd_pack,
                    &ctx->sd_heavy, &ctx->sd_dbg, &ctx->st_buf, &ctx->st_start, &ctx->st_q, &ctx->st_tasks, &ctx->st_lists,
                    &ctx->st_seen, &ctx->st_ctr, &ctx->st_out, &ctx->ch_npos, &ctx->ch_posoff, &ctx->ch_frac,
                    &ctx->ch_nout, &ctx->ch_noseed, &ctx->ch_nsw, &ctx->ch_need, &ctx->ch_swtab, &ctx->ch_alt,
                    &ctx->ch_kpos, &ctx->ch_rbeg, &ctx->ch_qinfo, &ctx->ch_label, &ctx->ch_score, &ctx->ch_slist,
                    &ctx->ch_ord, &ctx->ch_chains, &ctx->ch_nodes, &ctx->ch_ochains, &ctx->ch_oslist, &ctx->ch_bins, &ctx->ch_dbg, &ctx->ch_swoff, &ctx->ch_swtasks, &ctx->ch_swt,
                    &ctx->ch_swskip, &ctx->ch_swres, &ctx->ch_swscr, &ctx->ch_ocoff, &ctx->ch_osoff, &ctx->ch_rco,
                    &ctx->ch_cso, &ctx->ch_rid, &ctx->ch_cfrac, &ctx->ch_out, &ctx->ch_seeds, &ctx->ch_regoff,
                    &ctx->ch_regc})
    b->release();
  for (HostBuf* b : {&ctx->sdh_in, &ctx->chh_tot, &ctx->chh_rco, &ctx->chh_cso, &ctx->chh_chains, &ctx->chh_seeds, &ctx->chh_regs,
                     &ctx->chh_n})
    b->release();
  if (ctx->own_pac && ctx->d_pac) (void)hipFree(ctx->d_pac);
  if (ctx->d_ann_off) (void)hipFree(ctx->d_ann_off);
  if (ctx->d_ann_len) (void)hipFree(ctx->d_ann_len);
  delete ctx;
}

// validate the flattened batch on the host (cheap O(n) checks so that a
// malformed batch is an E_INVAL here, never an out-of-bounds access on device);
// one pass over reads -> chains -> seeds, which also yields the longest read
// the batch's dimensions and array pointers (O(1)): what the staging copy relies on
int check_batch_header(bwagpu_ctx_t* ctx, const bwagpu_batch_t* b) {
  if (!b) return fail(ctx, BWAGPU_E_INVAL, "batch is NULL");
  if (b->n_reads < 0 || b->n_chains < 0 || b->n_seeds < 0 || b->seq_bytes < 0)
    return fail(ctx, BWAGPU_E_INVAL, "negative batch dimension");
  if (b->n_reads == 0) return BWAGPU_OK;
  if (!b->seq_off || !b->read_chain_off || !b->chain_seed_off)
    return fail(ctx, BWAGPU_E_INVAL, "NULL offset array");
  if (b->seq_off[0] != 0 || b->seq_off[b->n_reads] != b->seq_bytes)
    return fail(ctx, BWAGPU_E_INVAL, "seq_off does not span seq_bytes");
  if (b->read_chain_off[0] != 0 || b->read_chain_off[b->n_reads] != b->n_chains)
    return fail(ctx, BWAGPU_E_INVAL, "read_chain_off does not span n_chains");
  if (b->chain_seed_off[0] != 0 || b->chain_seed_off[b->n_chains] != b->n_seeds)
    return fail(ctx, BWAGPU_E_INVAL, "chain_seed_off does not span n_seeds");
  if (b->n_chains && (!b->chain_rid || !b->chain_frac_rep)) return fail(ctx, BWAGPU_E_INVAL, "NULL chain array");
  if (b->n_seeds && !b->seeds) return fail(ctx, BWAGPU_E_INVAL, "NULL seeds");
  if (b->seq_bytes && !b->seq) return fail(ctx, BWAGPU_E_INVAL, "NULL seq");
  return BWAGPU_OK;
}

// reads [r0, r1) of a header-checked batch: seq_off and the offsets monotone,
// every read at most BWAGPU_MAX_READ_LEN (*bad_read), every seed inside its
// read and inside [0, 2*l_pac).  -> 0 ok, 1 seq_off, 2 read too long, 3 rco,
// 4 cso, 5 seed; *lmax = the longest read.
int check_reads(const bwagpu_batch_t* b, int64_t l_pac, int r0, int r1, int64_t* lmax, int* bad_read) {
  const int64_t two = l_pac << 1;
  const int64_t* so = b->seq_off;
  const int32_t* rco = b->read_chain_off;
  const int32_t* cso = b->chain_seed_off;
  const bwagpu_seed_t* sd = b->seeds;
  int64_t lm = 0;
  for (int r = r0; r < r1; ++r) {
    const int64_t l = so[r + 1] - so[r];
    if (l < 0) return 1;
    if (l > BWAGPU_MAX_READ_LEN) {
      *bad_read = r;
      return 2;
    }
    lm = std::max(lm, l);
    // every offset is range-checked BEFORE it indexes: a range may start
    // anywhere, and a later read's failing check must not come after an
    // earlier read walked past the caller's arrays
    const int c0 = rco[r], c1 = rco[r + 1];
    if (c0 < 0 || c1 < c0 || c1 > b->n_chains) return 3;
    bool bad_seed = false;
    for (int c = c0; c < c1; ++c) {
      const int k0 = cso[c], k1 = cso[c + 1];
      if (k0 < 0 || k1 < k0 || k1 > b->n_seeds) return 4;
      for (int k = k0; k < k1; ++k) {  // branch-free accumulation: one test per read
        const bwagpu_seed_t& s = sd[k];
        bad_seed |= (s.qbeg < 0) | (s.len <= 0) | ((int64_t)s.qbeg + s.len > l) | (s.rbeg < 0) | (s.rbeg + s.len > two);
      }
    }
    if (bad_seed) return 5;
  }
  *lmax = lm;
  return 0;
}

// the first failing range's code as one sequential pass would report it
int check_report(bwagpu_ctx_t* ctx, const bwagpu_batch_t* b, const int* code, const int* bad_read, int nt) {
  for (int t = 0; t < nt; ++t) {
    switch (code[t]) {
      case 1: return fail(ctx, BWAGPU_E_INVAL, "seq_off not monotone");
      case 2: {
        char m[128];
        snprintf(m, sizeof m, "read %d has length %lld > %d", bad_read[t],
                 (long long)(b->seq_off[bad_read[t] + 1] - b->seq_off[bad_read[t]]), BWAGPU_MAX_READ_LEN);
        return fail(ctx, BWAGPU_E_UNSUPPORTED, m);
      }
      case 3: return fail(ctx, BWAGPU_E_INVAL, "read_chain_off not monotone");
      case 4: return fail(ctx, BWAGPU_E_INVAL, "chain_seed_off not monotone");
      case 5: return fail(ctx, BWAGPU_E_INVAL, "seed outside its read or the reference");
      default: break;
    }
  }
  return BWAGPU_OK;
}

// every read, chain and seed (O(n), after check_batch_header): the longest read -> *lq_max_out
int check_batch_seeds(bwagpu_ctx_t* ctx, const bwagpu_batch_t* b, int* lq_max_out) {
  *lq_max_out = 0;
  if (b->n_reads == 0) return BWAGPU_OK;
  const int nt = b->n_seeds >= (1 << 16) ? 4 : 1;
  int code[4] = {0, 0, 0, 0}, bad_read[4] = {0, 0, 0, 0};
  int64_t lmaxs[4] = {0, 0, 0, 0};
  host_parallel(nt, [&](int t) {
    code[t] = check_reads(b, ctx->ref.l_pac, (int)((int64_t)b->n_reads * t / nt),
                          (int)((int64_t)b->n_reads * (t + 1) / nt), &lmaxs[t], &bad_read[t]);
  });
  if (int rc = check_report(ctx, b, code, bad_read, nt)) return rc;
  *lq_max_out = (int)std::max(std::max(lmaxs[0], lmaxs[1]), std::max(lmaxs[2], lmaxs[3]));
  return BWAGPU_OK;
}

// The staging copy and the check in one pass (bwagpu_chain2aln_submit): nt
// threads, each a read range in blocks of 1024 reads — a block's arrays are
// copied into the pinned staging buffer h (layout L), then checked while still
// in cache.  A block's copy ranges come from its boundary offsets, which are
// range-checked first, so a malformed batch never makes the copy leave the
// caller's arrays (sizes from the header); it is refused after the pass.
int stage_and_check(bwagpu_ctx_t* ctx, const bwagpu_batch_t* b, char* h, const InLayout& L, int* lq_max_out) {
  *lq_max_out = 0;
  const int nr = b->n_reads;
  if (nr == 0) return BWAGPU_OK;
  constexpr int kBlk = 1024, kMaxT = 8;
  const int nt = b->n_seeds >= (1 << 16) ? kMaxT : 1;
  const int nblk = (nr + kBlk - 1) / kBlk;
  int code[kMaxT] = {}, bad_read[kMaxT] = {};
  int64_t lmaxs[kMaxT] = {};
  auto work = [&](int t) {
    // this thread's blocks: [nblk*t/nt, nblk*(t+1)/nt), in order
    for (int k = (int)((int64_t)nblk * t / nt), ke = (int)((int64_t)nblk * (t + 1) / nt); k < ke; ++k) {
      const int r0 = k * kBlk, r1 = std::min(nr, r0 + kBlk);
      const int64_t b0 = b->seq_off[r0], b1 = b->seq_off[r1];
      const int c0 = b->read_chain_off[r0], c1 = b->read_chain_off[r1];
      if (b0 < 0 || b1 < b0 || b1 > b->seq_bytes) {
        code[t] = 1;
        return;
      }
      if (c0 < 0 || c1 < c0 || c1 > b->n_chains) {
        code[t] = 3;
        return;
      }
      const int k0 = b->chain_seed_off[c0], k1 = b->chain_seed_off[c1];
      if (k0 < 0 || k1 < k0 || k1 > b->n_seeds) {
        code[t] = 4;
        return;
      }
      const int re = r1 == nr ? r1 + 1 : r1, ce = c1 == b->n_chains ? c1 + 1 : c1;  // the last block: the end offsets
      memcpy(h + L.seq_off + sizeof(int64_t) * r0, b->seq_off + r0, sizeof(int64_t) * (size_t)(re - r0));
      memcpy(h + L.rco + sizeof(int32_t) * r0, b->read_chain_off + r0, sizeof(int32_t) * (size_t)(re - r0));
      memcpy(h + L.cso + sizeof(int32_t) * c0, b->chain_seed_off + c0, sizeof(int32_t) * (size_t)(ce - c0));
      if (c1 > c0) {
        memcpy(h + L.rid + sizeof(int32_t) * c0, b->chain_rid + c0, sizeof(int32_t) * (size_t)(c1 - c0));
        memcpy(h + L.frac + sizeof(float) * c0, b->chain_frac_rep + c0, sizeof(float) * (size_t)(c1 - c0));
      }
      if (k1 > k0) memcpy(h + L.seeds + sizeof(bwagpu_seed_t) * k0, b->seeds + k0, sizeof(bwagpu_seed_t) * (size_t)(k1 - k0));
      if (b1 > b0) memcpy(h + L.seq + b0, b->seq + b0, (size_t)(b1 - b0));
      int64_t lm = 0;
      if ((code[t] = check_reads(b, ctx->ref.l_pac, r0, r1, &lm, &bad_read[t]))) return;
      lmaxs[t] = std::max(lmaxs[t], lm);
    }
  };
  host_parallel(nt, work);
  if (int rc = check_report(ctx, b, code, bad_read, nt)) return rc;
  int64_t lm = 0;
  for (int t = 0; t < nt; ++t) lm = std::max(lm, lmaxs[t]);
  *lq_max_out = (int)lm;
  return BWAGPU_OK;
}

// LDS row-buffer bytes per group for reads up to lq_max (see rows_needed)
int tb_bytes_for(const DevOpt& o, int lq_max) {
  const int eb = std::max(o.pen_clip5, o.pen_clip3);
  const int cap = std::max(band_cap(lq_max, o.max_mat, eb, o.o_ins, o.e_ins),
                           band_cap(lq_max, o.max_mat, eb, o.o_del, o.e_del));
  const int we = std::min(o.w << 1, cap);
  const int n = lq_max + we + 2;
  return (n + 15) & ~15;
}

// BWAGPU_C2A_PATH=fast: the wave-per-read kernels (chain2aln_fast_kernel /
// chain2aln_kernel, DESIGN.md §3 "per-read kernels"); default: the speculative
// path (extension tasks + selection passes)
bool use_read_kernels() {
  const char* e = getenv("BWAGPU_C2A_PATH");
  return e && (strcmp(e, "fast") == 0 || strcmp(e, "read") == 0);
}

// dynamic LDS bytes of variant v's launch for reads up to lq_max
size_t variant_lds(const DevOpt& o, int v, int lq_max) {
  const Variant& vk = kVariants[v];
  const int lqv = std::min(lq_max, vk.max_len());
  const int tb = tb_bytes_for(o, std::max(lqv, 1));
  return vk.kind == VK_FAST ? (size_t)(kBlock / 64) * fast_wave_lds(tb) : (size_t)tb * (kBlock / vk.G);
}

// Options that need more LDS per workgroup than a launch may take are refused
// BEFORE anything is enqueued (a refusal after the H2D would leave a DMA
// reading the slot's pinned staging buffer while the caller reuses the slot).
int check_lds(bwagpu_ctx_t* ctx, int lq_max) {
  if (!use_read_kernels()) {
    if (spec_redo_cap(tb_bytes_for(ctx->opt, std::max(lq_max, 1))) < 64)
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "LDS row buffer too large for these options (w, pen_clip, read length)");
    return BWAGPU_OK;
  }
  for (int v = 0; v < kNumVariants; ++v) {
    if (variant_lds(ctx->opt, v, lq_max) > 64 * 1024)
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "LDS row buffer too large for these options (w, pen_clip, read length)");
  }
  return BWAGPU_OK;
}

// The caller stream st of a spec-path batch: a side stream for its heavy
// selection kernels on a hardware queue that none of this context's caller
// streams and other side streams use (streams_concurrent), or none at all
// (the heavy selection then runs on st) when six candidates all share one.
// A caller stream seen for the first time retires the side streams that share
// its queue (their slots choose again at their next batch).
void register_caller_locked(bwagpu_ctx_t* ctx, hipStream_t st) {
  for (hipStream_t c : ctx->callers)
    if (c == st) return;
  for (Slot* x : all_slots(ctx))
    if (x->side_chosen && x->spec.side && hipStreamSynchronize(x->spec.side) == hipSuccess &&
        !streams_concurrent(x->spec.side, st)) {  // spin on the (drained) side, probe st
      ctx->side_graveyard.push_back(x->spec.side);  // may still hold queued work: destroyed with the context
      x->spec.side = nullptr;
      x->side_chosen = false;
    }
  ctx->callers.push_back(st);
}

// *snap: the slot's streams as of this call, copied under side_mu — a later
// caller stream may retire s.spec.side from another thread (register_caller_locked)
// while this slot's launches are being enqueued; they use the copy (a retired
// side stream stays alive in the graveyard until the context goes)
hipError_t choose_side(bwagpu_ctx_t* ctx, Slot& s, hipStream_t st, SpecStreams* snap) {
  std::lock_guard<std::mutex> g(ctx->side_mu);
  register_caller_locked(ctx, st);
  if (s.side_chosen) {
    *snap = s.spec;
    return hipSuccess;
  }
  if (!s.spec.fork) {
    hipError_t e = hipEventCreateWithFlags(&s.spec.fork, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&s.spec.join, hipEventDisableTiming);
    if (e != hipSuccess) return e;
  }
  std::vector<hipStream_t> avoid = ctx->callers;
  for (Slot* x : all_slots(ctx))
    if (x != &s && x->side_chosen && x->spec.side) avoid.push_back(x->spec.side);
  std::vector<hipStream_t> tried;  // kept until the end: each holds its queue's place
  hipStream_t pick = nullptr;
  hipError_t e = hipSuccess;
  for (int t = 0; t < 6 && !pick; ++t) {
    hipStream_t c = nullptr;
    if ((e = hipStreamCreateWithFlags(&c, hipStreamNonBlocking)) != hipSuccess) break;
    bool ok = true;
    for (hipStream_t a : avoid)
      if (!streams_concurrent(c, a)) {  // spin on the candidate, never on a caller stream
        ok = false;
        break;
      }
    if (ok) pick = c;
    else tried.push_back(c);
  }
  for (hipStream_t c : tried) (void)hipStreamDestroy(c);  // only the probe ran on them
  if (e != hipSuccess) return e;
  s.spec.side = pick;
  s.side_chosen = true;
  *snap = s.spec;
  return hipSuccess;
}

int enqueue_spec(bwagpu_ctx_t* ctx, Slot& s, const DevBatch& db, int lq_max, bwagpu_alnreg_t* d_out, int32_t* d_n,
                 int64_t* d_stats, hipStream_t st) {
  const size_t nc = (size_t)std::max(db.n_chains, 1), ns = (size_t)std::max(db.n_seeds, 1),
               nr = (size_t)std::max(db.n_reads, 1);
  HIPC(s.d_win.ensure(sizeof(ChainWin) * nc), "hipMalloc(win)");
  HIPC(s.d_cread.ensure(sizeof(int32_t) * nc), "hipMalloc(chain_read)");
  HIPC(s.d_prog.ensure(sizeof(bwagpu_seed_t) * ns), "hipMalloc(prog)");
  HIPC(s.d_ext.ensure(sizeof(SeedExt) * ns), "hipMalloc(ext)");
  HIPC(s.d_tasks.ensure(sizeof(int2) * kSpecBins * (nc + (kSpecRounds - 1) * ns)), "hipMalloc(tasks)");
  HIPC(s.d_ctr.ensure(sizeof(int32_t) * SPC_WORDS), "hipMalloc(ctr)");
  HIPC(s.d_regpos.ensure(sizeof(int32_t) * ns), "hipMalloc(regpos)");
  HIPC(s.d_skipf.ensure(sizeof(int32_t) * ns), "hipMalloc(skipf)");
  HIPC(s.d_heavy.ensure(sizeof(int32_t) * nr), "hipMalloc(heavy)");
  HIPC(s.d_redo.ensure(sizeof(int32_t) * nr), "hipMalloc(redo)");
  HIPC(s.d_rbits.ensure(sizeof(uint32_t) * (nr / 32 + 1)), "hipMalloc(rbits)");
  HIPC(s.d_desc.ensure(sizeof(ReadDesc) * nr), "hipMalloc(desc)");
  HIPC(s.d_schain.ensure(sizeof(int32_t) * ns), "hipMalloc(seedchain)");
  HIPC(s.d_hinfo.ensure(sizeof(int4) * nr), "hipMalloc(hinfo)");
  HIPC(s.d_cov.ensure(sizeof(int32_t) * ns), "hipMalloc(cov)");
  HIPC(s.d_colent.ensure(sizeof(int32_t) * ns), "hipMalloc(colent)");
  HIPC(s.d_longc.ensure(sizeof(int32_t) * nc), "hipMalloc(longc)");
  HIPC(s.d_qh.ensure(sizeof(int32_t) * kQHWords), "hipMalloc(qh)");
  HIPC(s.d_sorth.ensure(sizeof(int32_t) * kSortWords), "hipMalloc(sorth)");
  HIPC(s.d_stasks.ensure(sizeof(int2) * kSpecBins * (nc + (kSpecRounds - 1) * ns)), "hipMalloc(stasks)");
  HIPC(s.d_ftask.ensure(sizeof(FatTask) * kSpecBins * (nc + (kSpecRounds - 1) * ns)), "hipMalloc(ftask)");
  HIPC(s.d_ftaskR.ensure(sizeof(FatTask) * kSpecBins * (nc + (kSpecRounds - 1) * ns)), "hipMalloc(ftaskR)");
  // pair matrices of heavy reads: sum over them of 2 * ns * ceil(ns / 64) words,
  // <= 2 * ns_total * (1 + ns_max / 64); reads that do not fit take the per-seed kernel
  const int64_t mat_words = std::max<int64_t>(1 << 20, 16 * (int64_t)ns);
  HIPC(s.d_mat.ensure(sizeof(uint64_t) * (size_t)mat_words), "hipMalloc(mat)");
  SpecArgs a;
  a.win = s.d_win.as<ChainWin>();
  a.chain_read = s.d_cread.as<int32_t>();
  a.prog = s.d_prog.as<bwagpu_seed_t>();
  a.ext = s.d_ext.as<SeedExt>();
  a.tasks = s.d_tasks.as<int2>();
  a.ctr = s.d_ctr.as<int32_t>();
  a.regpos = s.d_regpos.as<int32_t>();
  a.skipf = s.d_skipf.as<int32_t>();
  a.heavy = s.d_heavy.as<int32_t>();
  a.redo = s.d_redo.as<int32_t>();
  a.rbits = s.d_rbits.as<uint32_t>();
  a.rdesc = s.d_desc.as<ReadDesc>();
  a.seedchain = s.d_schain.as<int32_t>();
  a.hinfo = s.d_hinfo.as<int4>();
  a.mat = s.d_mat.as<uint64_t>();
  a.mat_words = (int64_t)(s.d_mat.cap / sizeof(uint64_t));
  a.cov = s.d_cov.as<int32_t>();
  a.colent = s.d_colent.as<int32_t>();
  a.longc = s.d_longc.as<int32_t>();
  a.qh = s.d_qh.as<int32_t>();
  a.sorth = s.d_sorth.as<int32_t>();
  a.stasks = s.d_stasks.as<int2>();
  a.ftask = s.d_ftask.as<FatTask>();
  a.ftaskR = s.d_ftaskR.as<FatTask>();
  static const int ext_prefetch = [] {  // A/B knob of the claim-ahead
    const char* e = getenv("BWAGPU_EXT_PREFETCH");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  a.ext_prefetch = ext_prefetch;
  static const int risky_first = [] {  // A/B knob (neutral, off)
    const char* e = getenv("BWAGPU_LIGHT_RISKY_FIRST");
    return e && e[0] == '1';
  }();
  a.risky_first = risky_first;
  static const int emu_strict = [] {  // A/B knob (0: misses extended inline)
    const char* e = getenv("BWAGPU_EMU_STRICT");
    return !(e && e[0] == '0');
  }();
  a.emu_strict = emu_strict;
  a.out = d_out;
  a.out_n = d_n;
  a.stats = d_stats;
  SpecStreams ss;
  HIPC(choose_side(ctx, s, st, &ss), "side stream");
  a.lq_bound = lq_max;
  const int tb = tb_bytes_for(ctx->opt, std::max(lq_max, 1));
  ss.form = ctx->ext_form;
  ss.pool = ctx->prof_ev.empty() ? nullptr : ctx->prof_ev.data();
  ss.pool_n = (int)ctx->prof_ev.size();
  ss.pool_used = &ctx->prof_used;
  // the batch's zeroed state (counters, queue heads, sort histograms, the
  // round-B bits, SeedExt slots, region counts): one launch, not six memsets
  HIPC(launch_spec_clear(a, db.n_reads, db.n_seeds, st), "spec clear");
  HIPC(launch_spec_chain2aln(ctx->opt, ctx->ref, db, a, tb, lq_max, st, ss), "spec chain2aln launch");
  return BWAGPU_OK;
}

// enqueue prep + binning + the per-variant kernels for a batch whose arrays
// are already in device memory (check_lds has passed for lq_max)
int enqueue_chain2aln(bwagpu_ctx_t* ctx, Slot& s, const DevBatch& db, int lq_max, bwagpu_alnreg_t* d_out,
                      int32_t* d_n, int64_t* d_stats, hipStream_t st) {
  if (!use_read_kernels()) return enqueue_spec(ctx, s, db, lq_max, d_out, d_n, d_stats, st);
  HIPC(s.d_win.ensure(sizeof(ChainWin) * (size_t)std::max(db.n_chains, 1)), "hipMalloc(win)");
  HIPC(s.d_srt.ensure(sizeof(uint64_t) * (size_t)std::max(db.n_seeds, 1)), "hipMalloc(srt)");
  HIPC(s.d_prog.ensure(sizeof(bwagpu_seed_t) * (size_t)std::max(db.n_seeds, 1)), "hipMalloc(prog)");
  const size_t nr = (size_t)std::max(db.n_reads, 1);
  HIPC(s.d_desc.ensure(sizeof(ReadDesc) * nr), "hipMalloc(desc)");
  // bins | read_list, n_reads each
  HIPC(s.d_lists.ensure(2 * sizeof(int32_t) * nr), "hipMalloc(lists)");
  int32_t* bins = s.d_lists.as<int32_t>();
  int32_t* read_list = bins + nr;
  HIPC(s.d_counts.ensure(sizeof(int32_t) * kCountWords), "hipMalloc(counts)");
  HIPC(hipMemsetAsync(s.d_counts.p, 0, sizeof(int32_t) * kCountWords, st), "memset counts");
  if (db.n_reads) HIPC(hipMemsetAsync(d_n, 0, sizeof(int32_t) * db.n_reads, st), "memset out_n");
  HIPC(launch_chain_prep(ctx->opt, ctx->ref, db, s.d_win.as<ChainWin>(), s.d_srt.as<uint64_t>(),
                         s.d_prog.as<bwagpu_seed_t>(), d_stats, st),
       "chain_prep launch");
  HIPC(launch_read_order(db, bins, s.d_counts.as<int32_t>() + kHistOff, s.d_counts.as<int32_t>(),
                         s.d_desc.as<ReadDesc>(), read_list, d_stats, st),
       "read order launch");
  C2AArgs a;
  a.read_list = read_list;
  a.desc = s.d_desc.as<ReadDesc>();
  a.counts = s.d_counts.as<int32_t>();
  a.win = s.d_win.as<ChainWin>();
  a.srt = s.d_srt.as<uint64_t>();
  a.prog = s.d_prog.as<bwagpu_seed_t>();
  a.out = d_out;
  a.out_n = d_n;
  a.stats = d_stats;
  for (int v = 0; v < kNumVariants; ++v) {
    const int lqv = std::min(lq_max, kVariants[v].max_len());
    const int tb = tb_bytes_for(ctx->opt, std::max(lqv, 1));
    HIPC(launch_chain2aln(v, ctx->opt, ctx->ref, db, db.n_reads, tb, a, st), "chain2aln launch");
  }
  return BWAGPU_OK;
}

}  // namespace

extern "C" {

int bwagpu_abi_version(void) { return BWAGPU_ABI_VERSION; }

int bwagpu_device_count(int* n) {
  if (!n) return BWAGPU_E_INVAL;
  int k = 0;
  if (hipGetDeviceCount(&k) != hipSuccess) k = 0;
  *n = k;
  return k > 0 ? BWAGPU_OK : BWAGPU_E_NODEVICE;
}

int bwagpu_create(int device, const bwagpu_opt_t* opt, const bwagpu_bns_t* bns, const uint8_t* pac_host,
                  bwagpu_ctx_t** out) {
  if (!pac_host) return BWAGPU_E_INVAL;
  bwagpu_ctx_t* ctx = nullptr;
  int rc = create_common(device, opt, bns, out, &ctx);
  if (rc == BWAGPU_OK) {
    const size_t pac_bytes = (size_t)(bns->l_pac / 4 + 1);  // bwa.c:281-282
    hipError_t e = hipMalloc(&ctx->d_pac, pac_bytes);
    if (e == hipSuccess) {
      ctx->own_pac = true;
      e = hipMemcpy(ctx->d_pac, pac_host, pac_bytes, hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) rc = hip_fail(ctx, e, "pac upload");
    ctx->ref.pac = (const uint8_t*)ctx->d_pac;
  }
  if (rc != BWAGPU_OK) {
    destroy_ctx(ctx);
    return rc;
  }
  *out = ctx;
  return BWAGPU_OK;
}

int bwagpu_create_resident(int device, const bwagpu_opt_t* opt, const bwagpu_bns_t* bns, const void* pac_device,
                           bwagpu_ctx_t** out) {
  if (!pac_device) return BWAGPU_E_INVAL;
  bwagpu_ctx_t* ctx = nullptr;
  int rc = create_common(device, opt, bns, out, &ctx);
  if (rc != BWAGPU_OK) {
    destroy_ctx(ctx);
    return rc;
  }
  ctx->d_pac = (void*)pac_device;
  ctx->own_pac = false;
  ctx->ref.pac = (const uint8_t*)pac_device;
  *out = ctx;
  return BWAGPU_OK;
}

int bwagpu_destroy(bwagpu_ctx_t* ctx) {
  if (!ctx) return BWAGPU_E_INVAL;
  destroy_ctx(ctx);
  return BWAGPU_OK;
}

const char* bwagpu_last_error(const bwagpu_ctx_t* ctx) { return ctx ? ctx->err.c_str() : "NULL context"; }

int bwagpu_set_watchdog_ms(bwagpu_ctx_t* ctx, int ms) {
  if (!ctx || ms < 0) return BWAGPU_E_INVAL;
  ctx->watchdog_ms = ms;
  return BWAGPU_OK;
}

namespace {
// the ABI's slot layout (read r's regions from chain_seed_off[read_chain_off[r]])
// from a finished batch's dense results; the offsets come from the staged input
void expand_slots(const Slot& s, bwagpu_alnreg_t* dst) {
  const char* h = s.h_in.as<const char>();
  const int32_t* rco = s.kept ? s.keep_rco.data() : (const int32_t*)(h + s.in_rco);
  const int32_t* cso = s.kept ? s.keep_cso.data() : (const int32_t*)(h + s.in_cso);
  const int32_t* n = s.h_n.as<const int32_t>();
  const int32_t* off = s.h_off.as<const int32_t>();
  const bwagpu_alnreg_t* src = s.h_dense.as<const bwagpu_alnreg_t>();
  for (int32_t r = 0; r < s.n_reads; ++r)
    if (n[r]) memcpy(dst + cso[rco[r]], src + off[r], sizeof(bwagpu_alnreg_t) * (size_t)n[r]);
}
}  // namespace

int bwagpu_chain2aln_submit(bwagpu_ctx_t* ctx, int slot, const bwagpu_batch_t* b) {
  if (!ctx || slot < 0 || slot >= BWAGPU_NUM_SLOTS) return BWAGPU_E_INVAL;
  Slot& s = ctx->slot[slot];
  if (s.busy) return fail(ctx, BWAGPU_E_INVAL, "slot already has a batch in flight");
  // the previous batch's results end here, whether or not this submit succeeds
  s.has_results = false;
  s.kept = false;
  s.slot_view = false;
  int lq_max = 0;
  int rc = check_batch_header(ctx, b);
  if (rc) return rc;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  s.t_submit = std::chrono::steady_clock::now();
  InLayout L;
  L.make(*b);
  HIPC(s.h_in.ensure(L.total), "hipHostMalloc(in)");
  HIPC(s.d_in.ensure(L.total), "hipMalloc(in)");
  HIPC(s.d_out.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max(b->n_seeds, 1)), "hipMalloc(out)");
  HIPC(s.d_n.ensure(sizeof(int32_t) * (size_t)std::max(b->n_reads, 1)), "hipMalloc(out_n)");
  HIPC(s.d_stats.ensure(sizeof(int64_t) * ST_N), "hipMalloc(stats)");
  HIPC(s.h_dense.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max(b->n_seeds, 1)), "hipHostMalloc(out)");
  HIPC(s.h_n.ensure(sizeof(int32_t) * (size_t)std::max(b->n_reads, 1)), "hipHostMalloc(out_n)");
  HIPC(s.h_off.ensure(sizeof(int32_t) * (size_t)(b->n_reads + 1)), "hipHostMalloc(out_off)");
  HIPC(s.d_off.ensure(sizeof(int32_t) * (size_t)(b->n_reads + 1)), "hipMalloc(out_off)");
  HIPC(s.h_stats.ensure(sizeof(int64_t) * ST_N), "hipHostMalloc(stats)");
  s.slot_view = false;
  // stage into pinned memory so the caller's buffers are free on return —
  // unless the caller packed into that memory already (bwagpu_chain2aln_stage)
  char* h = s.h_in.as<char>();
  const bool staged = b->n_reads > 0 && (const void*)b->seq_off == (const void*)(h + L.seq_off) &&
                      (const void*)b->seeds == (const void*)(h + L.seeds) &&
                      (const void*)b->seq == (const void*)(h + L.seq) &&
                      (const void*)b->chain_seed_off == (const void*)(h + L.cso);
  // the staging copy (~20 MB for a C2 record) and the check of every read,
  // chain and seed in one pass on a few threads (stage_and_check): nothing is
  // enqueued before both are done, so a refused batch leaves no DMA reading
  // the staging buffer
  if (!staged && b->n_reads) {
    rc = stage_and_check(ctx, b, h, L, &lq_max);
  } else {
    if (!staged) memcpy(h + L.cso, b->chain_seed_off, sizeof(int32_t) * (size_t)(b->n_chains + 1));
    rc = check_batch_seeds(ctx, b, &lq_max);
  }
  if (rc) return rc;
  if ((rc = check_lds(ctx, lq_max))) return rc;

  hipStream_t st = nullptr;
  HIPC(lazy_stream(s, &st), "hipStreamCreate");
  HIPC(hipEventRecord(s.ev0, st), "event");
  HIPC(hipMemcpyAsync(s.d_in.p, s.h_in.p, L.total, hipMemcpyHostToDevice, st), "H2D batch");
  HIPC(hipMemsetAsync(s.d_stats.p, 0, sizeof(int64_t) * ST_N, st), "memset stats");
  char* d = s.d_in.as<char>();
  DevBatch db;
  db.n_reads = b->n_reads;
  db.n_chains = b->n_chains;
  db.n_seeds = b->n_seeds;
  db.seq_off = (const int64_t*)(d + L.seq_off);
  db.seq = (const uint8_t*)(d + L.seq);
  db.read_chain_off = (const int32_t*)(d + L.rco);
  db.chain_seed_off = (const int32_t*)(d + L.cso);
  db.chain_rid = (const int32_t*)(d + L.rid);
  db.chain_frac_rep = (const float*)(d + L.frac);
  db.seeds = (const bwagpu_seed_t*)(d + L.seeds);
  HIPC(hipEventRecord(s.ev1, st), "event");
  rc = enqueue_chain2aln(ctx, s, db, lq_max, s.d_out.as<bwagpu_alnreg_t>(), s.d_n.as<int32_t>(),
                         s.d_stats.as<int64_t>(), st);
  if (rc) {
    // work already queued on the slot's stream may still read h_in / d_in:
    // drain it before the caller may reuse the slot
    (void)hipStreamSynchronize(st);
    return rc;
  }
  HIPC(hipEventRecord(s.ev2, st), "event");
  // the results: per-read offsets, then the regions densely into pinned memory
  // (the device writes them over PCIe: only the sum of n is moved, not the
  // n_seeds slots the kernels fill)
  int32_t* h_off_dev = nullptr;
  bwagpu_alnreg_t* h_dense_dev = nullptr;
  HIPC(hipHostGetDevicePointer((void**)&h_off_dev, s.h_off.p, 0), "hipHostGetDevicePointer");
  HIPC(hipHostGetDevicePointer((void**)&h_dense_dev, s.h_dense.p, 0), "hipHostGetDevicePointer");
  hipLaunchKernelGGL(dense_scan_kernel, dim3(1), dim3(kDenseScanBlock), 0, st, s.d_n.as<int32_t>(), b->n_reads,
                     s.d_off.as<int32_t>(), h_off_dev);
  if (b->n_reads)
    hipLaunchKernelGGL(dense_copy_kernel, dim3((unsigned)((b->n_reads + 15) / 16)), dim3(256), 0, st,
                       s.d_out.as<bwagpu_alnreg_t>(), s.d_n.as<int32_t>(), s.d_off.as<int32_t>(), db.read_chain_off,
                       db.chain_seed_off, b->n_reads, h_dense_dev);
  HIPC(hipGetLastError(), "dense results launch");
  if (b->n_reads)
    HIPC(hipMemcpyAsync(s.h_n.p, s.d_n.p, sizeof(int32_t) * (size_t)b->n_reads, hipMemcpyDeviceToHost, st),
         "D2H counts");
  HIPC(hipMemcpyAsync(s.h_stats.p, s.d_stats.p, sizeof(int64_t) * ST_N, hipMemcpyDeviceToHost, st), "D2H stats");
  HIPC(hipEventRecord(s.ev3, st), "event");
  s.h2d = (int64_t)L.total;
  s.in_rco = L.rco;
  s.in_cso = L.cso;
  // the batch's sizes only once it is in flight: _wait and _results read them
  s.n_reads = b->n_reads;
  s.n_chains = b->n_chains;
  s.n_seeds = b->n_seeds;
  s.busy = true;
  return BWAGPU_OK;
}

int bwagpu_chain2aln_wait(bwagpu_ctx_t* ctx, int slot, bwagpu_alnreg_t* out_regs, int32_t* out_n) {
  if (!ctx || slot < 0 || slot >= BWAGPU_NUM_SLOTS) return BWAGPU_E_INVAL;
  Slot& s = ctx->slot[slot];
  if (!s.busy) return fail(ctx, BWAGPU_E_INVAL, "slot has no batch in flight");
  if (ctx->fail_after == 0) {  // injected failure: the batch stays in flight, as after a real watchdog expiry
    ctx->fail_after = -1;
    return fail(ctx, ctx->fail_code, "injected failure (bwagpu_debug_fail_wait)");
  }
  if (ctx->fail_after > 0) --ctx->fail_after;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  // watchdog (SWTask::finish, SWTask.cpp:162-169): poll the completion event,
  // backing off from 20 to 320 us (every query takes the runtime's lock, which
  // other host threads driving the device contend for)
  const auto t0 = std::chrono::steady_clock::now();
  int nap_us = 20;
  for (;;) {
    hipError_t q = hipEventQuery(s.ev3);
    if (q == hipSuccess) break;
    if (q != hipErrorNotReady) {
      s.busy = false;
      return hip_fail(ctx, q, "batch execution");
    }
    if (ctx->watchdog_ms > 0 &&
        std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count() >
            ctx->watchdog_ms) {
      return fail(ctx, BWAGPU_E_HANG, "watchdog: batch did not finish in time");
    }
    std::this_thread::sleep_for(std::chrono::microseconds(nap_us));
    nap_us = std::min(nap_us * 2, 320);
  }
  s.busy = false;
  s.has_results = true;
  const int64_t* st = s.h_stats.as<int64_t>();
  float k_ms = 0, t_ms = 0;
  (void)hipEventElapsedTime(&k_ms, s.ev1, s.ev2);
  (void)hipEventElapsedTime(&t_ms, s.ev0, s.ev3);
  s.last.kernel_ms = k_ms;
  s.last.total_ms = t_ms;
  s.last.cells = st[ST_CELLS];
  s.last.rows = st[ST_ROWS];
  s.last.ext_calls = st[ST_CALLS];
  const int32_t* off = s.h_off.as<int32_t>();
  s.d2h = (int64_t)sizeof(bwagpu_alnreg_t) * off[s.n_reads] + (int64_t)sizeof(int32_t) * (2 * (int64_t)s.n_reads + 1);
  s.last.h2d_bytes = s.h2d;
  s.last.d2h_bytes = s.d2h;
  if (st[ST_ERR] & ERR_LEN) return fail(ctx, BWAGPU_E_UNSUPPORTED, "read longer than BWAGPU_MAX_READ_LEN");
  // on a flagged chain the results are still copied: every other chain's
  // regions are valid, the flagged ones were skipped (the caller's error path)
  if (out_n && s.n_reads) memcpy(out_n, s.h_n.p, sizeof(int32_t) * (size_t)s.n_reads);
  if (out_regs && s.n_seeds) expand_slots(s, out_regs);
  if (st[ST_ERR] & ERR_RID)
    return fail(ctx, BWAGPU_E_RESULTS, "a chain's first seed is not inside contig chain_rid (bwamem.c:669 assert)");
  return BWAGPU_OK;
}

int bwagpu_chain2aln_stage(bwagpu_ctx_t* ctx, int slot, int32_t n_reads, int32_t n_chains, int32_t n_seeds,
                           int64_t seq_bytes, bwagpu_batch_t* view) {
  if (!ctx || slot < 0 || slot >= BWAGPU_NUM_SLOTS || !view || n_reads < 0 || n_chains < 0 || n_seeds < 0 ||
      seq_bytes < 0)
    return BWAGPU_E_INVAL;
  Slot& s = ctx->slot[slot];
  if (s.busy) return fail(ctx, BWAGPU_E_INVAL, "slot already has a batch in flight");
  bwagpu_batch_t b{};
  b.n_reads = n_reads;
  b.n_chains = n_chains;
  b.n_seeds = n_seeds;
  b.seq_bytes = seq_bytes;
  InLayout L;
  L.make(b);
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  // the caller packs the next batch over h_in: the finished batch's offsets
  // move out first, so that its _results (valid until the next _submit) can
  // still build the slot layout
  if (s.has_results && !s.slot_view && !s.kept && s.n_reads) {
    const char* hp = s.h_in.as<const char>();
    const int32_t* rco = (const int32_t*)(hp + s.in_rco);
    s.keep_rco.assign(rco, rco + s.n_reads + 1);
    const int32_t* cso = (const int32_t*)(hp + s.in_cso);
    s.keep_cso.assign(cso, cso + s.n_chains + 1);
    s.kept = true;
  }
  HIPC(s.h_in.ensure(L.total), "hipHostMalloc(in)");
  char* h = s.h_in.as<char>();
  b.seq_off = (const int64_t*)(h + L.seq_off);
  b.seq = (const uint8_t*)(h + L.seq);
  b.read_chain_off = (const int32_t*)(h + L.rco);
  b.chain_seed_off = (const int32_t*)(h + L.cso);
  b.chain_rid = (const int32_t*)(h + L.rid);
  b.chain_frac_rep = (const float*)(h + L.frac);
  b.seeds = (const bwagpu_seed_t*)(h + L.seeds);
  *view = b;
  return BWAGPU_OK;
}

int bwagpu_chain2aln_results(bwagpu_ctx_t* ctx, int slot, const bwagpu_alnreg_t** regs, const int32_t** n) {
  if (!ctx || slot < 0 || slot >= BWAGPU_NUM_SLOTS || !regs || !n) return BWAGPU_E_INVAL;
  Slot& s = ctx->slot[slot];
  if (s.busy) return fail(ctx, BWAGPU_E_INVAL, "slot's batch still in flight (wait first)");
  if (!s.has_results) return fail(ctx, BWAGPU_E_INVAL, "slot has no results");
  if (!s.slot_view) {  // the slot layout, built from the dense results once per batch
    HIPC(s.h_out.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max(s.n_seeds, 1)), "hipHostMalloc(out)");
    if (s.n_seeds) expand_slots(s, s.h_out.as<bwagpu_alnreg_t>());
    s.slot_view = true;
  }
  *regs = s.h_out.as<const bwagpu_alnreg_t>();
  *n = s.h_n.as<const int32_t>();
  return BWAGPU_OK;
}

int bwagpu_chain2aln_results_dense(bwagpu_ctx_t* ctx, int slot, const bwagpu_alnreg_t** regs, const int32_t** n,
                                   const int32_t** off) {
  if (!ctx || slot < 0 || slot >= BWAGPU_NUM_SLOTS || !regs || !n || !off) return BWAGPU_E_INVAL;
  Slot& s = ctx->slot[slot];
  if (s.busy) return fail(ctx, BWAGPU_E_INVAL, "slot's batch still in flight (wait first)");
  if (!s.has_results || !s.h_dense.p || !s.h_off.p) return fail(ctx, BWAGPU_E_INVAL, "slot has no results");
  *regs = s.h_dense.as<const bwagpu_alnreg_t>();
  *n = s.h_n.as<const int32_t>();
  *off = s.h_off.as<const int32_t>();
  return BWAGPU_OK;
}

int bwagpu_chain2aln(bwagpu_ctx_t* ctx, const bwagpu_batch_t* b, bwagpu_alnreg_t* out_regs, int32_t* out_n) {
  int rc = bwagpu_chain2aln_submit(ctx, 0, b);
  if (rc) return rc;
  return bwagpu_chain2aln_wait(ctx, 0, out_regs, out_n);
}

int bwagpu_chain2aln_device(bwagpu_ctx_t* ctx, const bwagpu_batch_t* db_in, bwagpu_alnreg_t* dev_out,
                            int32_t* dev_n, int64_t* dev_stats, void* stream) {
  if (!ctx || !db_in || !dev_out || !dev_n) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  // reads are bounded by bwagpu_set_device_read_len (default BWAGPU_MAX_READ_LEN)
  // on the speculative path, by BWAGPU_MAX_READ_LEN on the per-read one; the
  // LDS row buffers are sized for the bound
  const int lq_bound = use_read_kernels() ? BWAGPU_MAX_READ_LEN : ctx->dev_read_len;
  int rc = check_lds(ctx, lq_bound);
  if (rc) return rc;
  hipStream_t st = (hipStream_t)stream;
  if (!st) HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int k = 0;
  while (k < BWAGPU_NUM_SLOTS && ctx->dev_stream[k] && ctx->dev_stream[k] != st) ++k;
  if (k == BWAGPU_NUM_SLOTS) return fail(ctx, BWAGPU_E_INVAL, "more than BWAGPU_NUM_SLOTS streams on one context");
  ctx->dev_stream[k] = st;
  Slot& s = ctx->dev_scratch[k];
  DevBatch db;
  db.n_reads = db_in->n_reads;
  db.n_chains = db_in->n_chains;
  db.n_seeds = db_in->n_seeds;
  db.seq_off = db_in->seq_off;
  db.seq = db_in->seq;
  db.read_chain_off = db_in->read_chain_off;
  db.chain_seed_off = db_in->chain_seed_off;
  db.chain_rid = db_in->chain_rid;
  db.chain_frac_rep = db_in->chain_frac_rep;
  db.seeds = db_in->seeds;
  int64_t* stats = dev_stats;
  if (!stats) {
    HIPC(s.d_stats.ensure(sizeof(int64_t) * ST_N), "hipMalloc(stats)");
    stats = s.d_stats.as<int64_t>();
    HIPC(hipMemsetAsync(stats, 0, sizeof(int64_t) * ST_N, st), "memset stats");
  }
  return enqueue_chain2aln(ctx, s, db, lq_bound, dev_out, dev_n, stats, st);
}

int bwagpu_extend_batch(bwagpu_ctx_t* ctx, int32_t n, const bwagpu_ext_task_t* tasks, const uint8_t* qpool,
                        int64_t qpool_len, const uint8_t* tpool, int64_t tpool_len, bwagpu_ext_result_t* results) {
  if (!ctx || n < 0 || (n && (!tasks || !results))) return BWAGPU_E_INVAL;
  if (n == 0) return BWAGPU_OK;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  // validate and bin on the host
  // bins: the wave kernels by column segments, then the four-per-wave kernel
  // (packed 16-bit DP) for the tasks it takes (extend4_kernel)
  std::vector<int32_t> lists[kNumExtVariants + 1];
  const bool quad = ctx->ext_form == 0;
  bool t5 = false;
  int lq_max = 1;
  for (int32_t k = 0; k < n; ++k) {
    const bwagpu_ext_task_t& t = tasks[k];
    if (t.qlen < 0 || t.tlen < 0 || t.qoff < 0 || t.toff < 0 || t.qoff + t.qlen > qpool_len ||
        t.toff + t.tlen > tpool_len || t.w < 0)
      return fail(ctx, BWAGPU_E_INVAL, "task outside its pools");
    if (t.qlen + 1 > kExtVariants[kNumExtVariants - 1].max_len()) return fail(ctx, BWAGPU_E_UNSUPPORTED, "qlen too long");
    int v = kNumExtVariants - 1;
    for (int i = kNumExtVariants - 1; i >= 0; --i)
      if (t.qlen + 1 <= kExtVariants[i].max_len()) v = i;
    if (quad && t.h0 > 0 && t.qlen >= 1 && t.qlen + 1 <= 256 &&
        quad_bound_ok(ctx->opt, t.h0 + (long)t.qlen * ctx->opt.max_mat) && quad_rows_ok(ctx->opt, t.tlen)) {
      bool nt = true;  // no N in the target rows
      for (int64_t i = t.toff; i < t.toff + t.tlen && nt; ++i) nt = tpool[i] <= 3;
      if (nt) v = kNumExtVariants;
    }
    lists[v].push_back(k);
    lq_max = std::max(lq_max, t.qlen + 1);
  }
  for (int64_t i = 0; i < tpool_len && !t5; ++i) t5 = tpool[i] > 3;
  for (int64_t i = 0; i < qpool_len; ++i)
    if (qpool[i] > 4) return fail(ctx, BWAGPU_E_INVAL, "query base > 4");
  for (int64_t i = 0; i < tpool_len; ++i)
    if (tpool[i] > 4) return fail(ctx, BWAGPU_E_INVAL, "target base > 4");
  // LDS rows needed per task (rows_needed on the host) -> per-variant max
  Slot& s = ctx->slot[0];
  hipStream_t st = nullptr;
  HIPC(lazy_stream(s, &st), "hipStreamCreate");
  DevBuf d_tasks, d_list, d_q, d_t, d_res, d_stats;
  auto cleanup = [&]() {
    d_tasks.release(); d_list.release(); d_q.release(); d_t.release(); d_res.release(); d_stats.release();
  };
  auto ck = [&](hipError_t e, const char* what) {
    if (e != hipSuccess) {
      cleanup();
      return hip_fail(ctx, e, what);
    }
    return 0;
  };
  int rc;
  if ((rc = ck(d_tasks.ensure(sizeof(bwagpu_ext_task_t) * n), "hipMalloc"))) return rc;
  if ((rc = ck(d_list.ensure(sizeof(int32_t) * n), "hipMalloc"))) return rc;
  if ((rc = ck(d_q.ensure((size_t)qpool_len + 1), "hipMalloc"))) return rc;
  if ((rc = ck(d_t.ensure((size_t)tpool_len + 1), "hipMalloc"))) return rc;
  if ((rc = ck(d_res.ensure(sizeof(bwagpu_ext_result_t) * n), "hipMalloc"))) return rc;
  if ((rc = ck(d_stats.ensure(sizeof(int64_t) * ST_N), "hipMalloc"))) return rc;
  if ((rc = ck(hipMemcpyAsync(d_tasks.p, tasks, sizeof(bwagpu_ext_task_t) * n, hipMemcpyHostToDevice, st), "H2D"))) return rc;
  if (qpool_len && (rc = ck(hipMemcpyAsync(d_q.p, qpool, (size_t)qpool_len, hipMemcpyHostToDevice, st), "H2D"))) return rc;
  if (tpool_len && (rc = ck(hipMemcpyAsync(d_t.p, tpool, (size_t)tpool_len, hipMemcpyHostToDevice, st), "H2D"))) return rc;
  if ((rc = ck(hipMemsetAsync(d_stats.p, 0, sizeof(int64_t) * ST_N, st), "memset"))) return rc;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, st);
  int32_t off = 0;
  std::vector<int32_t> all;
  for (int v = 0; v <= kNumExtVariants; ++v) all.insert(all.end(), lists[v].begin(), lists[v].end());
  if ((rc = ck(hipMemcpyAsync(d_list.p, all.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st), "H2D"))) return rc;
  for (int v = 0; v <= kNumExtVariants; ++v) {
    const int32_t nv = (int32_t)lists[v].size();
    if (nv) {
      int rows = 16;
      for (int32_t k : lists[v]) {
        const bwagpu_ext_task_t& t = tasks[k];
        int mi = band_cap(t.qlen, ctx->opt.max_mat, t.end_bonus, ctx->opt.o_ins, ctx->opt.e_ins);
        int md = band_cap(t.qlen, ctx->opt.max_mat, t.end_bonus, ctx->opt.o_del, ctx->opt.e_del);
        int we = std::min(t.w, std::min(mi, md));
        rows = std::max(rows, std::min(t.tlen, t.qlen + we + 1));
      }
      const int tb = (rows + 2 + 15) & ~15;
      const int gpb = v < kNumExtVariants ? kBlock / kExtVariants[v].G : 2 * kBlock / 32;
      if ((size_t)tb * gpb > 64 * 1024) {
        cleanup();
        return fail(ctx, BWAGPU_E_UNSUPPORTED, "task needs too many LDS rows");
      }
      hipError_t e =
          v < kNumExtVariants
              ? launch_extend(v, t5, ctx->opt, n, d_tasks.as<bwagpu_ext_task_t>(), d_list.as<int32_t>() + off, nv,
                              d_q.as<uint8_t>(), d_t.as<uint8_t>(), tb, d_res.as<bwagpu_ext_result_t>(),
                              d_stats.as<int64_t>(), st)
              : launch_extend4(ctx->opt, d_tasks.as<bwagpu_ext_task_t>(), d_list.as<int32_t>() + off, nv,
                               d_q.as<uint8_t>(), d_t.as<uint8_t>(), tb, d_res.as<bwagpu_ext_result_t>(),
                               d_stats.as<int64_t>(), st);
      if ((rc = ck(e, "extend launch"))) return rc;
    }
    off += nv;
  }
  (void)hipEventRecord(e1, st);
  int64_t hs[ST_N];
  if ((rc = ck(hipMemcpyAsync(results, d_res.p, sizeof(bwagpu_ext_result_t) * n, hipMemcpyDeviceToHost, st), "D2H"))) return rc;
  if ((rc = ck(hipMemcpyAsync(hs, d_stats.p, sizeof(hs), hipMemcpyDeviceToHost, st), "D2H"))) return rc;
  if ((rc = ck(hipStreamSynchronize(st), "extend batch"))) return rc;
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  s.last = bwagpu_stats_t{};
  s.last.kernel_ms = ms;
  s.last.cells = hs[ST_CELLS];
  s.last.rows = hs[ST_ROWS];
  s.last.ext_calls = hs[ST_CALLS];
  cleanup();
  return BWAGPU_OK;
}

}  // extern "C"

namespace {
int launch_align2_concurrent(bwagpu_ctx_t* ctx, hipStream_t st, const std::vector<int>& bins, const A2Args& base,
                             const int32_t* list_off, const int32_t* counts_host, int32_t* d_counts,
                             int32_t* d_cursors, size_t list_stride) {
  constexpr int NS = bwagpu_ctx::kA2Streams;
  for (int i = 0; i < NS; ++i) {
    if (!ctx->a2_st[i]) HIPC(hipStreamCreateWithFlags(&ctx->a2_st[i], hipStreamNonBlocking), "stream");
    if (!ctx->a2_join[i]) HIPC(hipEventCreateWithFlags(&ctx->a2_join[i], hipEventDisableTiming), "event");
  }
  if (!ctx->a2_fork) HIPC(hipEventCreateWithFlags(&ctx->a2_fork, hipEventDisableTiming), "event");
  const int used = std::min<int>(NS, (int)bins.size());
  HIPC(hipEventRecord(ctx->a2_fork, st), "event");
  for (int i = 0; i < used; ++i) HIPC(hipStreamWaitEvent(ctx->a2_st[i], ctx->a2_fork, 0), "stream wait");
  for (size_t k = 0; k < bins.size(); ++k) {
    const int b = bins[k];
    A2Args a = base;
    a.list = base.list + (list_off ? list_off[b] : (size_t)b * list_stride);
    a.count = d_counts + b;
    a.cursor = d_cursors + b;
    HIPC(launch_align2(b, a, make_a2prof(ctx->opt, b >= kA2Buckets), counts_host ? counts_host[b] : 0,
                       ctx->a2_st[k % used]),
         "align2 launch");
  }
  for (int i = 0; i < used; ++i) {
    HIPC(hipEventRecord(ctx->a2_join[i], ctx->a2_st[i]), "event");
    HIPC(hipStreamWaitEvent(st, ctx->a2_join[i], 0), "stream wait");
  }
  return BWAGPU_OK;
}
}  // namespace

extern "C" {

// mem_reg2aln's CIGAR part (bwa/bwamem.c:1104-1174) per job.  Jobs are binned on
// the host by query segments (kernel template) and by the size of their
// direction matrix (ksw_global2's z, ncol x tlen bytes, ksw.c:511-512): the
// matrix sits in LDS for jobs up to kR2ZSmall / kR2ZLarge bytes and in a
// per-wave HBM slice beyond.
namespace {
constexpr int kR2ZSmall = 8 * 1024, kR2ZLarge = 24 * 1024;
constexpr int kR2MaxRef = 8192;  // reference window bytes per job (LDS)
}  // namespace

int bwagpu_reg2aln_batch(bwagpu_ctx_t* ctx, int32_t n, const bwagpu_reg2aln_task_t* tasks, const uint8_t* qpool,
                         int64_t qpool_len, int32_t max_ops, int32_t max_md, bwagpu_aln_t* out, uint32_t* cigar,
                         char* md) {
  if (!ctx || n < 0 || (n && (!tasks || !out || !cigar || !md)) || qpool_len < 0 || (qpool_len && !qpool) ||
      max_ops < 1 || max_md < 1)
    return BWAGPU_E_INVAL;
  if (n == 0) return BWAGPU_OK;
  const DevOpt& o = ctx->opt;
  const int64_t l_pac = ctx->ref.l_pac, two = l_pac << 1;
  const int wmax = o.w << 2;
  // validate; bin by [query bucket][matrix class 0 LDS small, 1 LDS large, 2 HBM]
  struct Bin {
    std::vector<int32_t> ids;
    int qmax = 0, rmax = 0;
    int64_t zmax = 0;
  };
  Bin bins[kR2Buckets][3];
  std::vector<int64_t> cost((size_t)n, 0);
  for (int32_t k = 0; k < n; ++k) {
    const bwagpu_reg2aln_task_t& t = tasks[k];
    if (t.l_seq < 0 || t.qoff < 0 || t.qoff + t.l_seq > qpool_len)
      return fail(ctx, BWAGPU_E_INVAL, "job's read outside the query pool");
    int lq = 0, rl = 0, cls = 0;
    int64_t zb = 0;
    if (t.rb >= 0 && t.re >= 0) {
      const int64_t beg = t.rb, end = t.re > two ? two : t.re;
      const bool ok = t.qe - t.qb > 0 && t.rb < t.re && !(t.rb < l_pac && t.re > l_pac) &&
                      (beg >= l_pac || end <= l_pac) && end - beg == t.re - t.rb;
      if (ok) {
        if (t.qb < 0 || t.qe > t.l_seq) return fail(ctx, BWAGPU_E_INVAL, "job's qb/qe outside its read");
        lq = t.qe - t.qb;
        if (lq > BWAGPU_MAX_READ_LEN) return fail(ctx, BWAGPU_E_UNSUPPORTED, "qe - qb > BWAGPU_MAX_READ_LEN");
        if (t.re - t.rb > kR2MaxRef) return fail(ctx, BWAGPU_E_UNSUPPORTED, "re - rb > 8192");
        rl = (int)(t.re - t.rb);
        // the widest band any try can use: the first try's w2 (infer_bw,
        // bwamem.c:1123-1126) doubled at most twice (1132), capped at
        // opt->w << 2, then bwa.c:152-159
        auto infer = [&](int q_, int r_) {
          if (lq == rl && lq * o.a - t.truesc < (q_ + r_ - o.a) << 1) return 0;
          const int w = (int)((double)(std::min(lq, rl) * o.a - t.truesc - q_) / r_ + 2.);
          return std::max(w, std::abs(lq - rl));
        };
        int w2 = std::max(infer(o.o_del, o.e_del), infer(o.o_ins, o.e_ins));
        if (w2 > o.w) w2 = std::min(w2, t.w);
        w2 = std::min(w2, wmax);
        const int w2max = (int)std::min<int64_t>((int64_t)w2 << 2, wmax);
        const int half = (lq + 1) >> 1;
        const int mi = (int)((double)(half * o.mat[0] - o.o_ins) / o.e_ins + 1.);
        const int mdl = (int)((double)(half * o.mat[0] - o.o_del) / o.e_del + 1.);
        const int mg = std::max(std::max(mi, mdl), 1), dl = std::abs(rl - lq);
        const int wb = std::max(std::min((mg + dl + 1) >> 1, w2max), dl + 3);
        zb = (int64_t)std::min(lq, 2 * wb + 1) * rl;
        cls = zb <= kR2ZSmall ? 0 : (zb <= kR2ZLarge ? 1 : 2);
      }
    }
    Bin& b = bins[r2_bucket_of(lq)][cls];
    b.ids.push_back(k);
    b.qmax = std::max(b.qmax, lq);
    b.rmax = std::max(b.rmax, rl);
    b.zmax = std::max(b.zmax, zb);
    cost[(size_t)k] = zb + lq + rl;
  }
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  HIPC(ctx->r2_tasks.ensure(sizeof(bwagpu_reg2aln_task_t) * n), "hipMalloc");
  HIPC(ctx->r2_q.ensure((size_t)qpool_len + 1), "hipMalloc");
  HIPC(ctx->r2_out.ensure(sizeof(bwagpu_aln_t) * n), "hipMalloc");
  HIPC(ctx->r2_cig.ensure(sizeof(uint32_t) * (size_t)n * max_ops), "hipMalloc");
  HIPC(ctx->r2_md.ensure((size_t)n * max_md), "hipMalloc");
  HIPC(ctx->r2_lists.ensure(sizeof(int32_t) * n), "hipMalloc");
  HIPC(ctx->r2_stats.ensure(sizeof(int64_t) * ST_N), "hipMalloc");
  std::vector<int32_t> all;
  all.reserve((size_t)n);
  for (auto& row : bins)
    for (auto& b : row) {
      // largest matrices first: the last claims are the small jobs
      std::stable_sort(b.ids.begin(), b.ids.end(), [&](int32_t x, int32_t y) { return cost[x] > cost[y]; });
      all.insert(all.end(), b.ids.begin(), b.ids.end());
    }
  HIPC(hipMemcpyAsync(ctx->r2_tasks.p, tasks, sizeof(bwagpu_reg2aln_task_t) * n, hipMemcpyHostToDevice, st), "H2D");
  if (qpool_len) HIPC(hipMemcpyAsync(ctx->r2_q.p, qpool, (size_t)qpool_len, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemcpyAsync(ctx->r2_lists.p, all.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemsetAsync(ctx->r2_stats.p, 0, sizeof(int64_t) * ST_N, st), "memset");
  // bins run concurrently on the context's side streams, largest first
  constexpr int NS = bwagpu_ctx::kA2Streams;
  for (int i = 0; i < NS; ++i) {
    if (!ctx->a2_st[i]) HIPC(hipStreamCreateWithFlags(&ctx->a2_st[i], hipStreamNonBlocking), "stream");
    if (!ctx->a2_join[i]) HIPC(hipEventCreateWithFlags(&ctx->a2_join[i], hipEventDisableTiming), "event");
  }
  if (!ctx->a2_fork) HIPC(hipEventCreateWithFlags(&ctx->a2_fork, hipEventDisableTiming), "event");
  struct Launch {
    int bk, cls;
    int32_t off;
    int64_t work;
  };
  std::vector<Launch> launches;
  {
    int32_t off = 0;
    for (int bk = 0; bk < kR2Buckets; ++bk)
      for (int cls = 0; cls < 3; ++cls) {
        const Bin& b = bins[bk][cls];
        if (b.ids.empty()) continue;
        int64_t w = 0;
        for (int32_t k : b.ids) w += cost[(size_t)k];
        launches.push_back({bk, cls, off, w});
        off += (int32_t)b.ids.size();
      }
  }
  std::sort(launches.begin(), launches.end(), [](const Launch& x, const Launch& y) { return x.work > y.work; });
  const int used = std::min<int>(NS, (int)launches.size());
  hipEvent_t e0 = nullptr, e1 = nullptr;
  HIPC(hipEventCreate(&e0), "event");
  HIPC(hipEventCreate(&e1), "event");
  HIPC(hipEventRecord(e0, st), "event");
  HIPC(hipEventRecord(ctx->a2_fork, st), "event");
  for (int i = 0; i < used; ++i) HIPC(hipStreamWaitEvent(ctx->a2_st[i], ctx->a2_fork, 0), "stream wait");
  auto make_args = [&](const Launch& L, int& wpb) {
    const Bin& b = bins[L.bk][L.cls];
    R2AArgs a{};
    a.tasks = ctx->r2_tasks.as<bwagpu_reg2aln_task_t>();
    a.qpool = ctx->r2_q.as<uint8_t>();
    a.list = ctx->r2_lists.as<int32_t>() + L.off;
    a.n = (int)b.ids.size();
    a.max_ops = max_ops;
    a.max_md = max_md;
    a.out = ctx->r2_out.as<bwagpu_aln_t>();
    a.cigar = ctx->r2_cig.as<uint32_t>();
    a.md = ctx->r2_md.as<char>();
    a.stats = ctx->r2_stats.as<int64_t>();
    a.qcap = (b.qmax + 16) & ~15;
    a.rcap = (b.rmax + 16) & ~15;
    a.ocap = a.qcap + a.rcap + 4;
    int lpw = a.qcap + a.rcap + 4 * a.ocap;
    if (L.cls < 2) lpw += L.cls == 0 ? kR2ZSmall : kR2ZLarge;
    a.lds_per_wave = (lpw + 15) & ~15;
    wpb = L.cls == 1 ? 1 : 4;  // LDS-heavy bins: one wave per workgroup packs LDS finer
    a.zstride = L.cls == 2 ? ((b.zmax + 255) & ~(int64_t)255) : 0;
    return a;
  };
  // grids first (HBM matrix slices: one per launched wave, at most 1 GiB per bin)
  size_t zoff = 0;
  for (Launch& L : launches) {
    int wpb = 4;
    const R2AArgs a = make_args(L, wpb);
    if ((size_t)wpb * a.lds_per_wave > 160 * 1024) {
      (void)hipEventDestroy(e0);
      (void)hipEventDestroy(e1);
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "reg2aln job needs more LDS than a workgroup has");
    }
    int waves = r2_resident_waves(kR2CD[L.bk], (size_t)wpb * a.lds_per_wave, wpb);
    if (L.cls == 2) {
      waves = (int)std::min<int64_t>(waves, std::max<int64_t>(4, ((int64_t)1 << 30) / a.zstride));
      zoff += (size_t)a.zstride * waves;
    }
    L.work = waves;
  }
  HIPC(ctx->r2_z.ensure(std::max<size_t>(zoff, 256)), "hipMalloc(reg2aln matrices)");
  zoff = 0;
  for (size_t li = 0; li < launches.size(); ++li) {
    const Launch& L = launches[li];
    int wpb = 4;
    R2AArgs a = make_args(L, wpb);
    const int nb = a.n, waves = (int)L.work;
    if (L.cls == 2) {
      a.zglob = ctx->r2_z.as<uint8_t>() + zoff;
      zoff += (size_t)a.zstride * waves;
    }
    const int blocks = std::max(1, std::min((nb + wpb - 1) / wpb, waves / wpb));
    HIPC(launch_reg2aln(kR2CD[L.bk], o, ctx->ref, a, blocks, wpb, ctx->a2_st[li % used]), "reg2aln launch");
  }
  for (int i = 0; i < used; ++i) {
    HIPC(hipEventRecord(ctx->a2_join[i], ctx->a2_st[i]), "event");
    HIPC(hipStreamWaitEvent(st, ctx->a2_join[i], 0), "stream wait");
  }
  HIPC(hipEventRecord(e1, st), "event");
  HIPC(hipMemcpyAsync(out, ctx->r2_out.p, sizeof(bwagpu_aln_t) * n, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipMemcpyAsync(cigar, ctx->r2_cig.p, sizeof(uint32_t) * (size_t)n * max_ops, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipMemcpyAsync(md, ctx->r2_md.p, (size_t)n * max_md, hipMemcpyDeviceToHost, st), "D2H");
  int64_t hst[ST_N];
  HIPC(hipMemcpyAsync(hst, ctx->r2_stats.p, sizeof(hst), hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "reg2aln execution");
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  Slot& s0 = ctx->slot[0];
  s0.last = bwagpu_stats_t{};
  s0.last.kernel_ms = ms;
  s0.last.cells = hst[ST_CELLS];
  s0.last.rows = hst[ST_ROWS];
  s0.last.ext_calls = hst[ST_CALLS];
  return BWAGPU_OK;
}

int bwagpu_align2_batch(bwagpu_ctx_t* ctx, int32_t n, const bwagpu_align2_task_t* tasks, const uint8_t* qpool,
                        int64_t qpool_len, const uint8_t* tpool, int64_t tpool_len, bwagpu_kswr_t* results) {
  if (!ctx || n < 0 || (n && (!tasks || !results)) || qpool_len < 0 || tpool_len < 0 ||
      (qpool_len && !qpool) || (tpool_len && !tpool))
    return BWAGPU_E_INVAL;
  if (n == 0) return BWAGPU_OK;
  if (const char* why = align2_opt_unsupported(ctx->opt)) return fail(ctx, BWAGPU_E_UNSUPPORTED, why);
  // validate and bin on the host
  std::vector<int32_t> lists[kA2Bins];
  std::vector<int64_t> boff((size_t)n);
  int64_t scratch = 0;
  for (int32_t k = 0; k < n; ++k) {
    const bwagpu_align2_task_t& t = tasks[k];
    if (t.qlen < 0 || t.tlen < 0 || t.qoff < 0 || t.toff < 0 || t.qoff + t.qlen > qpool_len ||
        t.toff + t.tlen > tpool_len)
      return fail(ctx, BWAGPU_E_INVAL, "task outside its pools");
    if (t.qlen > BWAGPU_MAX_READ_LEN) return fail(ctx, BWAGPU_E_UNSUPPORTED, "qlen > BWAGPU_MAX_READ_LEN");
    const bool u8 = (t.xtra & BWAGPU_KSW_XBYTE) != 0;
    if (!u8 && (int64_t)t.qlen * ctx->opt.max_mat > 32767)
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "i16 scores could saturate (qlen * max score > 32767)");
    lists[a2_bin_of(t.qlen, u8)].push_back(k);
    boff[(size_t)k] = scratch;
    scratch += (int64_t)t.tlen + 1;
  }
  for (int64_t i = 0; i < qpool_len; ++i)
    if (qpool[i] > 4) return fail(ctx, BWAGPU_E_INVAL, "query base > 4");
  for (int64_t i = 0; i < tpool_len; ++i)
    if (tpool[i] > 4) return fail(ctx, BWAGPU_E_INVAL, "target base > 4");
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  Slot& s = ctx->slot[0];
  hipStream_t st = nullptr;
  HIPC(lazy_stream(s, &st), "hipStreamCreate");
  HIPC(ctx->a2_tasks.ensure(sizeof(bwagpu_align2_task_t) * n), "hipMalloc");
  HIPC(ctx->a2_q.ensure((size_t)qpool_len + 1), "hipMalloc");
  HIPC(ctx->a2_t.ensure((size_t)tpool_len + 1), "hipMalloc");
  HIPC(ctx->a2_out.ensure(sizeof(bwagpu_kswr_t) * n), "hipMalloc");
  HIPC(ctx->a2_scratch.ensure(sizeof(int2) * (size_t)scratch), "hipMalloc");
  HIPC(ctx->a2_lists.ensure(sizeof(int32_t) * n), "hipMalloc");
  // counts[kA2Bins] | cursors[kA2Bins] | stats[ST_N]
  HIPC(ctx->a2_counts.ensure(sizeof(int32_t) * 2 * kA2Bins + sizeof(int64_t) * ST_N), "hipMalloc");
  HIPC(ctx->a2_boff.ensure(sizeof(int64_t) * n), "hipMalloc");
  std::vector<int32_t> all;
  all.reserve((size_t)n);
  int32_t counts[2 * kA2Bins] = {}, list_off[kA2Bins];
  std::vector<std::pair<int64_t, int>> order;  // bins by total rows, largest first
  for (int b = 0; b < kA2Bins; ++b) {
    // longest target first inside a bin (rows ~ tlen): the last claims are the short tasks
    std::stable_sort(lists[b].begin(), lists[b].end(),
                     [&](int32_t x, int32_t y) { return tasks[x].tlen > tasks[y].tlen; });
    counts[b] = (int32_t)lists[b].size();
    list_off[b] = (int32_t)all.size();
    all.insert(all.end(), lists[b].begin(), lists[b].end());
    int64_t rows = 0;
    for (int32_t k : lists[b]) rows += tasks[k].tlen;
    if (counts[b]) order.push_back({rows * kA2CD[b % kA2Buckets], b});
  }
  std::sort(order.begin(), order.end(), [](const std::pair<int64_t, int>& x, const std::pair<int64_t, int>& y) {
    return x.first > y.first;
  });
  std::vector<int> bins;
  for (auto& o : order) bins.push_back(o.second);
  int32_t* d_counts = ctx->a2_counts.as<int32_t>();
  int64_t* d_stats = (int64_t*)(d_counts + 2 * kA2Bins);
  HIPC(hipMemcpyAsync(ctx->a2_tasks.p, tasks, sizeof(bwagpu_align2_task_t) * n, hipMemcpyHostToDevice, st), "H2D");
  if (qpool_len) HIPC(hipMemcpyAsync(ctx->a2_q.p, qpool, (size_t)qpool_len, hipMemcpyHostToDevice, st), "H2D");
  if (tpool_len) HIPC(hipMemcpyAsync(ctx->a2_t.p, tpool, (size_t)tpool_len, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemcpyAsync(ctx->a2_lists.p, all.data(), sizeof(int32_t) * n, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemcpyAsync(d_counts, counts, sizeof(counts), hipMemcpyHostToDevice, st), "H2D");  // + zero cursors
  HIPC(hipMemsetAsync(d_stats, 0, sizeof(int64_t) * ST_N, st), "memset");
  HIPC(hipMemcpyAsync(ctx->a2_boff.p, boff.data(), sizeof(int64_t) * n, hipMemcpyHostToDevice, st), "H2D");
  hipEvent_t e0 = nullptr, e1 = nullptr;  // own events: slot 0's may time an in-flight chain2aln batch
  HIPC(hipEventCreate(&e0), "event");
  HIPC(hipEventCreate(&e1), "event");
  HIPC(hipEventRecord(e0, st), "event");
  {
    A2Args base{ctx->a2_tasks.as<bwagpu_align2_task_t>(), ctx->a2_q.as<uint8_t>(), ctx->a2_t.as<uint8_t>(),
                ctx->a2_out.as<bwagpu_kswr_t>(), ctx->a2_scratch.as<int2>(), ctx->a2_boff.as<int64_t>(),
                ctx->a2_lists.as<int32_t>(), nullptr, nullptr, d_stats};
    const int rc = launch_align2_concurrent(ctx, st, bins, base, list_off, counts, d_counts, d_counts + kA2Bins, 0);
    if (rc) return rc;
  }
  HIPC(hipEventRecord(e1, st), "event");
  int64_t hs[ST_N];
  HIPC(hipMemcpyAsync(results, ctx->a2_out.p, sizeof(bwagpu_kswr_t) * n, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipMemcpyAsync(hs, d_stats, sizeof(hs), hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "align2 batch");
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  s.last = bwagpu_stats_t{};
  s.last.kernel_ms = ms;
  s.last.cells = hs[ST_CELLS];
  s.last.rows = hs[ST_ROWS];
  s.last.ext_calls = hs[ST_CALLS];
  return BWAGPU_OK;
}

int bwagpu_align2_device(bwagpu_ctx_t* ctx, int32_t n, const bwagpu_align2_task_t* dev_tasks,
                         const uint8_t* dev_qpool, const uint8_t* dev_tpool, bwagpu_kswr_t* dev_results,
                         void* dev_scratch, void* stream) {
  if (!ctx || n < 0 || (n && (!dev_tasks || !dev_results || !dev_scratch))) return BWAGPU_E_INVAL;
  if (n == 0) return BWAGPU_OK;
  if (const char* why = align2_opt_unsupported(ctx->opt)) return fail(ctx, BWAGPU_E_UNSUPPORTED, why);
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = (hipStream_t)stream;
  if (!st) HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  HIPC(ctx->a2_lists.ensure(sizeof(int32_t) * (size_t)kA2Bins * n), "hipMalloc");
  HIPC(ctx->a2_boff.ensure(sizeof(int64_t) * n), "hipMalloc");
  // counts[kA2Bins] | cursors[kA2Bins] | scratch cursor (u64) | stats[ST_N]
  const size_t cbytes = sizeof(int32_t) * 2 * kA2Bins + sizeof(int64_t) * (1 + ST_N);
  HIPC(ctx->a2_counts.ensure(cbytes), "hipMalloc");
  int32_t* d_counts = ctx->a2_counts.as<int32_t>();
  unsigned long long* cursor = (unsigned long long*)(d_counts + 2 * kA2Bins);
  int64_t* d_stats = (int64_t*)(cursor + 1);
  HIPC(hipMemsetAsync(d_counts, 0, cbytes, st), "memset");
  HIPC(launch_align2_bins(dev_tasks, n, ctx->a2_lists.as<int32_t>(), d_counts, ctx->a2_boff.as<int64_t>(), cursor,
                          dev_results, d_stats, st),
       "align2 bin launch");
  // counts are on the device only: every bin's kernel is launched with a
  // resident-capacity grid; an empty bin's waves exit on their first claim
  std::vector<int> bins;
  for (int b : {2, 3, 10, 11, 1, 9, 0, 8, 4, 12, 5, 13, 6, 14, 7, 15}) bins.push_back(b);
  A2Args base{dev_tasks, dev_qpool, dev_tpool, dev_results, (int2*)dev_scratch, ctx->a2_boff.as<int64_t>(),
              ctx->a2_lists.as<int32_t>(), nullptr, nullptr, d_stats};
  return launch_align2_concurrent(ctx, st, bins, base, nullptr, nullptr, d_counts, d_counts + kA2Bins, (size_t)n);
}

int bwagpu_debug_set_trace(bwagpu_ctx_t* ctx, void* dev_ptr) {
  if (!ctx) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  HIPC(set_trace(dev_ptr), "set trace");
  HIPC(set_trace_spec(dev_ptr), "set trace");
  return BWAGPU_OK;
}

int bwagpu_debug_fail_wait(bwagpu_ctx_t* ctx, int after_n_waits, int code) {
  if (!ctx || code <= 0) return BWAGPU_E_INVAL;
  ctx->fail_after = after_n_waits;
  ctx->fail_code = code;
  return BWAGPU_OK;
}


int bwagpu_debug_occupancy(bwagpu_ctx_t* ctx, void* stream, int64_t* out) {
  if (!ctx || !out) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = (hipStream_t)stream;
  if (!st) HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int k = 0;
  while (k < BWAGPU_NUM_SLOTS && ctx->dev_stream[k] != st) ++k;
  if (k == BWAGPU_NUM_SLOTS || !ctx->dev_scratch[k].d_ctr.p) return fail(ctx, BWAGPU_E_INVAL, "no device-entry batch on this stream");
  HIPC(hipStreamSynchronize(st), "hipStreamSynchronize");
  int32_t c[SPC_WORDS];
  HIPC(hipMemcpy(c, ctx->dev_scratch[k].d_ctr.p, sizeof c, hipMemcpyDeviceToHost), "hipMemcpy(ctr)");
  memcpy(out, c + 32, 14 * sizeof(int64_t));
#ifdef BWAGPU_OCC_DIAG
  return BWAGPU_OK;
#else
  return fail(ctx, BWAGPU_E_UNSUPPORTED, "built without BWAGPU_OCC_DIAG");
#endif
}

int bwagpu_debug_spec_counters(bwagpu_ctx_t* ctx, void* stream, int64_t* out) {
  if (!ctx || !out) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = (hipStream_t)stream;
  if (!st) HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int k = 0;
  while (k < BWAGPU_NUM_SLOTS && ctx->dev_stream[k] != st) ++k;
  if (k == BWAGPU_NUM_SLOTS || !ctx->dev_scratch[k].d_ctr.p) return fail(ctx, BWAGPU_E_INVAL, "no device-entry batch on this stream");
  HIPC(hipStreamSynchronize(st), "hipStreamSynchronize");
  int32_t c[SPC_WORDS];
  HIPC(hipMemcpy(c, ctx->dev_scratch[k].d_ctr.p, sizeof c, hipMemcpyDeviceToHost), "hipMemcpy(ctr)");
  for (int r = 0; r < kSpecRounds; ++r) {
    out[r] = 0;
    for (int b = 0; b < kSpecBins; ++b) out[r] += c[SPC_CNT + r * kSpecBins + b];
  }
  int64_t spec = 0;
  memcpy(&spec, c + SPC_SPEC64, 8);
  out[3] = spec;
  out[4] = c[SPC_MISS];
  out[5] = c[SPC_HEAVY_N];
  out[6] = c[SPC_REDO_N];
  out[7] = c[SPC_HCOLS];
  return BWAGPU_OK;
}

int bwagpu_debug_spec_ext(bwagpu_ctx_t* ctx, void* stream, void* host_out, int32_t n) {
  if (!ctx || !host_out || n < 0) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = (hipStream_t)stream;
  if (!st) HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int k = 0;
  while (k < BWAGPU_NUM_SLOTS && ctx->dev_stream[k] != st) ++k;
  if (k == BWAGPU_NUM_SLOTS || !ctx->dev_scratch[k].d_ext.p || ctx->dev_scratch[k].d_ext.cap < sizeof(SeedExt) * (size_t)n)
    return fail(ctx, BWAGPU_E_INVAL, "no device-entry batch of that size on this stream");
  HIPC(hipStreamSynchronize(st), "hipStreamSynchronize");
  HIPC(hipMemcpy(host_out, ctx->dev_scratch[k].d_ext.p, sizeof(SeedExt) * (size_t)n, hipMemcpyDeviceToHost),
       "hipMemcpy(ext)");
  return BWAGPU_OK;
}

int bwagpu_debug_ext_form(int form) { return set_ext_form(form); }

int bwagpu_streams_concurrent(void* a, void* b) {
  if (!a || !b || a == b) return BWAGPU_E_INVAL;
  return streams_concurrent((hipStream_t)a, (hipStream_t)b) ? 1 : 0;
}

int bwagpu_ctx_ext_form(bwagpu_ctx_t* ctx, int form) {
  if (!ctx) return BWAGPU_E_INVAL;
  const int prev = ctx->ext_form;
  if (form >= 0) ctx->ext_form = form > 2 ? 1 : form;
  return prev;
}

int bwagpu_ctx_row_bound(bwagpu_ctx_t* ctx, int on) {
  if (!ctx) return BWAGPU_E_INVAL;
  const int prev = ctx->opt.row_bound;
  if (on >= 0) ctx->opt.row_bound = on ? 1 : 0;
  return prev;
}

int bwagpu_debug_ext_kernel(bwagpu_ctx_t* ctx, int32_t lq_max) {
  if (!ctx || lq_max < 1 || lq_max > BWAGPU_MAX_READ_LEN) return BWAGPU_E_INVAL;
  return ext_kernel_for(ctx->opt, ctx->ext_form, tb_bytes_for(ctx->opt, lq_max));
}

int bwagpu_prof_start(bwagpu_ctx_t* ctx, int max_launches) {
  if (!ctx || max_launches < 0) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  for (hipEvent_t e : ctx->prof_ev) HIPC(hipEventSynchronize(e), "hipEventSynchronize");
  for (hipEvent_t e : ctx->prof_ev) (void)hipEventDestroy(e);
  ctx->prof_ev.clear();
  ctx->prof_used = 0;
  for (int i = 0; i < 2 * max_launches; ++i) {
    hipEvent_t e = nullptr;
    HIPC(hipEventCreate(&e), "hipEventCreate");
    ctx->prof_ev.push_back(e);
  }
  return BWAGPU_OK;
}

int bwagpu_prof_read(bwagpu_ctx_t* ctx, double* total_ms, int32_t* launches) {
  if (!ctx || !total_ms || !launches) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  double t = 0;
  for (int i = 0; i + 1 < ctx->prof_used; i += 2) {
    HIPC(hipEventSynchronize(ctx->prof_ev[i + 1]), "hipEventSynchronize");
    float ms = 0;
    HIPC(hipEventElapsedTime(&ms, ctx->prof_ev[i], ctx->prof_ev[i + 1]), "hipEventElapsedTime");
    t += ms;
  }
  *total_ms = t;
  *launches = ctx->prof_used / 2;
  return BWAGPU_OK;
}

int bwagpu_prof_intervals(bwagpu_ctx_t* ctx, double* start_ms, double* end_ms, int32_t max, int32_t* n) {
  if (!ctx || !n || max < 0 || (max && (!start_ms || !end_ms))) return BWAGPU_E_INVAL;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  int k = 0;
  for (int i = 0; i + 1 < ctx->prof_used && k < max; i += 2, ++k) {
    HIPC(hipEventSynchronize(ctx->prof_ev[i + 1]), "hipEventSynchronize");
    float a = 0, b = 0;
    HIPC(hipEventElapsedTime(&a, ctx->prof_ev[0], ctx->prof_ev[i]), "hipEventElapsedTime");
    HIPC(hipEventElapsedTime(&b, ctx->prof_ev[0], ctx->prof_ev[i + 1]), "hipEventElapsedTime");
    start_ms[k] = a;
    end_ms[k] = b;
  }
  *n = k;
  return BWAGPU_OK;
}

int bwagpu_last_stats(const bwagpu_ctx_t* ctx, int slot, bwagpu_stats_t* out) {
  if (!ctx || !out || slot < 0 || slot >= BWAGPU_NUM_SLOTS) return BWAGPU_E_INVAL;
  *out = ctx->slot[slot].last;
  return BWAGPU_OK;
}

}  // extern "C"

// ------------------------------------------------------------------ seeding
extern "C" int bwagpu_set_bwt(bwagpu_ctx_t* ctx, const bwagpu_bwt_t* bwt) {
  if (!ctx || !bwt || !bwt->bwt || bwt->bwt_size == 0) return BWAGPU_E_INVAL;
  // the occurrence array covers every position: 16 words per 128 positions
  if (bwt->bwt_size < ((bwt->seq_len + 127) >> 7) * 16 || bwt->L2[4] != bwt->seq_len || bwt->primary > bwt->seq_len)
    return fail(ctx, BWAGPU_E_INVAL, "bwt header inconsistent with its occurrence array");
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  HIPC(ctx->bwt_words.ensure(sizeof(uint32_t) * bwt->bwt_size + 64), "hipMalloc");
  HIPC(hipMemcpy(ctx->bwt_words.p, bwt->bwt, sizeof(uint32_t) * bwt->bwt_size, hipMemcpyHostToDevice), "H2D");
  ctx->bwt.primary = bwt->primary;
  for (int i = 0; i < 5; ++i) ctx->bwt.L2[i] = bwt->L2[i];
  ctx->bwt.seq_len = bwt->seq_len;
  ctx->bwt.bwt = ctx->bwt_words.as<uint32_t>();
  {  // the device occurrence layout (seed.hip: 64-position blocks)
    HIPC(ctx->occ_d.ensure(2 * sizeof(uint4) * (size_t)occ64_blocks(bwt->seq_len)), "hipMalloc");
    ctx->bwt.sup_shift = ctx->sup_shift;
    HIPC(ctx->sup_d.ensure(4 * sizeof(uint64_t) * (size_t)occ64_supers(bwt->seq_len, ctx->sup_shift)), "hipMalloc");
    HIPC(hipMemset(ctx->occ_d.p, 0, 2 * sizeof(uint4) * (size_t)occ64_blocks(bwt->seq_len)), "memset");
    hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
    HIPC(launch_build_occ64(ctx->bwt, ctx->occ_d.as<uint4>(), ctx->sup_d.as<uint64_t>(), st), "build_occ64 launch");
    HIPC(hipStreamSynchronize(st), "sync");
    ctx->bwt.occ = ctx->occ_d.as<uint4>();
    ctx->bwt.sup = ctx->sup_d.as<uint64_t>();
  }
  ctx->bwt.sa = nullptr;
  ctx->bwt.sa_mask = 0;
  ctx->bwt.sa_shift = 0;
  ctx->bwt.sa_full32 = nullptr;
  ctx->bwt.sa_full64 = nullptr;
  if (bwt->sa) {
    const int iv = bwt->sa_intv;
    if (iv < 1 || (iv & (iv - 1)) || bwt->n_sa < bwt->seq_len / (uint64_t)iv + 1)
      return fail(ctx, BWAGPU_E_INVAL, "suffix array sample interval / size inconsistent");
    HIPC(ctx->sa_d.ensure(sizeof(uint64_t) * bwt->n_sa), "hipMalloc");
    HIPC(hipMemcpy(ctx->sa_d.p, bwt->sa, sizeof(uint64_t) * bwt->n_sa, hipMemcpyHostToDevice), "H2D");
    ctx->bwt.sa = ctx->sa_d.as<uint64_t>();
    ctx->bwt.sa_mask = (uint64_t)iv - 1;
    while ((1 << ctx->bwt.sa_shift) < iv) ++ctx->bwt.sa_shift;
    // every row's entry in HBM (one load per bwt_sa instead of a walk of ~sa_intv
    // dependent occurrence lookups): 32-bit entries below 2^32 rows (chr21: 0.37
    // GB), 64-bit above (GRCh38: 50 GB of the 288), within 64 GB and a quarter
    // of the free memory; BWAGPU_SA_FULL=0 keeps the sampled walk, =64 forces
    // 64-bit entries (tests)
    const char* fe = getenv("BWAGPU_SA_FULL");
    const bool narrow = bwt->seq_len < 0xffffffffull && !(fe && strcmp(fe, "64") == 0);
    const uint64_t bytes = (bwt->seq_len + 1) * (narrow ? 4 : 8);
    size_t free_b = 0, total_b = 0;
    if (!(fe && strcmp(fe, "0") == 0) && iv > 1 && hipMemGetInfo(&free_b, &total_b) == hipSuccess &&
        bytes <= ((uint64_t)64 << 30) && bytes <= free_b / 4) {
      HIPC(ctx->sa_full.ensure((size_t)bytes), "hipMalloc");
      hipStream_t st = nullptr;
      HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
      HIPC(launch_sa_expand(ctx->bwt, narrow ? ctx->sa_full.as<uint32_t>() : nullptr,
                            narrow ? nullptr : ctx->sa_full.as<uint64_t>(), st),
           "sa_expand launch");
      HIPC(hipStreamSynchronize(st), "sync");
      if (narrow) ctx->bwt.sa_full32 = ctx->sa_full.as<uint32_t>();
      else ctx->bwt.sa_full64 = ctx->sa_full.as<uint64_t>();
    }
  }
  ctx->has_bwt = true;
  return BWAGPU_OK;
}

extern "C" int bwagpu_bwt_sa(bwagpu_ctx_t* ctx, int64_t n, const uint64_t* k, uint64_t* out) {
  if (!ctx || n < 0 || (n && (!k || !out))) return BWAGPU_E_INVAL;
  if (!ctx->has_bwt || !ctx->bwt.sa) return fail(ctx, BWAGPU_E_INVAL, "no suffix array: pass it to bwagpu_set_bwt");
  for (int64_t i = 0; i < n; ++i)
    if (k[i] > ctx->bwt.seq_len) return fail(ctx, BWAGPU_E_INVAL, "BWT position past seq_len");
  if (n == 0) return BWAGPU_OK;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  HIPC(ctx->sa_in.ensure(sizeof(uint64_t) * (size_t)n), "hipMalloc");
  HIPC(ctx->sa_out.ensure(sizeof(uint64_t) * (size_t)n), "hipMalloc");
  HIPC(hipMemcpyAsync(ctx->sa_in.p, k, sizeof(uint64_t) * (size_t)n, hipMemcpyHostToDevice, st), "H2D");
  HIPC(launch_bwt_sa(ctx->bwt, n, ctx->sa_in.as<uint64_t>(), ctx->sa_out.as<uint64_t>(), st), "bwt_sa launch");
  HIPC(hipMemcpyAsync(out, ctx->sa_out.p, sizeof(uint64_t) * (size_t)n, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  return BWAGPU_OK;
}

namespace {

// the checks of bwagpu_collect_intv's arguments; *bases = the batch's bases
// The pinned staging buffer of seeding's reads (seq_off, then the bases),
// once the previous call's H2D out of it is done (a caller that returned
// early on an error never synchronized its stream)
int seed_pin(bwagpu_ctx_t* ctx, int32_t n_reads, int64_t nb, char** pin) {
  if (ctx->sdh_done) HIPC(hipEventSynchronize(ctx->sdh_done), "hipEventSynchronize");
  else HIPC(hipEventCreateWithFlags(&ctx->sdh_done, hipEventDisableTiming), "hipEventCreate");
  HIPC(ctx->sdh_in.ensure(sizeof(int64_t) * ((size_t)n_reads + 1) + (size_t)nb), "hipHostMalloc");
  *pin = ctx->sdh_in.as<char>();
  return BWAGPU_OK;
}

// Checks a seeding batch: the read lengths and every base (nt4: 0..4), on up
// to 8 threads for a batch of megabases.  stage: the same pass also copies
// the reads into the pinned staging buffer (seed_pin; seed_enqueue then skips
// its copy).  *lq_max (optional) = the longest read.
int seed_validate(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* opt, int32_t n_reads, const int64_t* seq_off,
                  const uint8_t* seq, int64_t* bases, bool stage = false, int* lq_max = nullptr) {
  if (!ctx->has_bwt) return fail(ctx, BWAGPU_E_INVAL, "no FM-index: call bwagpu_set_bwt first");
  if (opt->min_seed_len < 1 || opt->split_width < 0) return fail(ctx, BWAGPU_E_INVAL, "bad seeding options");
  *bases = 0;
  if (lq_max) *lq_max = 0;
  if (n_reads == 0) return BWAGPU_OK;
  const int64_t nb = seq_off[n_reads] - seq_off[0];
  if (seq_off[0] != 0 || nb < 0 || (nb && !seq)) return fail(ctx, BWAGPU_E_INVAL, "seq_off must start at 0");
  char* pin = nullptr;
  if (stage) {
    int rc = seed_pin(ctx, n_reads, nb, &pin);
    if (rc) return rc;
  }
  const size_t ob = sizeof(int64_t) * ((size_t)n_reads + 1);
  // one thread takes ~1 ms per 10 Mbases
  const int nt = nb >= (1 << 22) ? 8 : 1;
  int len_bad[8] = {}, base_bad[8] = {};
  int64_t lms[8] = {};
  auto part = [&](int t) {
    int64_t lm = 0;
    for (int32_t r = (int32_t)((int64_t)n_reads * t / nt); r < (int32_t)((int64_t)n_reads * (t + 1) / nt); ++r) {
      const int64_t l = seq_off[r + 1] - seq_off[r];
      if (l < 0) len_bad[t] |= 1;
      if (l > BWAGPU_MAX_SEED_READ) len_bad[t] |= 2;
      lm = std::max(lm, l);
    }
    lms[t] = lm;
    if (pin && t == 0) memcpy(pin, seq_off, ob);
    // eight bytes at a time: (b & 0x7f) + 0x7b carries into bit 7 iff b > 4
    int64_t i = (nb * t / nt) & ~(int64_t)7;
    const int64_t e = t == nt - 1 ? nb : (nb * (t + 1) / nt) & ~(int64_t)7;
    uint64_t bad = 0;
    char* const dst = pin ? pin + ob : nullptr;
    for (; i + 8 <= e; i += 8) {
      uint64_t w;
      memcpy(&w, seq + i, 8);
      bad |= (((w & 0x7f7f7f7f7f7f7f7fULL) + 0x7b7b7b7b7b7b7b7bULL) | w) & 0x8080808080808080ULL;
      if (dst) memcpy(dst + i, &w, 8);
    }
    for (; i < e; ++i) {
      bad |= seq[i] > 4;
      if (dst) dst[i] = (char)seq[i];
    }
    base_bad[t] = bad != 0;
  };
  host_parallel(nt, part);
  int lb = 0, bb = 0;
  int64_t lm = 0;
  for (int t = 0; t < nt; ++t) {
    lb |= len_bad[t];
    bb |= base_bad[t];
    lm = std::max(lm, lms[t]);
  }
  if (lb & 1) return fail(ctx, BWAGPU_E_INVAL, "seq_off not monotone");
  if (lb & 2) return fail(ctx, BWAGPU_E_UNSUPPORTED, "read longer than BWAGPU_MAX_SEED_READ");
  if (bb) return fail(ctx, BWAGPU_E_INVAL, "read base > 4 (bases are nt4)");
  *bases = nb;
  if (lq_max) *lq_max = (int)lm;
  return BWAGPU_OK;
}

// H2D of the reads (when upload) and mem_collect_intv into per-read slots of
// max_per_read intervals (ctx->sd_*), enqueued on st
int seed_enqueue(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* opt, int32_t n_reads, const int64_t* seq_off,
                 const uint8_t* seq, int64_t bases, int32_t max_per_read, bool upload, hipStream_t st, SeedArgs& a,
                 bool staged = false) {
  HIPC(ctx->sd_off.ensure(sizeof(int64_t) * ((size_t)n_reads + 1)), "hipMalloc");
  HIPC(ctx->sd_seq.ensure((size_t)bases + 1), "hipMalloc");
  HIPC(ctx->sd_out.ensure(sizeof(bwagpu_intv_t) * (size_t)n_reads * (size_t)max_per_read), "hipMalloc");
  HIPC(ctx->sd_n.ensure(sizeof(int32_t) * (size_t)n_reads), "hipMalloc");
  HIPC(ctx->sd_scratch.ensure(sizeof(bwagpu_intv_t) * (size_t)seed_scratch_entries(bases, n_reads)), "hipMalloc");
  if (upload) {  // through a pinned staging buffer filled on a few threads (a pageable H2D runs at a fraction)
    const size_t ob = sizeof(int64_t) * ((size_t)n_reads + 1);
    char* pin = ctx->sdh_in.as<char>();
    if (!staged) {  // else seed_validate's pass filled it
      int rc = seed_pin(ctx, n_reads, bases, &pin);
      if (rc) return rc;
      const int nt = bases >= (1 << 22) ? 8 : 1;
      auto part = [&](int t) {
        const size_t b0 = (size_t)bases * t / nt, b1 = (size_t)bases * (t + 1) / nt;
        memcpy(pin + ob + b0, seq + b0, b1 - b0);
        if (t == 0) memcpy(pin, seq_off, ob);
      };
      host_parallel(nt, part);
    }
    HIPC(hipMemcpyAsync(ctx->sd_off.p, pin, ob, hipMemcpyHostToDevice, st), "H2D");
    if (bases) HIPC(hipMemcpyAsync(ctx->sd_seq.p, pin + ob, (size_t)bases, hipMemcpyHostToDevice, st), "H2D");
    HIPC(hipEventRecord(ctx->sdh_done, st), "hipEventRecord");
  }
  a = SeedArgs{};
  a.n_reads = n_reads;
  a.seq_off = ctx->sd_off.as<int64_t>();
  a.seq = ctx->sd_seq.as<uint8_t>();
  a.max_per_read = max_per_read;
  a.out = ctx->sd_out.as<bwagpu_intv_t>();
  a.out_n = ctx->sd_n.as<int32_t>();
  a.scratch = ctx->sd_scratch.as<bwagpu_intv_t>();
  a.min_seed_len = opt->min_seed_len;
  a.split_width = opt->split_width;
  a.max_mem_intv = opt->max_mem_intv;
  a.split_len = (int)(opt->min_seed_len * opt->split_factor + .499);  // bwamem.c:124
  HIPC(ctx->sd_heavy.ensure(sizeof(int32_t) * (3 * (size_t)n_reads + 1)), "hipMalloc");
  a.budget = ctx->seed_budget;
  a.heavy = ctx->sd_heavy.as<int32_t>() + 1;
  a.n_heavy = ctx->sd_heavy.as<int32_t>();
  a.flags = a.heavy + n_reads;
  a.p3_n = a.flags + n_reads;
  if (getenv("BWAGPU_SEED_DBG")) {  // per-lane tier-1 stamps (tools_dev)
    HIPC(ctx->sd_dbg.ensure(sizeof(int64_t) * 8 * (size_t)n_reads), "hipMalloc");
    HIPC(hipMemsetAsync(ctx->sd_dbg.p, 0, sizeof(int64_t) * 8 * (size_t)n_reads, st), "memset");
    a.dbg = ctx->sd_dbg.as<int64_t>();
  }
  HIPC(launch_collect_intv(ctx->bwt, a, st), "collect_intv launch");
  return BWAGPU_OK;
}

}  // namespace

extern "C" int bwagpu_collect_intv(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* opt, int32_t n_reads,
                                   const int64_t* seq_off, const uint8_t* seq, int32_t max_per_read,
                                   bwagpu_intv_t* out, int64_t out_cap, int32_t* out_n) {
  if (!ctx || !opt || n_reads < 0 || max_per_read < 1 || out_cap < 0 || (n_reads && (!seq_off || !out_n)) ||
      (out_cap && !out))
    return BWAGPU_E_INVAL;
  int64_t bases = 0;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  int rc = seed_validate(ctx, opt, n_reads, seq_off, seq, &bases, true);
  if (rc) return rc;
  if (n_reads == 0) return BWAGPU_OK;
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  SeedArgs a;
  if ((rc = seed_enqueue(ctx, opt, n_reads, seq_off, seq, bases, max_per_read, true, st, a, true))) return rc;
  HIPC(hipMemcpyAsync(out_n, ctx->sd_n.p, sizeof(int32_t) * (size_t)n_reads, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  if (const char* dp = getenv("BWAGPU_SEED_DBG")) {
    std::vector<int64_t> d(8 * (size_t)n_reads);
    HIPC(hipMemcpy(d.data(), ctx->sd_dbg.p, sizeof(int64_t) * d.size(), hipMemcpyDeviceToHost), "D2H");
    if (FILE* f = fopen(dp, "ab")) {
      fwrite(d.data(), sizeof(int64_t), d.size(), f);
      fclose(f);
    }
  }
  // pack the per-read slots back to back (read order) and copy only those
  std::vector<int64_t> off((size_t)n_reads + 1, 0);
  for (int32_t r = 0; r < n_reads; ++r) {
    if (out_n[r] < 0) return fail(ctx, BWAGPU_E_UNSUPPORTED, "a read has more than max_per_read intervals");
    off[(size_t)r + 1] = off[(size_t)r] + out_n[r];
  }
  const int64_t total = off[(size_t)n_reads];
  if (total > out_cap) return fail(ctx, BWAGPU_E_UNSUPPORTED, "the batch has more than out_cap intervals");
  if (total == 0) return BWAGPU_OK;
  HIPC(ctx->sd_poff.ensure(sizeof(int64_t) * off.size()), "hipMalloc");
  HIPC(ctx->sd_pack.ensure(sizeof(bwagpu_intv_t) * (size_t)total), "hipMalloc");
  HIPC(hipMemcpyAsync(ctx->sd_poff.p, off.data(), sizeof(int64_t) * off.size(), hipMemcpyHostToDevice, st), "H2D");
  HIPC(launch_pack_intv(a, ctx->sd_poff.as<int64_t>(), ctx->sd_pack.as<bwagpu_intv_t>(), st), "pack launch");
  HIPC(hipMemcpyAsync(out, ctx->sd_pack.p, sizeof(bwagpu_intv_t) * (size_t)total, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  return BWAGPU_OK;
}

extern "C" int bwagpu_debug_seed_budget(bwagpu_ctx_t* ctx, int32_t budget) {
  if (!ctx || budget < 0) return BWAGPU_E_INVAL;
  ctx->seed_budget = budget;
  return BWAGPU_OK;
}

extern "C" int bwagpu_set_device_read_len(bwagpu_ctx_t* ctx, int32_t max_len) {
  if (!ctx || max_len < 1 || max_len > BWAGPU_MAX_READ_LEN) return BWAGPU_E_INVAL;
  ctx->dev_read_len = max_len;
  return BWAGPU_OK;
}

extern "C" int bwagpu_debug_sup_shift(bwagpu_ctx_t* ctx, int32_t shift) {
  if (!ctx || shift < 7 || shift > 32) return BWAGPU_E_INVAL;  // a superblock is whole 128-position bwa blocks
  ctx->sup_shift = shift;
  return BWAGPU_OK;
}

// The FPGA back end's own job (sw_top, xlnx/XCLAgent.cpp:89-106) on its wire
// format: the host walks the record chain (one load per read record — the
// "end" words of packReadData, FPGAPipeline.cpp:258,336) and checks lengths;
// the device decodes and checks everything else (stream_decode_kernel) and
// extends every task (stream_ext_kernel).  Device-found problems come back as
// BWAGPU_E_RESULTS, the fpgaResultsError of processOutput's checks
// (FPGAPipeline.cpp:38-74).
extern "C" int bwagpu_sw_stream(bwagpu_ctx_t* ctx, const int32_t* i_buf, int64_t i_words, int16_t* o_buf,
                                int32_t o_cap_tasks, int32_t* o_tasks) {
  if (!ctx || !o_tasks || i_words < 0 || o_cap_tasks < 0 || (i_words && !i_buf) || (o_cap_tasks && !o_buf))
    return BWAGPU_E_INVAL;
  *o_tasks = 0;
  if (i_words == 0) return BWAGPU_OK;
  std::vector<int64_t> starts;
  int lq_max = 1;
  for (int64_t p = 0; p < i_words;) {
    const int64_t end = i_buf[p];
    if (end <= p + 2 || end > i_words) return fail(ctx, BWAGPU_E_INVAL, "stream: a record's end word is out of range");
    const int lq = i_buf[p + 1];
    if (lq < 0) return fail(ctx, BWAGPU_E_INVAL, "stream: negative read length");
    if (lq > BWAGPU_MAX_READ_LEN) return fail(ctx, BWAGPU_E_UNSUPPORTED, "stream: read longer than BWAGPU_MAX_READ_LEN");
    lq_max = std::max(lq_max, lq);
    starts.push_back(p);
    p = end;
  }
  const int tb = tb_bytes_for(ctx->opt, lq_max);
  if ((size_t)(kBlock / 64) * 2 * tb > 64 * 1024)
    return fail(ctx, BWAGPU_E_UNSUPPORTED, "LDS row buffer too large for these options (w, pen_clip, read length)");
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  const size_t cap = (size_t)std::max(o_cap_tasks, 1), nr = starts.size();
  HIPC(ctx->st_buf.ensure(sizeof(int32_t) * (size_t)i_words), "hipMalloc");
  HIPC(ctx->st_start.ensure(sizeof(int64_t) * nr), "hipMalloc");
  HIPC(ctx->st_q.ensure(8 * (size_t)i_words), "hipMalloc");
  HIPC(ctx->st_tasks.ensure(sizeof(StreamTask) * cap), "hipMalloc");
  HIPC(ctx->st_lists.ensure(sizeof(int32_t) * kSpecBins * cap), "hipMalloc");
  HIPC(ctx->st_seen.ensure(sizeof(int32_t) * cap), "hipMalloc");
  HIPC(ctx->st_ctr.ensure(sizeof(int32_t) * kStrCtrWords), "hipMalloc");
  HIPC(ctx->st_out.ensure(sizeof(int32_t) * 5 * cap), "hipMalloc");
  HIPC(hipMemcpyAsync(ctx->st_buf.p, i_buf, sizeof(int32_t) * (size_t)i_words, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemcpyAsync(ctx->st_start.p, starts.data(), sizeof(int64_t) * nr, hipMemcpyHostToDevice, st), "H2D");
  HIPC(hipMemsetAsync(ctx->st_seen.p, 0, sizeof(int32_t) * cap, st), "memset");
  HIPC(hipMemsetAsync(ctx->st_ctr.p, 0, sizeof(int32_t) * kStrCtrWords, st), "memset");
  StreamArgs a;
  a.buf = ctx->st_buf.as<int32_t>();
  a.rstart = ctx->st_start.as<int64_t>();
  a.n_reads = (int32_t)nr;
  a.cap = (int32_t)cap;
  a.l_pac = ctx->ref.l_pac;
  a.qpool = ctx->st_q.as<uint8_t>();
  a.tasks = ctx->st_tasks.as<StreamTask>();
  a.lists = ctx->st_lists.as<int32_t>();
  a.seen = ctx->st_seen.as<int32_t>();
  a.ctr = ctx->st_ctr.as<int32_t>();
  a.out = ctx->st_out.as<int32_t>();
  if (o_cap_tasks == 0) a.cap = 0;  // every task index is then out of range
  HIPC(launch_sw_stream(ctx->opt, ctx->ref, a, tb, st), "sw_stream launch");
  int32_t c[8];
  HIPC(hipMemcpyAsync(c, ctx->st_ctr.p, sizeof c, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  if (c[kStrErr]) {
    const int e = c[kStrErr];
    return fail(ctx, BWAGPU_E_RESULTS,
                std::string("stream: ") + (e & STR_ERR_RECORD ? "a record does not end at its end word; " : "") +
                    (e & STR_ERR_TASK ? "task index out of range; " : "") +
                    (e & STR_ERR_DUP ? "task index repeated; " : "") +
                    (e & STR_ERR_SEED ? "seed outside its read or window; " : "") +
                    (e & STR_ERR_BASE ? "base > 4; " : ""));
  }
  if (c[kStrDecoded] != c[kStrMax]) return fail(ctx, BWAGPU_E_RESULTS, "stream: task indices are not 0..n-1");
  const int32_t n = c[kStrMax];
  if (n) HIPC(hipMemcpy(o_buf, ctx->st_out.p, sizeof(int32_t) * 5 * (size_t)n, hipMemcpyDeviceToHost), "D2H");
  *o_tasks = n;
  return BWAGPU_OK;
}

// ------------------------------------------------------------------ chaining
// SeqsToChains on the device (chain.h): mem_collect_intv, mem_chain's body,
// mem_chain_flt and mem_flt_chained_seeds, with three host round trips for
// sizes (positions, mem_seed_sw tasks when a read is long enough for them,
// chains out).
namespace {

int run_chaining(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* sopt, const bwagpu_chainopt_t* copt, int32_t n_reads,
                 const int64_t* seq_off, const uint8_t* seq, bool raw, hipStream_t st, int64_t* n_chains,
                 int64_t* n_seeds, int* lq_max_out, bool to_host = false) {
  *n_chains = *n_seeds = 0;
  if (copt->max_occ < 1 || copt->max_chain_gap < 0 || copt->max_chain_extend < 0 || !(copt->mask_level >= 0) ||
      !(copt->drop_ratio >= 0))
    return fail(ctx, BWAGPU_E_INVAL, "bad chaining options");
  if (!ctx->bwt.sa) return fail(ctx, BWAGPU_E_INVAL, "no suffix array: pass it to bwagpu_set_bwt");
  {  // the largest LDS bin's arena (chain.h) needs gfx950's 160 KB per workgroup
    int lds_max = 0;
    HIPC(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device), "attribute");
    if ((size_t)lds_max < lds_arena(kBinCap[kLdsBins - 1]))
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "device LDS per workgroup is smaller than the chaining arena");
  }
  int64_t bases = 0;
  int lq_max = 0;
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  int rc = seed_validate(ctx, sopt, n_reads, seq_off, seq, &bases, true, &lq_max);  // + the staging copy
  if (rc) return rc;
  *lq_max_out = lq_max;
  if (n_reads == 0) return BWAGPU_OK;
  // mem_flt_chained_seeds' gate and min_HSP_score per read length
  // (bwamem.c:609-611), in the host's double arithmetic
  std::vector<int32_t> tab((size_t)lq_max + 1, -1);
  bool any_sw = false;
  {
    std::vector<char> has((size_t)lq_max + 1, 0);
    for (int32_t r = 0; r < n_reads; ++r) has[(size_t)(seq_off[r + 1] - seq_off[r])] = 1;
    for (int l = 1; l <= lq_max; ++l) {
      const double min_l = copt->min_chain_weight ? 1.1f * copt->min_chain_weight : 5.5f * log((double)l);
      if (min_l > 0.05f * l) continue;
      tab[(size_t)l] = (int)(ctx->opt.a * min_l + .499);
      any_sw = any_sw || (has[(size_t)l] && l >= sopt->min_seed_len);
    }
  }
  if (!raw && any_sw)
    if (const char* why = align2_opt_unsupported(ctx->opt)) return fail(ctx, BWAGPU_E_UNSUPPORTED, why);
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  int32_t mpr = std::max(64, 2 * lq_max + 64);  // interval slots per read (grown on overflow)
  SeedArgs sa;
  if ((rc = seed_enqueue(ctx, sopt, n_reads, seq_off, seq, bases, mpr, true, st, sa, true))) return rc;
  const size_t nr = (size_t)n_reads;
  HIPC(ctx->ch_npos.ensure(sizeof(int32_t) * nr), "hipMalloc");
  HIPC(ctx->ch_posoff.ensure(sizeof(int64_t) * (nr + 1)), "hipMalloc");
  HIPC(ctx->ch_frac.ensure(sizeof(float) * nr), "hipMalloc");
  HIPC(ctx->ch_nout.ensure(sizeof(int32_t) * nr), "hipMalloc");
  HIPC(ctx->ch_noseed.ensure(sizeof(int32_t) * nr), "hipMalloc");
  HIPC(ctx->ch_nsw.ensure(sizeof(int32_t) * nr), "hipMalloc");
  HIPC(ctx->ch_need.ensure(sizeof(int32_t)), "hipMalloc");
  HIPC(ctx->ch_swtab.ensure(sizeof(int32_t) * tab.size()), "hipMalloc");
  HIPC(ctx->chh_tot.ensure(sizeof(int64_t) * 8), "hipHostMalloc");
  HIPC(hipMemcpyAsync(ctx->ch_swtab.p, tab.data(), sizeof(int32_t) * tab.size(), hipMemcpyHostToDevice, st), "H2D");
  int64_t* tot = ctx->chh_tot.as<int64_t>();
  ChainArgs a{};
  a.n_reads = n_reads;
  a.seq_off = sa.seq_off;
  a.seq = sa.seq;
  a.max_occ = copt->max_occ;
  a.max_chain_gap = copt->max_chain_gap;
  a.min_chain_weight = copt->min_chain_weight;
  a.max_chain_extend = copt->max_chain_extend;
  a.mask_level = copt->mask_level;
  a.drop_ratio = copt->drop_ratio;
  a.min_seed_len = sopt->min_seed_len;
  a.w = ctx->opt.w;
  a.a = ctx->opt.a;
  a.raw = raw ? 1 : 0;
  a.l_pac = ctx->ref.l_pac;
  a.n_seqs = ctx->ref.n_seqs;
  a.ann_off = ctx->ref.ann_offset;
  a.ann_len = ctx->ref.ann_len;
  a.is_alt = ctx->has_alt ? ctx->ch_alt.as<uint8_t>() : nullptr;
  a.pac = ctx->ref.pac;
  a.sw_tab = ctx->ch_swtab.as<int32_t>();
  a.n_pos = ctx->ch_npos.as<int32_t>();
  a.pos_off = ctx->ch_posoff.as<int64_t>();
  a.frac_rep = ctx->ch_frac.as<float>();
  a.n_out = ctx->ch_nout.as<int32_t>();
  a.n_oseed = ctx->ch_noseed.as<int32_t>();
  a.n_sw = ctx->ch_nsw.as<int32_t>();
  a.need = ctx->ch_need.as<int32_t>();
  for (int pass = 0;; ++pass) {  // positions per read; a read out of interval slots reruns the search
    a.intv = sa.out;
    a.intv_n = sa.out_n;
    a.max_per_read = sa.max_per_read;
    HIPC(hipMemsetAsync(a.need, 0, sizeof(int32_t), st), "memset");
    HIPC(launch_chain_count(a, st), "chain_count launch");
    HIPC(launch_scan_i32(a.n_pos, a.pos_off, n_reads, st), "scan launch");
    HIPC(hipMemcpyAsync(tot, a.pos_off + n_reads, sizeof(int64_t), hipMemcpyDeviceToHost, st), "D2H");
    HIPC(hipMemcpyAsync(tot + 1, a.need, sizeof(int32_t), hipMemcpyDeviceToHost, st), "D2H");
    HIPC(hipStreamSynchronize(st), "sync");
    const int32_t need = (int32_t)(uint32_t)tot[1];
    if (need <= 0) break;
    if (pass) return fail(ctx, BWAGPU_E_DEVICE, "interval slots still overflow");
    if ((rc = seed_enqueue(ctx, sopt, n_reads, seq_off, seq, bases, need, false, st, sa))) return rc;
  }
  const int64_t P = tot[0];
  const size_t p1 = (size_t)std::max<int64_t>(P, 1);
  HIPC(ctx->ch_kpos.ensure(sizeof(uint64_t) * p1), "hipMalloc");
  HIPC(ctx->ch_rbeg.ensure(sizeof(uint64_t) * p1), "hipMalloc");
  HIPC(ctx->ch_qinfo.ensure(sizeof(int2) * p1), "hipMalloc");
  HIPC(ctx->ch_label.ensure(sizeof(int32_t) * p1), "hipMalloc");
  HIPC(ctx->ch_score.ensure(sizeof(int32_t) * p1), "hipMalloc");
  HIPC(ctx->ch_slist.ensure(sizeof(int32_t) * p1), "hipMalloc");
  HIPC(ctx->ch_ord.ensure(sizeof(int32_t) * p1), "hipMalloc");
  HIPC(ctx->ch_chains.ensure(sizeof(LChain) * p1), "hipMalloc");
  HIPC(ctx->ch_nodes.ensure(sizeof(BNode32) * (size_t)node_total(P, n_reads)), "hipMalloc");
  HIPC(ctx->ch_ochains.ensure(sizeof(DChain) * p1), "hipMalloc");
  HIPC(ctx->ch_oslist.ensure(sizeof(int32_t) * p1), "hipMalloc");
  HIPC(ctx->ch_bins.ensure(sizeof(int32_t) * ((size_t)(kLdsBins + 1) * nr + kLdsBins + 1)), "hipMalloc");
  a.kpos = ctx->ch_kpos.as<uint64_t>();
  a.rbeg = ctx->ch_rbeg.as<uint64_t>();
  a.qinfo = ctx->ch_qinfo.as<int2>();
  a.label = ctx->ch_label.as<int32_t>();
  a.score = ctx->ch_score.as<int32_t>();
  a.slist = ctx->ch_slist.as<int32_t>();
  a.ord = ctx->ch_ord.as<int32_t>();
  a.lchains = ctx->ch_chains.as<LChain>();
  a.lnodes = ctx->ch_nodes.as<BNode32>();
  a.ochains = ctx->ch_ochains.as<DChain>();
  a.oslist = ctx->ch_oslist.as<int32_t>();
  a.bin_count = ctx->ch_bins.as<int32_t>();
  a.bin_list = a.bin_count + kLdsBins + 1;
  HIPC(launch_chain_emit(a, st), "chain_emit launch");
  if (P) HIPC(launch_bwt_sa(ctx->bwt, P, a.kpos, a.rbeg, st), "bwt_sa launch");
  if (!ctx->ch_cs.fork) {
    HIPC(hipStreamCreateWithFlags(&ctx->ch_cs.side[0], hipStreamNonBlocking), "hipStreamCreate");
    HIPC(hipEventCreateWithFlags(&ctx->ch_cs.join[0], hipEventDisableTiming), "hipEventCreate");
    HIPC(hipEventCreateWithFlags(&ctx->ch_cs.fork, hipEventDisableTiming), "hipEventCreate");
  }
  const char* dbg_env = getenv("BWAGPU_CHAIN_PHASES");
  const bool dbg_on = dbg_env && dbg_env[0] == '1';
  if (dbg_on) {
    HIPC(ctx->ch_dbg.ensure(sizeof(uint64_t) * 8 * nr), "hipMalloc");
    HIPC(hipMemsetAsync(ctx->ch_dbg.p, 0, sizeof(uint64_t) * 8 * nr, st), "memset");
    a.dbg = ctx->ch_dbg.as<uint64_t>();
  }
  HIPC(launch_chain_build(a, st, ctx->ch_cs), "chain_build launch");
  if (dbg_on) {  // the slowest reads' phase times (100 MHz ticks) to stderr
    std::vector<uint64_t> d(8 * nr);
    HIPC(hipMemcpyAsync(d.data(), ctx->ch_dbg.p, sizeof(uint64_t) * 8 * nr, hipMemcpyDeviceToHost, st), "D2H");
    HIPC(hipStreamSynchronize(st), "sync");
    std::vector<int> idx;
    for (int r = 0; r < n_reads; ++r)
      if (d[8 * (size_t)r + 6]) idx.push_back(r);
    std::sort(idx.begin(), idx.end(), [&](int x, int y) {
      return d[8 * (size_t)x + 6] - d[8 * (size_t)x] > d[8 * (size_t)y + 6] - d[8 * (size_t)y];
    });
    for (size_t k = 0; k < idx.size() && k < 8; ++k) {
      const uint64_t* q = &d[8 * (size_t)idx[k]];
      fprintf(stderr, "[chain phases] read %d pos %u chains %u: loop %.1f trav %.1f prep %.1f sort %.1f flt %.1f out %.1f us\n",
              idx[k], (unsigned)(q[7] & 0xffffffff), (unsigned)(q[7] >> 32), (q[1] - q[0]) / 100.0,
              (q[2] - q[1]) / 100.0, (q[3] ? q[3] - q[2] : 0) / 100.0, (q[4] ? q[4] - q[3] : 0) / 100.0,
              (q[5] - (q[4] ? q[4] : q[2])) / 100.0, (q[6] - q[5]) / 100.0);
    }
  }
  if (!raw && any_sw) {  // mem_flt_chained_seeds: every kept seed of a long read realigned
    HIPC(ctx->ch_swoff.ensure(sizeof(int64_t) * (nr + 1)), "hipMalloc");
    HIPC(launch_scan_i32(a.n_sw, ctx->ch_swoff.as<int64_t>(), n_reads, st), "scan launch");
    HIPC(hipMemcpyAsync(tot + 2, ctx->ch_swoff.as<int64_t>() + n_reads, sizeof(int64_t), hipMemcpyDeviceToHost, st),
         "D2H");
    HIPC(hipStreamSynchronize(st), "sync");
    const int64_t T = tot[2];
    if (T > INT32_MAX / 2) return fail(ctx, BWAGPU_E_UNSUPPORTED, "too many seeds to realign");
    if (T) {
      HIPC(ctx->ch_swtasks.ensure(sizeof(bwagpu_align2_task_t) * (size_t)T), "hipMalloc");
      HIPC(ctx->ch_swt.ensure((size_t)kSwWin * (size_t)T), "hipMalloc");
      HIPC(ctx->ch_swskip.ensure(sizeof(int32_t) * (size_t)T), "hipMalloc");
      HIPC(ctx->ch_swres.ensure(sizeof(bwagpu_kswr_t) * (size_t)T), "hipMalloc");
      HIPC(ctx->ch_swscr.ensure(8 * ((size_t)kSwWin * (size_t)T + (size_t)T)), "hipMalloc");
      ChainSw sw{ctx->ch_swoff.as<int64_t>(), ctx->ch_swtasks.as<bwagpu_align2_task_t>(), ctx->ch_swt.as<uint8_t>(),
                 ctx->ch_swskip.as<int32_t>(), ctx->ch_swres.as<bwagpu_kswr_t>()};
      HIPC(launch_chain_sw_prep(a, sw, st), "chain_sw_prep launch");
      if ((rc = bwagpu_align2_device(ctx, (int32_t)T, sw.tasks, sa.seq, sw.tpool, ctx->ch_swres.as<bwagpu_kswr_t>(),
                                     ctx->ch_swscr.p, st)))
        return rc;
      HIPC(launch_chain_sw_apply(a, sw, st), "chain_sw_apply launch");
    }
  }
  HIPC(ctx->ch_ocoff.ensure(sizeof(int64_t) * (nr + 1)), "hipMalloc");
  HIPC(ctx->ch_osoff.ensure(sizeof(int64_t) * (nr + 1)), "hipMalloc");
  HIPC(launch_scan_i32(a.n_out, ctx->ch_ocoff.as<int64_t>(), n_reads, st), "scan launch");
  HIPC(launch_scan_i32(a.n_oseed, ctx->ch_osoff.as<int64_t>(), n_reads, st), "scan launch");
  HIPC(hipMemcpyAsync(tot + 3, ctx->ch_ocoff.as<int64_t>() + n_reads, sizeof(int64_t), hipMemcpyDeviceToHost, st),
       "D2H");
  HIPC(hipMemcpyAsync(tot + 4, ctx->ch_osoff.as<int64_t>() + n_reads, sizeof(int64_t), hipMemcpyDeviceToHost, st),
       "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  const int64_t nc = tot[3], ns = tot[4];
  if (nc > INT32_MAX - 1 || ns > INT32_MAX - 1) return fail(ctx, BWAGPU_E_UNSUPPORTED, "batch has too many chains");
  HIPC(ctx->ch_rco.ensure(sizeof(int32_t) * (nr + 1)), "hipMalloc");
  HIPC(ctx->ch_cso.ensure(sizeof(int32_t) * ((size_t)nc + 1)), "hipMalloc");
  HIPC(ctx->ch_rid.ensure(sizeof(int32_t) * (size_t)std::max<int64_t>(nc, 1)), "hipMalloc");
  HIPC(ctx->ch_cfrac.ensure(sizeof(float) * (size_t)std::max<int64_t>(nc, 1)), "hipMalloc");
  HIPC(ctx->ch_out.ensure(sizeof(bwagpu_chain_t) * (size_t)std::max<int64_t>(nc, 1)), "hipMalloc");
  HIPC(ctx->ch_seeds.ensure(sizeof(bwagpu_seed_t) * (size_t)std::max<int64_t>(ns, 1)), "hipMalloc");
  ChainPack pk{ctx->ch_ocoff.as<int64_t>(), ctx->ch_osoff.as<int64_t>(), ctx->ch_rco.as<int32_t>(),
               ctx->ch_cso.as<int32_t>(), ctx->ch_rid.as<int32_t>(), ctx->ch_cfrac.as<float>(),
               ctx->ch_out.as<bwagpu_chain_t>(), ctx->ch_seeds.as<bwagpu_seed_t>()};
  if (to_host) {  // bwagpu_seqs2chains: the chains written over PCIe into its pinned results (no D2H step)
    HIPC(ctx->chh_rco.ensure(sizeof(int32_t) * (nr + 1)), "hipHostMalloc");
    HIPC(ctx->chh_cso.ensure(sizeof(int32_t) * ((size_t)nc + 1)), "hipHostMalloc");
    HIPC(ctx->chh_chains.ensure(sizeof(bwagpu_chain_t) * (size_t)std::max<int64_t>(nc, 1)), "hipHostMalloc");
    HIPC(ctx->chh_seeds.ensure(sizeof(bwagpu_seed_t) * (size_t)std::max<int64_t>(ns, 1)), "hipHostMalloc");
    HIPC(hipHostGetDevicePointer((void**)&pk.read_chain_off, ctx->chh_rco.p, 0), "hipHostGetDevicePointer");
    HIPC(hipHostGetDevicePointer((void**)&pk.chain_seed_off, ctx->chh_cso.p, 0), "hipHostGetDevicePointer");
    HIPC(hipHostGetDevicePointer((void**)&pk.chains, ctx->chh_chains.p, 0), "hipHostGetDevicePointer");
    HIPC(hipHostGetDevicePointer((void**)&pk.seeds, ctx->chh_seeds.p, 0), "hipHostGetDevicePointer");
  }
  HIPC(launch_chain_pack(a, pk, st), "chain_pack launch");
  *n_chains = nc;
  *n_seeds = ns;
  return BWAGPU_OK;
}

}  // namespace

extern "C" int bwagpu_set_alt(bwagpu_ctx_t* ctx, const uint8_t* is_alt) {
  if (!ctx) return BWAGPU_E_INVAL;
  if (!is_alt) {
    ctx->has_alt = false;
    return BWAGPU_OK;
  }
  HIPC(hipSetDevice(ctx->device), "hipSetDevice");
  HIPC(ctx->ch_alt.ensure((size_t)std::max(ctx->ref.n_seqs, 1)), "hipMalloc");
  HIPC(hipMemcpy(ctx->ch_alt.p, is_alt, (size_t)ctx->ref.n_seqs, hipMemcpyHostToDevice), "H2D");
  ctx->has_alt = true;
  return BWAGPU_OK;
}

extern "C" int bwagpu_seqs2chains(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* sopt, const bwagpu_chainopt_t* copt,
                                  int32_t n_reads, const int64_t* seq_off, const uint8_t* seq, int32_t raw,
                                  bwagpu_chains_t* out) {
  if (!ctx || !sopt || !copt || !out || n_reads < 0 || (n_reads && !seq_off)) return BWAGPU_E_INVAL;
  *out = bwagpu_chains_t{};
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int64_t nc = 0, ns = 0;
  int lq = 0;
  int rc = run_chaining(ctx, sopt, copt, n_reads, seq_off, seq, raw != 0, st, &nc, &ns, &lq, true);
  if (rc) return rc;
  const size_t nr = (size_t)n_reads;
  HIPC(ctx->chh_rco.ensure(sizeof(int32_t) * (nr + 1)), "hipHostMalloc");
  HIPC(ctx->chh_cso.ensure(sizeof(int32_t) * ((size_t)nc + 1)), "hipHostMalloc");
  HIPC(ctx->chh_chains.ensure(sizeof(bwagpu_chain_t) * (size_t)std::max<int64_t>(nc, 1)), "hipHostMalloc");
  HIPC(ctx->chh_seeds.ensure(sizeof(bwagpu_seed_t) * (size_t)std::max<int64_t>(ns, 1)), "hipHostMalloc");
  if (n_reads) {
    HIPC(hipStreamSynchronize(st), "sync");  // chain_pack wrote the results into the pinned buffers
  } else {
    ctx->chh_rco.as<int32_t>()[0] = 0;
    ctx->chh_cso.as<int32_t>()[0] = 0;
  }
  out->n_reads = n_reads;
  out->n_chains = (int32_t)nc;
  out->n_seeds = ns;
  out->read_chain_off = ctx->chh_rco.as<int32_t>();
  out->chain_seed_off = ctx->chh_cso.as<int32_t>();
  out->chains = ctx->chh_chains.as<bwagpu_chain_t>();
  out->seeds = ctx->chh_seeds.as<bwagpu_seed_t>();
  return BWAGPU_OK;
}

extern "C" int bwagpu_seqs2regions(bwagpu_ctx_t* ctx, const bwagpu_seedopt_t* sopt, const bwagpu_chainopt_t* copt,
                                   int32_t n_reads, const int64_t* seq_off, const uint8_t* seq, int32_t* out_n,
                                   const bwagpu_alnreg_t** regs, int64_t* n_regs) {
  if (!ctx || !sopt || !copt || !regs || !n_regs || n_reads < 0 || (n_reads && (!seq_off || !out_n)))
    return BWAGPU_E_INVAL;
  *regs = nullptr;
  *n_regs = 0;
  for (int32_t r = 0; r < n_reads; ++r)
    if (seq_off[r + 1] - seq_off[r] > BWAGPU_MAX_READ_LEN)
      return fail(ctx, BWAGPU_E_UNSUPPORTED, "read longer than BWAGPU_MAX_READ_LEN");
  hipStream_t st = nullptr;
  HIPC(lazy_stream(ctx->slot[0], &st), "hipStreamCreate");
  int64_t nc = 0, ns = 0;
  int lq = 0;
  int rc = run_chaining(ctx, sopt, copt, n_reads, seq_off, seq, false, st, &nc, &ns, &lq);
  if (rc) return rc;
  if (n_reads == 0) return BWAGPU_OK;
  if ((rc = check_lds(ctx, lq))) return rc;
  Slot& s = ctx->ch_slot;
  const size_t nr = (size_t)n_reads;
  HIPC(s.d_out.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max<int64_t>(ns, 1)), "hipMalloc(out)");
  HIPC(s.d_n.ensure(sizeof(int32_t) * nr), "hipMalloc(out_n)");
  HIPC(s.d_stats.ensure(sizeof(int64_t) * ST_N), "hipMalloc(stats)");
  HIPC(hipMemsetAsync(s.d_stats.p, 0, sizeof(int64_t) * ST_N, st), "memset stats");
  DevBatch db;
  db.n_reads = n_reads;
  db.n_chains = (int32_t)nc;
  db.n_seeds = (int32_t)ns;
  db.seq_off = ctx->sd_off.as<int64_t>();
  db.seq = ctx->sd_seq.as<uint8_t>();
  db.read_chain_off = ctx->ch_rco.as<int32_t>();
  db.chain_seed_off = ctx->ch_cso.as<int32_t>();
  db.chain_rid = ctx->ch_rid.as<int32_t>();
  db.chain_frac_rep = ctx->ch_cfrac.as<float>();
  db.seeds = ctx->ch_seeds.as<bwagpu_seed_t>();
  if ((rc = enqueue_chain2aln(ctx, s, db, lq, s.d_out.as<bwagpu_alnreg_t>(), s.d_n.as<int32_t>(),
                              s.d_stats.as<int64_t>(), st)))
    return rc;
  HIPC(ctx->ch_regoff.ensure(sizeof(int64_t) * (nr + 1)), "hipMalloc");
  HIPC(launch_scan_i32(s.d_n.as<int32_t>(), ctx->ch_regoff.as<int64_t>(), n_reads, st), "scan launch");
  int64_t* tot = ctx->chh_tot.as<int64_t>();
  HIPC(hipMemcpyAsync(tot + 5, ctx->ch_regoff.as<int64_t>() + n_reads, sizeof(int64_t), hipMemcpyDeviceToHost, st),
       "D2H");
  HIPC(hipMemcpyAsync(tot + 6, s.d_stats.as<int64_t>() + ST_ERR, sizeof(int64_t), hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipMemcpyAsync(out_n, s.d_n.p, sizeof(int32_t) * nr, hipMemcpyDeviceToHost, st), "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  const int64_t nreg = tot[5];
  HIPC(ctx->ch_regc.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max<int64_t>(nreg, 1)), "hipMalloc");
  HIPC(ctx->chh_regs.ensure(sizeof(bwagpu_alnreg_t) * (size_t)std::max<int64_t>(nreg, 1)), "hipHostMalloc");
  HIPC(launch_reg_compact(n_reads, db.read_chain_off, db.chain_seed_off, s.d_out.as<bwagpu_alnreg_t>(),
                          ctx->ch_regoff.as<int64_t>(), ctx->ch_regc.as<bwagpu_alnreg_t>(), st),
       "reg_compact launch");
  if (nreg)
    HIPC(hipMemcpyAsync(ctx->chh_regs.p, ctx->ch_regc.p, sizeof(bwagpu_alnreg_t) * (size_t)nreg, hipMemcpyDeviceToHost,
                        st),
         "D2H");
  HIPC(hipStreamSynchronize(st), "sync");
  *regs = ctx->chh_regs.as<const bwagpu_alnreg_t>();
  *n_regs = nreg;
  if (tot[6] & ERR_LEN) return fail(ctx, BWAGPU_E_UNSUPPORTED, "read longer than BWAGPU_MAX_READ_LEN");
  if (tot[6] & ERR_RID)
    return fail(ctx, BWAGPU_E_RESULTS, "a chain's first seed is not inside contig chain_rid (bwamem.c:669 assert)");
  return BWAGPU_OK;
}
