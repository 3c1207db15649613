// GPUPipeline.h — the GPU back end of bwa-flow's SW stage (stage 4,
// ChainsRecord -> RegionsRecord), in the place of src/fpga/FPGAPipeline.h.
//
//   GPUEnv               ~ BWAOCLEnv (src/fpga/BWAOCLEnv.h:41-114): one
//                          bwagpu context per device, reference resident
//   ChainsToRegionsGPU   ~ ChainsToRegionsFPGA (FPGAPipeline.h:14-31,
//                          FPGAPipeline.cpp:367-579): same base class, same
//                          constructor (n workers = n devices, CPU stage for
//                          fallback), same compute(wid) protocol
//
// Results are bit-identical to ChainsToRegions::compute (src/Pipeline.cpp:
// 503-544); alnreg and every alnreg[i].a are malloc'd (freeAligns,
// bwa_wrapper.cpp:824-830, can free them).  The chains go one of two ways
// (ChainOwnership): forwarded in the output record for RegionsToSam to free
// (Pipeline.cpp:559), as the FPGA stage does (FPGAPipeline.cpp:434), or freed
// here and NULL forwarded, as the CPU stage does (Pipeline.cpp:526-537).
#pragma once
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "bwagpu.h"
#include "records.h"
#ifdef BWAFLOW_NATIVE_HEADERS
#include "kflow/MapPartitionStage.h"  // the reference's kestrelFlow
#else
#include "kflow.h"  // std::thread mirror of it
#endif

#ifndef COMPUTE_DEPTH
#define COMPUTE_DEPTH 64
#endif

class ChainsToRegions;  // the CPU stage (src/Pipeline.h:162-171 / cpu_stage.h)

// The GPU environment (BWAOCLEnv, src/fpga/BWAOCLEnv.h:41-114): the packed
// reference resident ONCE per device — copied host->device to the first
// device and broadcast from there to the others over xGMI with RCCL
// (ncclBroadcast on an ncclCommInitAll communicator; librccl is dlopen'ed, and
// without it every device gets its own host copy) — and `per_device`
// bwagpu contexts per device sharing that copy (bwagpu_create_resident), one
// per stage worker.  Devices that fail to initialise are skipped (their
// workers retire at once, like an FPGA env with fewer PEs).
class GPUEnv {
 public:
  // force_rccl: 1 = broadcast over RCCL even with one device (a one-rank
  // communicator), 0 = only with several, -1 = from BWAGPU_FORCE_RCCL
  GPUEnv(const bwagpu_opt_t& opt, const bwagpu_bns_t& bns, const uint8_t* pac, int max_devices = 8,
         int watchdog_ms = 10000, int per_device = 1, int force_rccl = -1);
  ~GPUEnv();
  GPUEnv(const GPUEnv&) = delete;
  GPUEnv& operator=(const GPUEnv&) = delete;

  // contexts (= stage workers), devices they are on
  int num_devices() const { return (int)ctx_.size(); }
  int num_physical_devices() const { return (int)pac_dev_.size(); }
  bwagpu_ctx_t* ctx(int i) const { return i >= 0 && i < (int)ctx_.size() ? ctx_[i] : nullptr; }
  const std::string& status() const { return status_; }
  bool used_rccl() const { return rccl_; }

 private:
  std::vector<bwagpu_ctx_t*> ctx_;
  std::vector<void*> pac_dev_;  // the resident reference of each device (owned)
  std::vector<int> pac_devid_;
  bool rccl_ = false;
  std::string status_;
};

// A ChainsRecord flattened into the ABI's offset arrays (bwagpu_batch_t).
struct FlatBatch {
  std::vector<int64_t> seq_off;
  std::vector<uint8_t> seq;
  std::vector<int32_t> read_chain_off, chain_seed_off, chain_rid;
  std::vector<float> chain_frac_rep;
  std::vector<bwagpu_seed_t> seeds;
  std::vector<bwagpu_alnreg_t> regs;  // output slots (one per seed)
  std::vector<int32_t> n;             // regions per read
  std::vector<int64_t> seed_base;     // pack_staged: each read's first seed
  bwagpu_batch_t c{};

  void pack(const ChainsRecord& rec);  // ~ packReadData (FPGAPipeline.cpp:194-343)
  // the same, written straight into the slot's pinned DMA buffer
  // (bwagpu_chain2aln_stage): c then points there and _submit copies nothing
  int pack_staged(bwagpu_ctx_t* ctx, int slot, const ChainsRecord& rec);
  // ~ processOutput (FPGAPipeline.cpp:29-130): regions into malloc'd mem_alnreg_v
  mem_alnreg_v* unpack(int batch_num) const;
  // ... and from the dense ones (bwagpu_chain2aln_results_dense: read i's at regs[off[i]])
  static mem_alnreg_v* unpack_dense(const bwagpu_alnreg_t* regs, const int32_t* n, const int32_t* off,
                                    int batch_num);
};

// frees the chains of a record the way ChainsToRegions::compute does
void freeChainsRecordChains(mem_chain_v* chains, int batch_num);

// Background threads that free the records' chains (freeChainsRecordChains),
// so the stage workers do not; with several threads records are freed in no
// particular order.  A record's chains come from
// one SeqsToChains worker's glibc arena; one thread per record keeps a
// record's frees on one arena lock, and several threads free different
// records (different arenas) at once: threads() of them, BWAGPU_REAPER_THREADS
// (default 4).  drain() returns once everything queued is freed.
// BWAGPU_CHAIN_REAPER=0 frees inline on the worker instead.
class ChainReaper {
 public:
  ChainReaper() = default;
  ~ChainReaper();
  ChainReaper(const ChainReaper&) = delete;
  ChainReaper& operator=(const ChainReaper&) = delete;
  void release(mem_chain_v* chains, int batch_num);
  void drain();
  // records freed inline because kMaxQueued were already waiting
  int inline_frees() const { return n_inline_.load(); }
  static constexpr size_t kMaxQueued = 4 * BWAGPU_NUM_SLOTS;
  static int threads();
  // tests: while held the threads free nothing (a reaper that has fallen
  // behind), so releases past kMaxQueued take the inline path
  void hold(bool on);

 private:
  void run();
  std::mutex mu_;
  std::condition_variable cv_, idle_;
  std::deque<std::pair<mem_chain_v*, int>> q_;
  bool stop_ = false, started_ = false, held_ = false;
  int busy_ = 0;
  std::atomic<int> n_inline_{0};
  std::vector<std::thread> th_;
};

// Threads that finish records for the stage workers (BWAGPU_POST_THREADS,
// default 0 = on the worker itself): the malloc'd mem_alnreg_v of a record
// (FlatBatch::unpack_dense), its chains handed on or to the reaper, and the
// push to the next stage — while the worker packs and submits its next record
// into another slot.  A slot is reused only once its record has been posted.
class PostPool {
 public:
  PostPool() = default;
  ~PostPool();
  PostPool(const PostPool&) = delete;
  PostPool& operator=(const PostPool&) = delete;
  void post(std::function<void()> f);
  static int threads();

 private:
  void run();
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<std::function<void()>> q_;
  bool stop_ = false, started_ = false;
  std::vector<std::thread> th_;
};

// Who frees a record's chains once its regions are made.  kFree (the
// default) frees them on the stage's reaper threads; kForward hands them on
// exactly as the FPGA stage does.  Either is correct under RegionsToSam,
// which frees only non-NULL chains (Pipeline.cpp:559).
enum class ChainOwnership {
  kForward,  // the output record carries them; RegionsToSam frees them (Pipeline.cpp:559),
             // as after ChainsToRegionsFPGA (FPGAPipeline.cpp:434)
  kFree,     // freed by the stage (its ChainReaper), chains = NULL forwarded, as after
             // ChainsToRegions::compute (Pipeline.cpp:526-537)
};

class ChainsToRegionsGPU
    : public kestrelFlow::MapPartitionStage<ChainsRecord, RegionsRecord, COMPUTE_DEPTH, COMPUTE_DEPTH> {
 public:
  ChainsToRegionsGPU(int n = 1, ChainsToRegions* stage = nullptr, GPUEnv* env = nullptr,
                     ChainOwnership own = ChainOwnership::kFree)
      : kestrelFlow::MapPartitionStage<ChainsRecord, RegionsRecord, COMPUTE_DEPTH, COMPUTE_DEPTH>(n, false),
        n_active_(n),
        cpu_stage_(stage),
        env_(env),
        own_(own) {}

  void compute(int wid) override;
  ChainOwnership chain_ownership() const { return own_; }

  // counters (tests / logging)
  int records_on_gpu() const { return n_gpu_.load(); }
  int records_on_cpu() const { return n_cpu_.load(); }
  // records the device flagged (BWAGPU_E_RESULTS: a chain outside its contig,
  // where bwa asserts): emitted with that chain skipped, never handed to the CPU stage
  int records_failed() const { return n_failed_.load(); }
  // records each worker took (workers = env contexts)
  int records_of_worker(int wid) const { return wid >= 0 && wid < kMaxWorkers ? per_worker_[wid].load() : 0; }
  static constexpr int kMaxWorkers = 64;
  // host-side phase totals over all workers, seconds (the per-phase prep /
  // enqueue / dequeue / post totals FPGAPipeline.cpp:557-578 prints):
  // [0] pack (ChainsRecord -> flat arrays), [1] submit (pinned staging + H2D +
  // launches), [2] wait (device time not hidden + D2H), [3] post (malloc'd
  // mem_alnreg_v + freeing the chains, or handing them to the reaper; on the
  // PostPool's threads when it has any)
  void phase_seconds(double out[4]) const {
    for (int i = 0; i < 4; ++i) out[i] = (double)ns_[i].load() * 1e-9;
  }
  // device-side totals over the GPU records, seconds (HIP events of each
  // batch, bwagpu_last_stats): [0] kernels, [1] H2D + results to host
  void device_seconds(double out[2]) const {
    for (int i = 0; i < 2; ++i) out[i] = (double)dev_ns_[i].load() * 1e-9;
  }

 private:
  RegionsRecord on_cpu(const ChainsRecord& rec);
  void retire();
  // a finished record's regions -> its RegionsRecord, pushed downstream
  void post_record(int wid, const ChainsRecord& rec, const bwagpu_alnreg_t* rg, const int32_t* nn,
                   const int32_t* off);

  std::atomic<int> n_active_;
  ChainsToRegions* cpu_stage_;
  GPUEnv* env_;
  std::atomic<int> n_gpu_{0}, n_cpu_{0}, n_failed_{0};
  std::atomic<int> per_worker_[kMaxWorkers] = {};
  std::atomic<long long> ns_[4] = {};
  std::atomic<long long> dev_ns_[2] = {};
  ChainOwnership own_;
  ChainReaper reaper_;
  PostPool poster_;
};
