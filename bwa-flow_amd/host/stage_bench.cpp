// stage_bench.cpp — the drop-in SW stage end to end (lib/libgpustage.so, used
// by bench.py's `end_to_end` leg and tests/test_host_stage.py).
//
// Host ChainsRecords — malloc'd mem_chain_v / mem_chain_t / seeds per read, as
// bwa-flow's SeqsToChains hands them over (src/Pipeline.cpp:110-121) — go
// through a kflow pipeline whose stage 4 is ChainsToRegionsGPU alone
// (--disable_sw_cpu, main.cpp:320-329): FlatBatch::pack -> bwagpu submit (pinned
// staging, H2D, kernels, the regions written densely to pinned memory) -> wait ->
// malloc'd mem_alnreg_v per read; a second stage of sink_workers threads plays
// RegionsToSam: it frees the regions, and the chains when the stage forwards
// them (ChainOwnership::kForward, the FPGA stage's way; kFree: the stage frees them).
// The records are built before the clock starts (that is SeqsToChains' work).
#include <stdlib.h>
#include <string.h>
#include <sys/resource.h>

#include <chrono>
#include <thread>
#include <vector>

#include "GPUPipeline.h"

namespace {

ChainsRecord make_record(const bwagpu_batch_t& b, bseq1_t* seqs, uint64_t start_idx) {
  ChainsRecord rec{};
  rec.start_idx = start_idx;
  rec.batch_num = b.n_reads;
  rec.seqs = seqs;
  rec.chains = (mem_chain_v*)malloc(sizeof(mem_chain_v) * (size_t)(b.n_reads > 0 ? b.n_reads : 1));
  for (int r = 0; r < b.n_reads; ++r) {
    mem_chain_v& cv = rec.chains[r];
    const int c0 = b.read_chain_off[r], c1 = b.read_chain_off[r + 1];
    cv.n = cv.m = (size_t)(c1 - c0);
    cv.a = (mem_chain_t*)calloc(cv.n ? cv.n : 1, sizeof(mem_chain_t));
    for (int c = c0; c < c1; ++c) {
      mem_chain_t& ch = cv.a[c - c0];
      const int s0 = b.chain_seed_off[c], s1 = b.chain_seed_off[c + 1];
      ch.n = ch.m = s1 - s0;
      ch.rid = b.chain_rid[c];
      ch.frac_rep = b.chain_frac_rep[c];
      ch.seeds = (mem_seed_t*)malloc(sizeof(mem_seed_t) * (size_t)(ch.n ? ch.n : 1));
      for (int k = 0; k < ch.n; ++k) {
        ch.seeds[k].rbeg = b.seeds[s0 + k].rbeg;
        ch.seeds[k].qbeg = b.seeds[s0 + k].qbeg;
        ch.seeds[k].len = b.seeds[s0 + k].len;
        ch.seeds[k].score = b.seeds[s0 + k].score;
      }
    }
  }
  return rec;
}

// RegionsToSam's side of the records (src/Pipeline.cpp:547-560): frees the
// chains a record carries (Pipeline.cpp:559) and its regions, on n workers
// like the real stage; keeps the regions of the last rep for the parity check.
class RegionsSink : public kestrelFlow::MapStage<RegionsRecord, int, COMPUTE_DEPTH, COMPUTE_DEPTH> {
 public:
  RegionsSink(int n, ChainOwnership own, int n_batches, int reps, int32_t** out_n, bwagpu_alnreg_t** out_regs)
      : kestrelFlow::MapStage<RegionsRecord, int, COMPUTE_DEPTH, COMPUTE_DEPTH>(n),
        own_(own), n_batches_(n_batches), reps_(reps), out_n_(out_n), out_regs_(out_regs) {}
  int compute(RegionsRecord const& o) override {
    int bad = 0;
    if (own_ == ChainOwnership::kForward) {
      if (o.chains == nullptr && o.batch_num > 0) bad = 1;
      freeChainsRecordChains(o.chains, o.batch_num);
    } else if (o.chains != nullptr) {
      bad = 1;
    }
    const int k = (int)(o.start_idx % (uint64_t)n_batches_);
    const bool keep = o.start_idx / (uint64_t)n_batches_ == (uint64_t)(reps_ - 1) && out_n_ && out_regs_;
    size_t at = 0;
    for (int r = 0; r < o.batch_num; ++r) {
      const size_t m = o.alnreg[r].n;
      if (keep) {
        out_n_[k][r] = (int32_t)m;
        if (m) memcpy(out_regs_[k] + at, o.alnreg[r].a, sizeof(bwagpu_alnreg_t) * m);
        at += m;
      }
      free(o.alnreg[r].a);
    }
    free(o.alnreg);
    return bad;
  }

 private:
  ChainOwnership own_;
  int n_batches_, reps_;
  int32_t** out_n_;
  bwagpu_alnreg_t** out_regs_;
};

}  // namespace

extern "C" {

// Runs reps x n_batches records through the stage on up to max_devices
// devices with per_device stage workers (bwagpu contexts) on each; chain_mode
// 0 = ChainOwnership::kForward (the sink stage frees the chains, as RegionsToSam
// does), 1 = kFree.  times[0] = wall seconds from the first record in to the
// last record out and every chain freed, times[1..4] = the stage's phase
// totals (pack, submit, wait, post; summed over workers), times[5] = records
// on the GPU, times[6] = records the CPU fallback took, times[7] = stage
// workers (contexts) used, times[8..9] = device kernels / H2D + results (HIP
// events, summed over the GPU records), times[10..11] = the process's user /
// system CPU seconds over the timed run (getrusage: every thread's, the sink's
// and the chain frees' included).  The regions of the LAST rep of batch
// k go to out_n[k][r] / out_regs[k] (compact, read order).  Returns 0, or the
// number of records whose chains were not where the mode puts them.  A
// warm-up pass of min(reps, 2) x n_batches records runs first, untimed.
int gpustage_run(const bwagpu_opt_t* opt, const bwagpu_bns_t* bns, const uint8_t* pac, int n_batches,
                 const bwagpu_batch_t* batches, int reps, int max_devices, int per_device, int chain_mode,
                 int sink_workers, double* times, int32_t** out_n, bwagpu_alnreg_t** out_regs) {
  if (!opt || !bns || !pac || n_batches <= 0 || !batches || reps <= 0 || !times || per_device < 1 ||
      chain_mode < 0 || chain_mode > 1 || sink_workers < 1)
    return -1;
  const ChainOwnership own = chain_mode == 0 ? ChainOwnership::kForward : ChainOwnership::kFree;
  GPUEnv env(*opt, *bns, pac, max_devices, 10000, per_device);
  const int n_dev = env.num_devices();
  if (n_dev == 0) return -2;
  // the reads of every batch (shared by its reps: the stage never frees seqs)
  std::vector<std::vector<bseq1_t>> seqs((size_t)n_batches);
  for (int k = 0; k < n_batches; ++k) {
    const bwagpu_batch_t& b = batches[k];
    seqs[k].assign((size_t)(b.n_reads > 0 ? b.n_reads : 1), bseq1_t{});
    for (int r = 0; r < b.n_reads; ++r) {
      seqs[k][r].l_seq = (int)(b.seq_off[r + 1] - b.seq_off[r]);
      seqs[k][r].id = r;
      seqs[k][r].seq = (char*)b.seq + b.seq_off[r];
    }
  }
  // the records are built by several threads, as SeqsToChains' workers make
  // them: each record's chains sit in its builder's glibc arena
  auto build = [&](int n_reps) {
    std::vector<ChainsRecord> recs((size_t)n_reps * n_batches);
    std::vector<std::thread> builders;
    const int nt = 8;
    for (int t = 0; t < nt; ++t)
      builders.emplace_back([&, t] {
        for (size_t i = (size_t)t; i < recs.size(); i += nt) {
          const int k = (int)(i % (size_t)n_batches);
          recs[i] = make_record(batches[k], seqs[k].data(), (uint64_t)i);
        }
      });
    for (auto& b : builders) b.join();
    return recs;
  };
  // one pipeline run over recs; -> records with misplaced chains
  auto run = [&](std::vector<ChainsRecord>& recs, int n_reps, bool keep, double* t) {
    ChainsToRegionsGPU stage(n_dev, nullptr, &env, own);
    RegionsSink sink(sink_workers, own, n_batches, n_reps, keep ? out_n : nullptr, keep ? out_regs : nullptr);
    kestrelFlow::Pipeline pipe(2);
    pipe.addStage(0, &stage);
    pipe.addStage(1, &sink);
    pipe.start();
    int bad = 0;
    std::chrono::steady_clock::time_point t_end;
    std::thread consumer([&] {
      auto* q = pipe.output<int>();
      for (size_t got = 0; got < recs.size(); ++got) {
        int b = 0;
        q->pop(b);
        bad += b;
      }
      t_end = std::chrono::steady_clock::now();
    });
    struct rusage ru0;
    getrusage(RUSAGE_SELF, &ru0);
    const auto t0 = std::chrono::steady_clock::now();
    auto* in = pipe.input<ChainsRecord>();
    for (auto& r : recs) in->push(r);
    pipe.closeInput();
    consumer.join();
    pipe.wait();  // the workers are done, and the last one drained the stage's chain frees
    t_end = std::max(t_end, std::chrono::steady_clock::now());
    struct rusage ru1;
    getrusage(RUSAGE_SELF, &ru1);
    auto secs = [](const timeval& a, const timeval& b) { return (double)(b.tv_sec - a.tv_sec) + 1e-6 * (double)(b.tv_usec - a.tv_usec); };
    if (t) {
      t[10] = secs(ru0.ru_utime, ru1.ru_utime);
      t[11] = secs(ru0.ru_stime, ru1.ru_stime);
      t[0] = std::chrono::duration<double>(t_end - t0).count();
      stage.phase_seconds(t + 1);
      t[5] = stage.records_on_gpu();
      t[6] = stage.records_on_cpu();
      t[7] = n_dev;
      stage.device_seconds(t + 8);
    }
    return bad;
  };
  // a warm-up pass first (not timed): each context's first batches allocate
  // its slot buffers (pinned + device) and choose its side streams, a one-time
  // cost a pipeline over millions of reads does not see per record
  {
    std::vector<ChainsRecord> warm = build(std::min(reps, 2));
    const int wb = run(warm, std::min(reps, 2), false, nullptr);
    if (wb) return wb;
  }
  std::vector<ChainsRecord> recs = build(reps);
  return run(recs, reps, true, times);
}

}  // extern "C"
