// test_pipeline.cpp — drives the C++ host side (kflow mirror + ChainsToRegionsGPU)
// the way bwa-flow's main.cpp wires stage 4 (main.cpp:320-329, 365), on batch
// files written by tests/test_host_stage.py, and writes the regions back for
// comparison with the golden fixtures.  TEST INFRASTRUCTURE: the CPU stage's
// per-read body is the oracle (oracle/liboracle.so), standing in for bwa's
// mem_chain2aln.
//
// usage: test_pipeline <dir> <mode> <reads_per_record> <cpu_workers>
//   mode cpu        CPU stage only (no accelerator attached)
//   mode accx_none  GPU stage attached with no usable device: its workers
//                   retire at once and every record must come back to the CPU
//   mode gpu        CPU stage + GPU back end (addAccxBckStage, priority 10)
//   mode gpu_only   GPU stage as the sole stage (--disable_sw_cpu)
//   mode gpu_2ctx   the sole stage with TWO contexts on each device (two
//                   workers per GPU sharing one resident reference)
//   mode gpu_hang   CPU stage + GPU back end whose 3rd wait fails as a
//                   watchdog expiry does: in-flight records go to the CPU,
//                   the worker retires, accx dispatch is switched off
//   mode gpu_badrid the sole stage, record 1 holding a chain outside its
//                   contig: the error path (reported, chain skipped), the
//                   device stays in service
// TEST_CHAIN_MODE=free: the GPU stage frees the chains (the CPU stage's
// ownership) instead of forwarding them (the FPGA stage's, the default); the
// consumer frees forwarded chains as RegionsToSam does (Pipeline.cpp:559)
//   mode reaper     no stage: every record's chains go through a ChainReaper
//                   (the GPU stage's background frees) from cpu_workers
//                   threads at once; after drain() the heap must be back to
//                   its size before the records were built
#include <malloc.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "GPUPipeline.h"
#include "cpu_stage.h"
#include "bwagpu_debug.h"  // bwagpu_debug_fail_wait (the hang tests)
#include "oracle.h"

static std::vector<uint8_t> slurp(const std::string& p) {
  FILE* f = fopen(p.c_str(), "rb");
  if (!f) {
    fprintf(stderr, "cannot open %s\n", p.c_str());
    exit(2);
  }
  std::vector<uint8_t> v;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) v.insert(v.end(), buf, buf + k);
  fclose(f);
  return v;
}
template <typename T>
static std::vector<T> load(const std::string& d, const char* name) {
  auto b = slurp(d + "/" + name);
  std::vector<T> v(b.size() / sizeof(T));
  if (!v.empty()) memcpy(v.data(), b.data(), v.size() * sizeof(T));
  return v;
}

int main(int argc, char** argv) {
  if (argc < 5) return 2;
  const std::string dir = argv[1], mode = argv[2];
  const int per_rec = atoi(argv[3]), cpu_workers = atoi(argv[4]);

  bwagpu_opt_t opt;
  auto ob = slurp(dir + "/opt.bin");
  if (ob.size() != sizeof opt) return 3;
  memcpy(&opt, ob.data(), sizeof opt);
  auto lp = load<int64_t>(dir, "l_pac.bin");
  auto ann_off = load<int64_t>(dir, "ann_offset.bin");
  auto ann_len = load<int32_t>(dir, "ann_len.bin");
  auto pac = load<uint8_t>(dir, "pac.bin");
  bwagpu_bns_t bns{};
  bns.l_pac = lp.at(0);
  bns.n_seqs = (int32_t)ann_off.size();
  bns.ann_offset = ann_off.data();
  bns.ann_len = ann_len.data();

  auto seq_off = load<int64_t>(dir, "seq_off.bin");
  auto seq = load<uint8_t>(dir, "seq.bin");
  auto rco = load<int32_t>(dir, "read_chain_off.bin");
  auto cso = load<int32_t>(dir, "chain_seed_off.bin");
  auto rid = load<int32_t>(dir, "chain_rid.bin");
  auto frac = load<float>(dir, "chain_frac_rep.bin");
  auto seeds = load<bwagpu_seed_t>(dir, "seeds.bin");
  const int n_reads = (int)seq_off.size() - 1;

  // ChainsRecords with malloc'd chains/seeds (the stages free them)
  std::vector<bseq1_t> seqs(n_reads > 0 ? n_reads : 1);
  std::vector<ChainsRecord> recs;
  recs.reserve((size_t)(n_reads / std::max(per_rec, 1) + 1));
  const size_t heap0 = mallinfo2().uordblks;
  for (int r = 0; r < n_reads; ++r) {
    memset(&seqs[r], 0, sizeof(bseq1_t));
    seqs[r].l_seq = (int)(seq_off[r + 1] - seq_off[r]);
    seqs[r].id = r;
    seqs[r].seq = (char*)seq.data() + seq_off[r];
  }
  for (int r0 = 0; r0 < n_reads; r0 += per_rec) {
    const int nb = std::min(per_rec, n_reads - r0);
    ChainsRecord rec{};
    rec.start_idx = (uint64_t)r0;
    rec.batch_num = nb;
    rec.seqs = &seqs[r0];
    rec.chains = (mem_chain_v*)malloc(sizeof(mem_chain_v) * nb);
    for (int i = 0; i < nb; ++i) {
      const int r = r0 + i;
      mem_chain_v& cv = rec.chains[i];
      cv.n = cv.m = (size_t)(rco[r + 1] - rco[r]);
      cv.a = (mem_chain_t*)calloc(cv.n ? cv.n : 1, sizeof(mem_chain_t));
      for (size_t j = 0; j < cv.n; ++j) {
        const int c = rco[r] + (int)j;
        mem_chain_t& ch = cv.a[j];
        ch.n = ch.m = cso[c + 1] - cso[c];
        ch.rid = rid[c];
        ch.frac_rep = frac[c];
        ch.seeds = (mem_seed_t*)malloc(sizeof(mem_seed_t) * (ch.n ? ch.n : 1));
        for (int k = 0; k < ch.n; ++k) {
          const bwagpu_seed_t& t = seeds[cso[c] + k];
          ch.seeds[k].rbeg = t.rbeg;
          ch.seeds[k].qbeg = t.qbeg;
          ch.seeds[k].len = t.len;
          ch.seeds[k].score = t.score;
        }
      }
    }
    recs.push_back(rec);
  }

  if (mode == "reaper") {
    const size_t heap1 = mallinfo2().uordblks;
    size_t released = 0;
    {
      ChainReaper reaper;
      const bool held = getenv("TEST_REAPER_HOLD") != nullptr;  // a reaper that has fallen behind
      if (held) reaper.hold(true);
      std::vector<std::thread> th;
      const int t = std::max(cpu_workers, 1);
      for (int k = 0; k < t; ++k)
        th.emplace_back([&, k] {
          for (size_t i = (size_t)k; i < recs.size(); i += (size_t)t) reaper.release(recs[i].chains, recs[i].batch_num);
        });
      for (auto& x : th) x.join();
      if (held) reaper.hold(false);
      reaper.drain();
      released = recs.size();
      const size_t heap2 = mallinfo2().uordblks;
      printf("{\"records\": %zu, \"built_bytes\": %zu, \"left_bytes\": %lld, \"inline_frees\": %d}\n", released,
             heap1 - heap0, (long long)heap2 - (long long)heap0, reaper.inline_frees());
    }  // ~ChainReaper joins its thread
    return 0;
  }

  // CPU body: the oracle over one read (its chains in order, like the loop
  // in ChainsToRegions::compute)
  auto read_fn = [&](int l_seq, const uint8_t* q, const mem_chain_v& cv, mem_alnreg_v* av) {
    FlatBatch fb;
    ChainsRecord one{};
    bseq1_t s{};
    s.l_seq = l_seq;
    s.seq = (char*)q;
    one.batch_num = 1;
    one.seqs = &s;
    one.chains = const_cast<mem_chain_v*>(&cv);
    fb.pack(one);
    if (oracle_chain2aln_batch(&opt, &bns, pac.data(), &fb.c, fb.regs.data(), fb.n.data(), 1, nullptr) != 0) {
      fprintf(stderr, "oracle assertion\n");
      exit(4);
    }
    mem_alnreg_v* v = fb.unpack(1);
    *av = v[0];
    free(v);
  };

  ChainsToRegions cpu_stage(cpu_workers, read_fn);
  GPUEnv* env = nullptr;
  int n_dev = 0;
  const bool sole = mode == "gpu_only" || mode == "gpu_2ctx" || mode == "gpu_badrid" || mode == "gpu_rccl";
  if (mode == "gpu" || sole || mode == "gpu_hang") {
    // gpu_rccl: the reference reaches the device through GPUEnv's RCCL
    // broadcast (forced on a one-rank communicator when there is one device)
    env = new GPUEnv(opt, bns, pac.data(), 8, 10000, mode == "gpu_2ctx" ? 2 : 1, mode == "gpu_rccl" ? 1 : 0);
    n_dev = env->num_devices();
    if (n_dev == 0) {
      fprintf(stderr, "no device: %s\n", env->status().c_str());
      return 5;
    }
    if (mode == "gpu_hang") bwagpu_debug_fail_wait(env->ctx(0), 2, BWAGPU_E_HANG);
  }
  int bad_rid_read = -1;
  if (mode == "gpu_badrid" && recs.size() > 1) {  // the first chain of record 1 that has one
    ChainsRecord& rr = recs[1];
    for (int i = 0; i < rr.batch_num && bad_rid_read < 0; ++i)
      if (rr.chains[i].n) {
        mem_chain_t& ch = rr.chains[i].a[0];
        ch.rid = (ch.rid + 1) % bns.n_seqs;
        bad_rid_read = (int)rr.start_idx + i;
      }
  }
  const char* cm = getenv("TEST_CHAIN_MODE");
  const bool free_mode = cm && std::string(cm) == "free";
  ChainsToRegionsGPU gpu_stage(mode == "accx_none" ? 2 : std::max(n_dev, 1), &cpu_stage, env,
                               free_mode ? ChainOwnership::kFree : ChainOwnership::kForward);
  kestrelFlow::Pipeline pipe(1);
  if (sole) {
    pipe.addStage(0, &gpu_stage);
  } else {
    pipe.addStage(0, &cpu_stage);
    if (mode != "cpu") pipe.addAccxBckStage(0, &gpu_stage, 10.0f);
  }
  pipe.start();
  std::vector<RegionsRecord> outs;
  std::thread consumer([&] {
    auto* q = pipe.output<RegionsRecord>();
    while (outs.size() < recs.size()) {
      RegionsRecord r;
      q->pop(r);
      outs.push_back(r);
    }
  });
  auto* in = pipe.input<ChainsRecord>();
  for (auto& r : recs) in->push(r);
  pipe.closeInput();
  consumer.join();
  pipe.wait();

  std::sort(outs.begin(), outs.end(),
            [](const RegionsRecord& a, const RegionsRecord& b) { return a.start_idx < b.start_idx; });
  FILE* fr = fopen((dir + "/out_regs.bin").c_str(), "wb");
  FILE* fn = fopen((dir + "/out_n.bin").c_str(), "wb");
  int bad = 0, forwarded = 0;
  for (auto& o : outs) {
    if (o.chains != nullptr) {  // forwarded: RegionsToSam's free (Pipeline.cpp:559)
      forwarded++;
      if (free_mode) bad++;  // the stage should have freed them and forwarded NULL
      freeChainsRecordChains(o.chains, o.batch_num);
    }
    for (int i = 0; i < o.batch_num; ++i) {
      const int32_t k = (int32_t)o.alnreg[i].n;
      fwrite(&k, 4, 1, fn);
      if (k) fwrite(o.alnreg[i].a, sizeof(mem_alnreg_t), (size_t)k, fr);
      free(o.alnreg[i].a);
    }
    free(o.alnreg);
  }
  fclose(fr);
  fclose(fn);
  printf("{\"records\": %zu, \"outputs\": %zu, \"on_gpu\": %d, \"gpu_fallback_cpu\": %d, \"devices\": %d, "
         "\"bad_ownership\": %d, \"forwarded\": %d, \"failed\": %d, \"bad_rid_read\": %d, \"w0\": %d, \"w1\": %d, "
         "\"accx_on_at_end\": %d, \"rccl\": %d, \"env\": \"%s\"}\n",
         recs.size(), outs.size(), gpu_stage.records_on_gpu(), gpu_stage.records_on_cpu(), n_dev, bad, forwarded,
         gpu_stage.records_failed(), bad_rid_read, gpu_stage.records_of_worker(0), gpu_stage.records_of_worker(1),
         cpu_stage.useAccx() ? 1 : 0, env && env->used_rccl() ? 1 : 0, env ? env->status().c_str() : "");
  const int failed = gpu_stage.records_failed();
  delete env;
  // a record the device flagged (a chain outside its contig, where bwa itself
  // asserts, bwamem.c:669) was emitted with that chain skipped: the run must
  // not end as a success (error codes)
  return failed > 0 ? 7 : 0;
}
