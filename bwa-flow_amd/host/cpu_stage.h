// cpu_stage.h — the CPU SW stage's shape (src/Pipeline.h:162-171,
// ChainsToRegions::compute src/Pipeline.cpp:503-544) for builds outside
// bwa-flow.  The per-read body (bwa's mem_chain2aln over the read's chains,
// appending to its mem_alnreg_v) is injected: inside bwa-flow it is bwa
// itself; this repository's tests inject the CPU oracle.  No alignment code
// lives here.
#pragma once
#ifndef BWAFLOW_NATIVE_HEADERS
#include <stdint.h>
#include <stdlib.h>

#include <functional>

#include "GPUPipeline.h"

class ChainsToRegions
    : public kestrelFlow::MapStage<ChainsRecord, RegionsRecord, COMPUTE_DEPTH, COMPUTE_DEPTH> {
 public:
  using ReadFn = std::function<void(int l_seq, const uint8_t* seq, const mem_chain_v& chains, mem_alnreg_v* av)>;

  explicit ChainsToRegions(int n, ReadFn fn)
      : kestrelFlow::MapStage<ChainsRecord, RegionsRecord, COMPUTE_DEPTH, COMPUTE_DEPTH>(n), fn_(std::move(fn)) {}

  RegionsRecord compute(ChainsRecord const& record) override {
    mem_alnreg_v* alnreg = (mem_alnreg_v*)malloc(sizeof(mem_alnreg_v) * (size_t)(record.batch_num > 0 ? record.batch_num : 1));
    for (int i = 0; i < record.batch_num; ++i) {
      alnreg[i].n = alnreg[i].m = 0;
      alnreg[i].a = nullptr;
      fn_(record.seqs[i].l_seq, (const uint8_t*)record.seqs[i].seq, record.chains[i], &alnreg[i]);
    }
    freeChainsRecordChains(record.chains, record.batch_num);
    RegionsRecord out;
    out.start_idx = record.start_idx;
    out.batch_num = record.batch_num;
    out.seqs = record.seqs;
    out.chains = nullptr;
    out.alnreg = alnreg;
    return out;
  }

 private:
  ReadFn fn_;
};
#endif
