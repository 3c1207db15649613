// host_stage_mock.cpp — the drop-in stage's HOST side with the device taken
// out (a development tool, never shipped): stage_bench.cpp + GPUPipeline.cpp
// linked against this file instead of libbwagpu.so / libamdhip64.so.  The
// bwagpu_* entries GPUPipeline calls keep their contracts (a pinned-buffer
// view from _stage, a refused batch stays on its slot, results valid until the
// next _submit) but do no device work: _submit remembers which registered
// batch was staged (by its sizes) and _results_dense hands back that batch's
// regions, registered beforehand (mock_register).  What gpustage_run then
// measures is the host work of ChainsToRegionsGPU alone — pack, the malloc'd
// mem_alnreg_v, the chain frees, the sink — i.e. the ceiling the host puts on
// bench.py's end_to_end leg, on however many cores this machine has.
//
//   g++ -O2 -fPIC -shared -std=c++17 -I../../include -I../../bwa-flow_amd/host -I/opt/rocm/include
//       -D__HIP_PLATFORM_AMD__ host_stage_mock.cpp ../../bwa-flow_amd/host/stage_bench.cpp
//       ../../bwa-flow_amd/host/GPUPipeline.cpp -o libgpustage_mock.so -lpthread
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "bwagpu.h"

extern "C" {
// ---- the HIP calls GPUEnv makes (host memory stands in for the device's)
hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipMalloc(void** p, size_t n) {
  *p = malloc(n ? n : 1);
  return *p ? hipSuccess : hipErrorOutOfMemory;
}
hipError_t hipFree(void* p) {
  free(p);
  return hipSuccess;
}
hipError_t hipMemcpy(void* d, const void* s, size_t n, hipMemcpyKind) {
  memcpy(d, s, n);
  return hipSuccess;
}
hipError_t hipStreamCreate(hipStream_t* s) {
  *s = nullptr;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t) { return hipSuccess; }
hipError_t hipStreamDestroy(hipStream_t) { return hipSuccess; }
}

namespace {
struct Reg {
  int32_t n_reads, n_chains, n_seeds;
  std::vector<bwagpu_alnreg_t> dense;
  std::vector<int32_t> n, off;
};
std::vector<Reg> g_regs;

struct MSlot {
  std::vector<char> in;
  bool busy = false, has = false;
  int which = -1;
};
}  // namespace

struct bwagpu_ctx {
  MSlot slot[BWAGPU_NUM_SLOTS];
};

extern "C" {
// regions of one batch (dense: read r's at regs[off[r]], n[r] of them)
int mock_register(int32_t n_reads, int32_t n_chains, int32_t n_seeds, const bwagpu_alnreg_t* regs,
                  const int32_t* n) {
  Reg r;
  r.n_reads = n_reads;
  r.n_chains = n_chains;
  r.n_seeds = n_seeds;
  r.n.assign(n, n + n_reads);
  r.off.assign((size_t)n_reads + 1, 0);
  for (int i = 0; i < n_reads; ++i) r.off[i + 1] = r.off[i] + n[i];
  r.dense.assign(regs, regs + r.off[n_reads]);
  g_regs.push_back(std::move(r));
  return (int)g_regs.size() - 1;
}
void mock_clear() { g_regs.clear(); }

int bwagpu_device_count(int* n) {
  *n = 1;
  return BWAGPU_OK;
}
int bwagpu_create_resident(int, const bwagpu_opt_t*, const bwagpu_bns_t*, const void*, bwagpu_ctx_t** out) {
  *out = new bwagpu_ctx;
  return BWAGPU_OK;
}
int bwagpu_destroy(bwagpu_ctx_t* c) {
  delete c;
  return BWAGPU_OK;
}
int bwagpu_set_watchdog_ms(bwagpu_ctx_t*, int) { return BWAGPU_OK; }
const char* bwagpu_last_error(const bwagpu_ctx_t*) { return "mock"; }

int bwagpu_chain2aln_stage(bwagpu_ctx_t* ctx, int slot, int32_t n_reads, int32_t n_chains, int32_t n_seeds,
                           int64_t seq_bytes, bwagpu_batch_t* view) {
  MSlot& s = ctx->slot[slot];
  if (s.busy) return BWAGPU_E_INVAL;
  auto r256 = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t a = r256(8 * ((size_t)n_reads + 1)), b = r256(4 * ((size_t)n_reads + 1)),
               c = r256(4 * ((size_t)n_chains + 1)), d = r256(4 * (size_t)n_chains), e = r256(4 * (size_t)n_chains),
               f = r256(sizeof(bwagpu_seed_t) * (size_t)n_seeds), g = r256((size_t)seq_bytes);
  if (s.in.size() < a + b + c + d + e + f + g) s.in.resize(a + b + c + d + e + f + g);
  char* h = s.in.data();
  view->n_reads = n_reads;
  view->n_chains = n_chains;
  view->n_seeds = n_seeds;
  view->seq_bytes = seq_bytes;
  view->seq_off = (const int64_t*)h;
  view->read_chain_off = (const int32_t*)(h + a);
  view->chain_seed_off = (const int32_t*)(h + a + b);
  view->chain_rid = (const int32_t*)(h + a + b + c);
  view->chain_frac_rep = (const float*)(h + a + b + c + d);
  view->seeds = (const bwagpu_seed_t*)(h + a + b + c + d + e);
  view->seq = (const uint8_t*)(h + a + b + c + d + e + f);
  return BWAGPU_OK;
}

int bwagpu_chain2aln_submit(bwagpu_ctx_t* ctx, int slot, const bwagpu_batch_t* b) {
  MSlot& s = ctx->slot[slot];
  if (s.busy) return BWAGPU_E_INVAL;
  s.has = false;
  s.which = -1;
  for (size_t k = 0; k < g_regs.size(); ++k)
    if (g_regs[k].n_reads == b->n_reads && g_regs[k].n_chains == b->n_chains && g_regs[k].n_seeds == b->n_seeds)
      s.which = (int)k;
  if (s.which < 0) return BWAGPU_E_INVAL;
  s.busy = true;
  return BWAGPU_OK;
}

int bwagpu_chain2aln_wait(bwagpu_ctx_t* ctx, int slot, bwagpu_alnreg_t*, int32_t*) {
  MSlot& s = ctx->slot[slot];
  if (!s.busy) return BWAGPU_E_INVAL;
  s.busy = false;
  s.has = true;
  return BWAGPU_OK;
}

int bwagpu_chain2aln_results_dense(bwagpu_ctx_t* ctx, int slot, const bwagpu_alnreg_t** regs, const int32_t** n,
                                   const int32_t** off) {
  MSlot& s = ctx->slot[slot];
  if (!s.has) return BWAGPU_E_INVAL;
  const Reg& r = g_regs[(size_t)s.which];
  *regs = r.dense.data();
  *n = r.n.data();
  *off = r.off.data();
  return BWAGPU_OK;
}

int bwagpu_last_stats(const bwagpu_ctx_t*, int, bwagpu_stats_t* st) {
  memset(st, 0, sizeof *st);
  return BWAGPU_OK;
}
}
