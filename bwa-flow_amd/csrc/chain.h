// chain.h — internal declarations of the chaining kernels (chain.hip) shared
// with the C ABI (capi.hip).  Not part of the ABI.
//
// The device form of seeding's chaining (bwa-flow SeqsToChains after the
// interval search, src/bwa_wrapper.cpp:105-115): mem_chain's body
// (bwa/bwamem.c:260-330), test_and_merge (199-221), mem_chain_flt (336-396)
// and mem_flt_chained_seeds (607-624).  Data layout in HBM, per batch of
// reads: every read's SA positions (P in all) are laid out back to back in
// interval order at pos_off[r]; the read's chain records, its seed lists and
// its chain-order list share that index space (a read never makes more chains
// than it has positions), and its kbtree nodes sit at node_base(r).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bwagpu.h"
#include "seed.h"

namespace bwagpu {

// kbtree of mem_chain_t at KB_DEFAULT_SIZE 512 (kbtree.h:40-52): t =
// ((512 - 4 - 8) / (8 + sizeof(mem_chain_t) = 40) + 1) >> 1 = 5
constexpr int kBT = 5;
constexpr int kBN = 2 * kBT - 1;  // keys per node

// one kbtree node; keys are read-local chain ids (the chain's pos is its first
// seed's rbeg, read through the id).  16-bit ids in LDS, 32-bit in global memory.
template <class K>
struct BNodeT {
  K n, internal;
  K key[kBN];
  K child[kBN + 1];
};
typedef BNodeT<int16_t> BNode16;
typedef BNodeT<int32_t> BNode32;
static_assert(sizeof(BNode16) == 42 && sizeof(BNode32) == 84, "node layout");

// a chain while its read is chained: mem_chain_t's first and last seed,
// mem_chain_weight's running sums (the weight is built as seeds are appended,
// bwamem.c:223-244), and mem_chain_flt's fields
struct LChain {
  int64_t s0_rbeg, last_rbeg, endr;
  int32_t rid, n;
  int32_t first, soff, cur;
  int16_t s0_qbeg, last_qbeg, last_len, endq;
  int16_t wq, wr, w;  // wr saturates at 32767 (w = min(wq, wr), wq <= the read's length)
  int8_t is_alt, kept;
};
static_assert(sizeof(LChain) == 64, "chain layout");

struct DChain {  // a chain out of mem_chain_flt (its seeds at oslist[soff..soff+n))
  int64_t pos;
  int32_t rid, n, w, kept, first, is_alt, soff, pad_;
};
static_assert(sizeof(DChain) == 40, "out chain layout");

// the read's node arena: nodes <= keys / (t - 1) + 1 <= n_pos / 4 + 1
__host__ __device__ inline int64_t node_base(int64_t pos_off_r, int32_t r) { return (pos_off_r >> 2) + 2 * (int64_t)r; }
__host__ __device__ inline int64_t node_total(int64_t p_total, int32_t n_reads) {
  return (p_total >> 2) + 2 * (int64_t)n_reads + 2;
}

// reads are binned by their SA position count: a read of bin b (b < kLdsBins)
// is chained by one wave with its kbtree, chains and lists in LDS sized for
// kBinCap[b] positions; larger reads use the same code on global memory
constexpr int kLdsBins = 4;
constexpr int kBinCap[kLdsBins] = {32, 128, 512, 1536};
// chains | nodes | the seeds' rbeg (int64) | qbeg/len (int2) | label, slist, ord (int32)
__host__ __device__ constexpr size_t lds_nodes_bytes(int cap) {
  return ((size_t)(cap / 4 + 2) * sizeof(BNode16) + 7) & ~(size_t)7;
}
__host__ __device__ constexpr size_t lds_arena(int cap) {
  return (size_t)cap * sizeof(LChain) + lds_nodes_bytes(cap) + (8 + 8 + 3 * 4) * (size_t)cap;
}
static_assert(lds_arena(1536) <= 160 * 1024, "the largest bin fits one CU's LDS");

struct ChainArgs {
  int32_t n_reads;
  const int64_t* seq_off;
  const uint8_t* seq;
  const bwagpu_intv_t* intv;  // read r's intervals at r * max_per_read
  const int32_t* intv_n;
  int32_t max_per_read;
  // options (bwagpu_chainopt_t + the context's w / a + seeding's min_seed_len)
  int32_t max_occ, max_chain_gap, min_chain_weight, max_chain_extend, min_seed_len, w, a;
  float mask_level, drop_ratio;
  int32_t raw;  // 1: stop after mem_chain (no mem_chain_flt / mem_flt_chained_seeds)
  // reference (bns)
  int64_t l_pac;
  int32_t n_seqs;
  const int64_t* ann_off;
  const int32_t* ann_len;
  const uint8_t* is_alt;  // per contig, or NULL
  const uint8_t* pac;
  const int32_t* sw_tab;  // per read length: min_HSP_score when mem_flt_chained_seeds runs, else -1
  // per read
  int32_t* n_pos;       // SA positions (mem_chain's loop iterations)
  int64_t* pos_off;     // exclusive scan of n_pos, [n_reads + 1]
  float* frac_rep;      // l_rep / len
  int32_t* n_out;       // chains out
  int32_t* n_oseed;     // seeds over the chains out
  int32_t* n_sw;        // mem_seed_sw tasks
  int32_t* need;        // [0]: the largest interval count of an overflowed read
  int32_t* bin_list;    // [kLdsBins + 1][n_reads]
  int32_t* bin_count;   // [kLdsBins + 1]
  // per position, in the read's interval order
  uint64_t* kpos;   // BWT row
  uint64_t* rbeg;   // bwt_sa of it
  int2* qinfo;      // qbeg, len
  int32_t* score;   // seed score (len, or mem_seed_sw's)
  DChain* ochains;  // the read's chains out, in order
  int32_t* oslist;  // their seeds (positions), chain after chain
  // the global-memory arena of reads past the largest bin
  LChain* lchains;
  BNode32* lnodes;
  int32_t* label;
  int32_t* slist;
  int32_t* ord;
  uint64_t* dbg;  // diagnostics (BWAGPU_CHAIN_PHASES=1): per read, s_memrealtime at 8 phase ends
};

struct ChainPack {  // the chains out, in bwagpu_batch_t's layout
  const int64_t* oc_off;  // exclusive scan of n_out
  const int64_t* os_off;  // exclusive scan of n_oseed
  int32_t* read_chain_off;
  int32_t* chain_seed_off;
  int32_t* chain_rid;
  float* chain_frac;
  bwagpu_chain_t* chains;
  bwagpu_seed_t* seeds;
};

struct ChainSw {  // mem_seed_sw as ksw_align2 tasks
  const int64_t* sw_off;  // exclusive scan of n_sw
  bwagpu_align2_task_t* tasks;
  uint8_t* tpool;  // kSwWin bytes per task
  int32_t* skip;   // 1: the seed is not realigned (mem_seed_sw returns -1)
  const bwagpu_kswr_t* res;
};
constexpr int kSwWin = 200;  // MEM_SHORT_LEN: no window reaches it

// exclusive scan of n int32 into out[0..n]
hipError_t launch_scan_i32(const int32_t* in, int64_t* out, int32_t n, hipStream_t st);
hipError_t launch_chain_count(const ChainArgs& a, hipStream_t st);
hipError_t launch_chain_emit(const ChainArgs& a, hipStream_t st);
struct ChainStreams {  // the bins' side streams (fork / join with events)
  hipStream_t side[2];
  hipEvent_t fork, join[2];
};
hipError_t launch_chain_build(const ChainArgs& a, hipStream_t st, const ChainStreams& cs);  // bins, one launch each
hipError_t launch_chain_sw_prep(const ChainArgs& a, const ChainSw& s, hipStream_t st);
hipError_t launch_chain_sw_apply(const ChainArgs& a, const ChainSw& s, hipStream_t st);
hipError_t launch_chain_pack(const ChainArgs& a, const ChainPack& p, hipStream_t st);
// regions of read r at regs + chain_seed_off[read_chain_off[r]] (n[r] of
// them) -> back to back at dst + off[r]
hipError_t launch_reg_compact(int32_t n_reads, const int32_t* rco, const int32_t* cso, const bwagpu_alnreg_t* regs,
                              const int64_t* off, bwagpu_alnreg_t* dst, hipStream_t st);

}  // namespace bwagpu
