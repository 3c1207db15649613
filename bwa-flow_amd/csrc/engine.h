// engine.h — shared declarations between the HIP kernels (sw_kernels.hip) and
// the C-ABI implementation (capi.hip).  Internal; not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bwagpu.h"
#include "bwagpu_debug.h"

namespace bwagpu {

// Scoring parameters in the form the kernels use (from bwagpu_opt_t).
struct DevOpt {
  int a, o_del, e_del, o_ins, e_ins, oe_del, oe_ins;
  int pen_clip5, pen_clip3, w, zdrop, max_mat;
  int row_bound;  // extend_quad ends a call once no later row can change its outputs
  int8_t mat[28];
  // query profile words: qprof[q] byte t = mat[t*5 + q] (t = target base 0..3),
  // qprof4[q] = mat[20 + q] (target N; only bare task lists can hold one —
  // targets fetched from the pac are 0..3).  Kernel arguments, so the DP picks
  // its scores with register selects instead of loads.
  uint32_t qprof[5];
  int32_t qprof4[5];
};

// One read in processing order (chain2aln_fast_kernel), written after the sort.
struct ReadDesc {
  int64_t qoff;    // first base in seq
  int32_t rd;      // read index
  int32_t lq;      // read length
  int32_t c0;      // first chain
  int32_t nch;     // chains
  int32_t s0;      // first seed slot (= first output slot)
  int32_t ns;      // seeds over all chains
};

// Per-chain window computed by the prep kernel: [lo, hi) in the 2-strand
// coordinate space, already clipped like bns_fetch_seq (bntseq.c:421-446).
struct ChainWin {
  int64_t lo, hi;
};

// Device views of one flattened batch (pointers are device pointers).
struct DevBatch {
  int32_t n_reads, n_chains, n_seeds;
  const int64_t* seq_off;
  const uint8_t* seq;
  const int32_t* read_chain_off;
  const int32_t* chain_seed_off;
  const int32_t* chain_rid;
  const float* chain_frac_rep;
  const bwagpu_seed_t* seeds;
};

struct DevRef {
  int64_t l_pac;
  int32_t n_seqs;
  const uint8_t* pac;
  const int64_t* ann_offset;
  const int32_t* ann_len;
};

// stats words (int64): [0] cells [1] rows [2] ext calls [3] error flags
enum { ST_CELLS = 0, ST_ROWS = 1, ST_CALLS = 2, ST_ERR = 3, ST_N = 4 };
enum { ERR_RID = 1, ERR_LEN = 2 };

// Kernel variants: G lanes per read ("group"), C = max DP columns per lane.
// A read of length l needs G*C >= l (+1 column for eh[qlen], qlen <= l-1).
enum { VK_FAST = 0, VK_GENERIC = 1 };
struct Variant {
  int G, C;
  int kind;  // VK_FAST: chain2aln_fast_kernel (wave per read), VK_GENERIC: chain2aln_kernel
  __host__ __device__ int max_len() const { return G * C; }
};
// limits of the fast kernel: one lane (slot) per seed / chain / region of a read
constexpr int kFastMaxSeeds = 32;
constexpr int kFastMaxChains = 32;
constexpr int kSeqLds = 256;  // LDS bytes for the read's bases (fast variants: lq <= 256)
constexpr int kNumVariants = 3;
extern const Variant kVariants[kNumVariants];
// bare ksw_extend2 task lists (bwagpu_extend_batch): wave kernels by columns
constexpr int kNumExtVariants = 3;
extern const Variant kExtVariants[kNumExtVariants];
// read-order counters: [0..15] per-variant counts, [16 + 8v + xcc] queue heads
// (generic kernel), [kHistOff ..) the read-order histogram
constexpr int kHistOff = 128;
constexpr int kCountWords = kHistOff + kNumVariants * 256;
constexpr int kBlock = 256;  // threads per workgroup (4 waves)

// host-side launchers (sw_kernels.hip)
hipError_t launch_chain_prep(const DevOpt& o, const DevRef& ref, const DevBatch& b, ChainWin* win, uint64_t* srt,
                             bwagpu_seed_t* prog, int64_t* stats, hipStream_t st);
// read order for the wave kernels: counting sort by [variant | cost] that
// writes read_list[pos] and desc[pos] (bins: n_reads scratch, hist: 3*256
// zeroed counters, counts: per-variant read counts)
hipError_t launch_read_order(const DevBatch& b, int32_t* bins, int32_t* hist, int32_t* counts, ReadDesc* desc,
                             int32_t* list, int64_t* stats, hipStream_t st);
// read_list: reads sorted by key; d_count: per-variant counts (device); the
// variant's reads start at the sum of the lower variants' counts; max_list
// bounds the grid
// everything a chain2aln launch reads/writes besides the batch itself
struct C2AArgs {
  const int32_t* read_list;   // reads in processing order (sorted by key)
  const ReadDesc* desc;       // the same order, as descriptors (fast kernel)
  int32_t* counts;            // [0..15] per-variant counts, [16 + 8v + xcc] queue heads
  const ChainWin* win;        // per chain
  uint64_t* srt;              // per seed, sorted keys (generic kernel)
  const bwagpu_seed_t* prog;  // per seed, processing order, pad_ = 1 for key 0 (fast kernel)
  bwagpu_alnreg_t* out;
  int32_t* out_n;
  int64_t* stats;
};
hipError_t launch_chain2aln(int variant, const DevOpt& o, const DevRef& ref, const DevBatch& b, int32_t max_list,
                            int tb_bytes, const C2AArgs& a, hipStream_t st);
// LDS bytes per wave of chain2aln_fast_kernel for target row buffers of tb bytes
size_t fast_wave_lds(int tb);

hipError_t launch_extend(int variant, bool t5, const DevOpt& o, int32_t n_tasks,
                         const bwagpu_ext_task_t* tasks, const int32_t* task_list, int32_t n_list,
                         const uint8_t* qpool, const uint8_t* tpool, int tb_bytes,
                         bwagpu_ext_result_t* res, int64_t* stats, hipStream_t st);
// four tasks per wave (packed 16-bit DP): h0 > 0, no N in the target rows,
// qlen + 1 <= 256, scores within quad_scores_ok
hipError_t launch_extend4(const DevOpt& o, const bwagpu_ext_task_t* tasks, const int32_t* task_list, int32_t n_list,
                          const uint8_t* qpool, const uint8_t* tpool, int tb_bytes, bwagpu_ext_result_t* res,
                          int64_t* stats, hipStream_t st);

// ---------------------------------------------------------------- speculative path
// mem_chain2aln as (1) extension tasks computed ahead of the sequential
// containment logic and (2) a selection pass that replays that logic with the
// precomputed results (sw_kernels.hip, "speculative chain2aln").
// One seed's extension (bwamem.c:717-792) is a pure function of the seed, the
// read and its chain's window, so it can run before the sequential pass
// decides whether mem_chain2aln performs it.
struct SeedExt {
  int64_t rb, re;
  int32_t qb, qe, score, truesc, w;  // w = max of both sides' final band
  int32_t cells, rows, calls;        // the DP work (counted only if the region is used);
                                     // calls = ksw_extend2 calls + 1, so 0 = not computed
};  // 48 B; the per-batch memset 0 marks every slot "not computed"

// extension task lists: 3 length classes (kernel columns per lane) x 3 rounds
constexpr int kSpecBins = 3;                           // lq <= 160 / <= 256 / <= 1023
// (160: the pair kernel's first bin needs CPL <= 5 = 160 / 32; 2x150 reads all fall in it)
constexpr int kSpecBinLen[kSpecBins] = {160, 256, 1023};
constexpr int kSpecRounds = 3;                         // A, B, C
constexpr int kOrderLane = 8;                          // chains up to this many seeds are ordered by their spec_chain lane
constexpr int kSelLight = 64;                          // reads with more seeds go first
constexpr int kSelRegLds = 256;                        // regions per wave held in LDS
constexpr int kSelMatMaxSeeds = 4096;                  // heavy reads up to this many seeds use pair matrices
// counter words (int32) of one batch (zeroed per batch)
enum {
  SPC_CNT = 0,        // [round*3 + bin] task counts (rounds 0 = A, 1 = B, 2 = C)
  SPC_HEAVY_N = 16,   // reads with > kSelLight seeds
  SPC_SEL_CUR = 17,   // [pass] heavy-read cursors of the emulate / final pass, [2] redo cursor
  SPC_REDO_N = 20,    // reads the final pass could not finish (a missing extension)
  SPC_SPEC64 = 24,    // int64 at words 24-25: DP cells of every computed task (diagnostic)
  SPC_MISS = 26,      // extensions the redo pass computed inline
  SPC_MATW64 = 28,    // int64 at words 28-29: uint64 words of heavy-read pair matrices handed out
  SPC_HCOLS = 30,     // columns (seeds) of heavy reads with a pair matrix
  SPC_LONG_N = 31,    // chains with more than kOrderLane seeds (ordered by spec_order_kernel)
  // words 32-59: the packed kernels' occupancy counters (-DBWAGPU_OCC_DIAG)
  SPC_LCNT = 64,      // [list] phased extension: tasks with a left side (spec_side4_kernel's left list)
  SPC_RCNT = 73,      // [list] ... with a right side
  SPC_LIGHT_CUR = 82, // the final light pass's cursor over the reads without a round-B task
  SPC_WORDS = 128
};
// sharded queue heads of the extension task lists (SpecArgs::qh, zeroed per
// batch): head of (list, xcd) at word (list * 8 + xcd) * kQHStride — one
// 128-byte line each, so claims from different XCDs never meet on a line
// (device-scope atomics on one line serialize at ~88 per microsecond,
// MI355X_MICROARCH.md "dequeue"; measured here: 7.9 -> 6.6 ms per C2 batch
// when the nine lists' heads moved off the two shared lines)
constexpr int kQHStride = 32;
constexpr int kQHWords = 2 * kSpecRounds * kSpecBins * 8 * kQHStride;  // x 2: the phased extension's right lists
// pair-kernel task order (spec_sort_*): 1024 keys = (left qlen / 8, right qlen / 8)
constexpr int kSortKeys = 1024;
// (the phased extension sorts each list twice, by the left and by the right
// side's query length: its second histograms follow at kSortWordsR)
constexpr int kSortWordsR = kSpecRounds * 2 * kSortKeys;
constexpr int kSortWords = 2 * kSortWordsR;
// task list `list` (= round * kSpecBins + bin) starts at this entry of SpecArgs::tasks
__host__ __device__ inline size_t spec_list_off(int list, int n_chains, int n_seeds) {
  const int round = list / kSpecBins, bin = list % kSpecBins;
  return round == 0 ? (size_t)bin * n_chains
                    : (size_t)kSpecBins * n_chains + ((size_t)(round - 1) * kSpecBins + bin) * n_seeds;
}
// An extension task of the first two length bins with everything its start
// needs (spec_sort_scatter writes it beside stasks): the packed kernels read
// one 32-byte record per claimed task instead of the chain list entry -> seed,
// window, owner read -> read offsets (three dependent round trips), and read it
// one generation ahead (spec_ext4_kernel)
struct FatTask {
  int64_t rbeg, qoff;  // the seed's rbeg, its read's first base in DevBatch::seq
  int32_t pos;         // the seed's slot (SeedExt output)
  int32_t dlo, dhi;    // its chain's window: [rbeg - dlo, rbeg + dhi)
  uint32_t qls;        // qbeg | len << 10 | lq << 20 (each <= BWAGPU_MAX_READ_LEN)
};
static_assert(sizeof(FatTask) == 32, "FatTask layout");
static_assert(BWAGPU_MAX_READ_LEN < 1024, "FatTask packs qbeg / len / lq in 10 bits each");
struct SpecArgs {
  int lq_bound;               // reads longer than this set ERR_LEN and are skipped
  ChainWin* win;              // per chain
  int32_t* chain_read;        // per chain
  bwagpu_seed_t* prog;        // per seed, processing order (pad_ = 1: key 0)
  SeedExt* ext;               // per seed slot
  int2* tasks;                // (seed slot, chain) per task, lists at spec_list_off
  int32_t* ctr;               // SPC_* words
  int32_t* regpos;            // per seed slot: region i of a read -> seed slot (LDS overflow)
  int32_t* skipf;             // per seed slot: skip flags of chains > 256 seeds
  int32_t* heavy;             // reads with > kSelLight seeds
  int32_t* redo;              // reads the final pass left to the redo pass
  uint32_t* rbits;            // per read, a bit: the emulate pass left it a round-B task (zeroed per batch)
  ReadDesc* rdesc;            // per read (spec_reads_kernel)
  int32_t* seedchain;         // per seed slot: its chain
  int4* hinfo;                // per heavy-list entry: rd, matrix word offset (-1: none), first column, ns
  int32_t* colent;            // per heavy column: its heavy-list entry
  int32_t* longc;             // chains with more than kOrderLane seeds
  uint64_t* mat;              // heavy-read pair matrices: C[ns][nw] then O[ns][nw] per read
  int64_t mat_words;          // capacity of mat
  int32_t* cov;               // per seed slot: seedcov of its region (heavy reads)
  int32_t* qh;                // kQHWords: sharded queue heads of the extension task lists
  int32_t* sorth;             // kSortWords, zeroed per batch: per (round, bin < 2) key histograms / cursors
  int2* stasks;               // the C = 3 / 4 lists sorted by key (same offsets as tasks), for the pair kernel
  FatTask* ftask;             // the same lists as FatTask records (the packed kernels); the phased
                              // extension: the tasks with a left side, by that side's length
  FatTask* ftaskR;            // the phased extension: the tasks with a right side, by its length
  int risky_first;            // spec_select_light<SEL_FINAL>: reads with a round-B task first (BWAGPU_LIGHT_RISKY_FIRST)
  int emu_strict;             // spec_select_light<SEL_EMULATE>: round-B tasks for uncertain skips too (BWAGPU_EMU_STRICT)
  int ext_prefetch;           // spec_ext4_kernel: claim next tasks a generation ahead while more than
                              // ext_prefetch x 8 x (waves per XCD) remain (0: on demand)
  bwagpu_alnreg_t* out;
  int32_t* out_n;
  int64_t* stats;
};
// a side stream and two events: the heavy-read selection runs beside the light one
struct SpecStreams {
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  // kernel timing (bwagpu_prof_*): event pairs around every C = 3 extension
  // launch, taken from the context's pool while pool_used < pool_n
  hipEvent_t* pool = nullptr;
  int pool_n = 0;
  int* pool_used = nullptr;
  // the context's extension form (bwagpu_ctx_ext_form): 0 = eight / four seeds
  // per wave where the scores fit (default), 1 = two per wave, 2 = four per wave
  int form = 0;
};
// the form new contexts start with (bwagpu_debug_ext_form; process-wide default)
int set_ext_form(int form);
// the first length bin's extension kernel launch_ext_round picks for `form`
// and options `o` with target row buffers of tb_bytes: 8 = eight seeds per
// wave (spec_ext4_kernel<16,10,true>), 4 = four per wave with the 8-bit key
// (<32,5,true>), 5 = four per wave (<32,8,false>), 2 = two per wave
// (spec_ext2_kernel<5>)
int ext_kernel_for(const DevOpt& o, int form, int tb_bytes);
bool quad_scores_ok(const DevOpt& o, int lq);
bool quad_bound_ok(const DevOpt& o, long hb);
bool quad_rows_ok(const DevOpt& o, long rows);
bool quad_key8_ok(const DevOpt& o, int lq);
int ext_form();
hipError_t launch_spec_clear(const SpecArgs& a, int n_reads, int n_seeds, hipStream_t st);
hipError_t launch_spec_chain2aln(const DevOpt& o, const DevRef& ref, const DevBatch& b, const SpecArgs& a,
                                 int tb_bytes, int lq_max, hipStream_t st, const SpecStreams& ss);
// LDS bytes per workgroup of the largest spec launch; regions the redo pass
// holds in LDS for target rows of tb_bytes (must stay > 0)
size_t spec_select_lds(int tb_bytes);
// the lane kernel for short extension tasks (spec_extl_kernel): 0 off, 1 before
// the pair kernel, 2 beside it on the side stream; process-wide; returns the
// previous mode (mode < 0: query only)
int spec_redo_cap(int tb_bytes);

// ---------------------------------------------------------------- FPGA wire format
// bwagpu_sw_stream: packReadData's stream (src/fpga/FPGAPipeline.cpp:252-336)
// decoded by one lane per read record, every task one extend_seed.
struct StreamTask {
  bwagpu_seed_t s;  // rbeg, qbeg, len (score unused)
  int64_t lo, hi;   // the chain's window rmax
  int64_t qoff;     // the read's bases in StreamArgs::qpool
  int32_t lq, pad_;
};
// error flags (StreamArgs::ctr[kStrErr])
enum { STR_ERR_RECORD = 1, STR_ERR_TASK = 2, STR_ERR_DUP = 4, STR_ERR_SEED = 8, STR_ERR_BASE = 16 };
// counter words: [bin] task counts, kStrDecoded, kStrMax (max index + 1),
// kStrErr, then the sharded queue heads of the kSpecBins lists
enum { kStrDecoded = 4, kStrMax = 5, kStrErr = 6, kStrHeads = 64 };
constexpr int kStrCtrWords = kStrHeads + kSpecBins * 8 * kQHStride;
struct StreamArgs {
  const int32_t* buf;     // the stream
  const int64_t* rstart;  // first word of each read record (host walk)
  int32_t n_reads, cap;   // records; task capacity
  int64_t l_pac;
  uint8_t* qpool;         // 8 bytes per stream word: record at word p -> bases at 8 p
  StreamTask* tasks;      // [cap]
  int32_t* lists;         // kSpecBins lists of cap entries
  int32_t* seen;          // [cap], zeroed: duplicate task indices
  int32_t* ctr;           // kStrCtrWords, zeroed
  int32_t* out;           // 5 words per task
};
hipError_t launch_sw_stream(const DevOpt& o, const DevRef& ref, const StreamArgs& a, int tb_bytes, hipStream_t st);

// diagnostics: per-read trace buffer (device pointer, 8 x u32 per read; NULL = off)
hipError_t set_trace(void* dev_ptr);
hipError_t set_trace_spec(void* dev_ptr);  // spec.hip's copy of the trace pointer

// rows a task can touch: the band is empty once i - w >= qlen (ksw.c:417-419),
// so rows i <= qlen + w are the most ever read (the last one only to break)
__host__ __device__ inline int band_cap(int qlen, int max_mat, int end_bonus, int o, int e) {
  int l = (int)((double)(qlen * max_mat + end_bonus - o) / e + 1.);
  return l > 1 ? l : 1;
}

}  // namespace bwagpu
