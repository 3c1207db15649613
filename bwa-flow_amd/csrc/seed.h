// seed.h — internal declarations of the seeding kernels (seed.hip) shared
// with the C ABI (capi.hip).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bwagpu.h"

namespace bwagpu {

// the resident FM-index (bwt_t, bwa/bwt.h:46-57)
struct DevBwt {
  uint64_t primary;
  uint64_t L2[5];
  uint64_t seq_len;
  const uint32_t* bwt;   // bwa's layout (bwt.h:46-57): 128-base blocks of 4 uint64 counts + 8 words of 2-bit bases
  const uint4* occ;      // the device layout (build_occ64): 64-base blocks of 32 B, see seed.hip
  const uint64_t* sup;   // its 64-bit counts per 2^sup_shift positions: 4 per superblock
  int sup_shift;         // log2 of the superblock size: 32 (a test build of the index may use less, >= 7)
  const uint64_t* sa;    // sampled suffix array (NULL if not uploaded)
  uint64_t sa_mask;      // sa_intv - 1
  int sa_shift;          // log2(sa_intv)
  // the whole suffix array, one entry per row 0..seq_len, expanded from the
  // sample on the device (bwagpu_set_bwt) when it fits the budget: 32-bit
  // entries while seq_len < 2^32, else 64-bit; both NULL: the sampled walk
  const uint32_t* sa_full32;
  const uint64_t* sa_full64;
};

// the device occurrence layout of a BWT of seq_len positions ($ removed):
// blocks of 64 positions (2 x uint4 each) and one 4 x uint64 superblock
// record per 2^shift positions (32 in production; bwagpu_debug_sup_shift
// lowers it so that small test indexes cross superblock boundaries)
inline uint64_t occ64_blocks(uint64_t seq_len) { return (seq_len + 63) / 64 + 1; }
inline uint64_t occ64_supers(uint64_t seq_len, int shift) { return (seq_len >> shift) + 2; }
// builds b.occ / b.sup from b.bwt (every other field of b set)
hipError_t launch_build_occ64(const DevBwt& b, uint4* occ, uint64_t* sup, hipStream_t st);

struct SeedArgs {
  int32_t n_reads;
  const int64_t* seq_off;
  const uint8_t* seq;
  int32_t max_per_read;
  bwagpu_intv_t* out;       // n_reads * max_per_read
  int32_t* out_n;           // n_reads
  bwagpu_intv_t* scratch;   // read r: 4 lists of len_r + 2 at 4 * (seq_off[r] + 2r)
  int32_t min_seed_len, split_width, max_mem_intv, split_len;
  int32_t budget;     // bwt_extend calls tier 1 spends on one read before handing it to tier 2
  int32_t* heavy;     // n_reads: the reads handed over
  int32_t* n_heavy;   // their number
  int32_t* flags;     // n_reads: 1 = handed to tier 2
  int32_t* p3_n;      // n_reads: LAST-like intervals in the read's fourth list
  int64_t* dbg;       // NULL, or 4 per tier-1 lane: {extensions, steps, start, end} (wall_clock64)
};

// lists a read needs in the scratch buffer: 4 * (bases + 2 * reads) entries
inline int64_t seed_scratch_entries(int64_t bases, int32_t n_reads) { return 4 * (bases + 2 * (int64_t)n_reads); }

hipError_t launch_collect_intv(const DevBwt& b, const SeedArgs& a, hipStream_t st);
// bwt_sa for n positions
hipError_t launch_bwt_sa(const DevBwt& b, int64_t n, const uint64_t* k, uint64_t* out, hipStream_t st);
// every row's suffix array entry from the sample (b.sa set): o32 or o64 (one of them), seq_len + 1 entries
hipError_t launch_sa_expand(const DevBwt& b, uint32_t* o32, uint64_t* o64, hipStream_t st);
// packs the per-read slots: read r's out_n[r] intervals to dst + off[r]
hipError_t launch_pack_intv(const SeedArgs& a, const int64_t* off, bwagpu_intv_t* dst, hipStream_t st);

}  // namespace bwagpu
