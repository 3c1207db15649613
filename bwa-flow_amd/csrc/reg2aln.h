// reg2aln.h — internal declarations of the batched mem_reg2aln CIGAR kernels
// (reg2aln.hip) shared with the C ABI (capi.hip).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bwagpu.h"
#include "engine.h"

namespace bwagpu {

// Query-length buckets: one compiled kernel per strided segment count CD
// (eh[] slots 0..qlen over 64 lanes: qlen + 1 <= 64 * CD)
constexpr int kR2Buckets = 6;
extern const int kR2CD[kR2Buckets];  // {1, 2, 3, 4, 8, 16}
__host__ __device__ inline int r2_bucket_of(int qlen) {
  const int cd = (qlen + 64) >> 6;
  return cd <= 4 ? cd - 1 : (cd <= 8 ? 4 : 5);
}

struct R2AArgs {
  const bwagpu_reg2aln_task_t* tasks;
  const uint8_t* qpool;
  const int32_t* list;  // job ids of this bin, in processing order
  int n;                // jobs in list
  int max_ops, max_md;
  bwagpu_aln_t* out;
  uint32_t* cigar;
  char* md;
  uint8_t* zglob;   // NULL: direction matrix in LDS; else per-wave HBM slices of zstride bytes
  int64_t zstride;
  int qcap, rcap, ocap;  // per-wave LDS: query bytes, reference bytes, CIGAR-run words
  int lds_per_wave;      // qcap + rcap + 4 ocap (+ the LDS matrix), 16-aligned
  int64_t* stats;        // ST_* words, may be NULL
};

// wpb: waves per workgroup (1 for LDS-heavy bins: finer LDS packing per CU)
int r2_resident_waves(int cd, size_t lds_per_block, int wpb);
hipError_t launch_reg2aln(int cd, const DevOpt& o, const DevRef& ref, const R2AArgs& a, int n_blocks, int wpb,
                          hipStream_t st);

}  // namespace bwagpu
