// align2.h — internal declarations of the batched ksw_align2 kernels
// (align2.hip) shared with the C ABI (capi.hip).  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "bwagpu.h"
#include "engine.h"

namespace bwagpu {

// Segment-count buckets: one compiled kernel per (bucket, u8/i16).  A task's
// bucket is that of its first pass (p*ceil(qlen/p) columns over 64 lanes);
// its reverse pass has fewer columns and reuses the same body.
constexpr int kA2Buckets = 8;
extern const int kA2CD[kA2Buckets];  // {1, 2, 3, 4, 6, 8, 12, 16}
constexpr int kA2Bins = 2 * kA2Buckets;  // bins [0, 8): i16, [8, 16): u8

__host__ __device__ inline int a2_bin_of(int qlen, bool u8) {
  const int p = u8 ? 16 : 8;
  const int ncol = (qlen + p - 1) / p * p;
  const int cd = ncol > 64 ? (ncol + 63) / 64 : 1;
  const int b = cd <= 4 ? cd - 1 : cd <= 6 ? 4 : cd <= 8 ? 5 : cd <= 12 ? 6 : 7;
  return (u8 ? kA2Buckets : 0) + b;
}

// Query-profile rows for v_perm_b32: for target base t, the 8-byte pool
// {lo[t], hi[t]} holds the profile byte of query base 0..3 (lo), 4 (hi byte 0)
// and of a padding column (hi byte 1).  u8: (uint8)(mat + shift) and shift
// (ksw_qinit, ksw.c:88-95); i16: mat + 128 and 128 (the bias is removed in-kernel).
struct A2Prof {
  uint32_t lo[5], hi[5];
  int shift;  // u8: ksw_qinit's shift; i16: unused
  int qmax;   // max(mat, 0) (ksw.c:84)
  int e_del, oe_del, e_ins, oe_ins;
};

struct A2Args {
  const bwagpu_align2_task_t* tasks;
  const uint8_t* q;
  const uint8_t* t;
  bwagpu_kswr_t* out;
  int2* bscratch;       // row-maxima entries, task k from boff[k]
  const int64_t* boff;  // [n_tasks]
  const int32_t* list;  // task ids of this bin
  const int32_t* count; // device count of this bin
  int32_t* cursor;      // next unclaimed list index of this bin (zeroed before the launch)
  int64_t* stats;       // ST_* words, may be NULL
};

// one bin's kernel; n_hint = its task count when the host knows it (grid
// sized to it), 0 = unknown (grid = resident capacity, tasks read from *count)
hipError_t launch_align2(int bin, const A2Args& a, const A2Prof& P, int n_hint, hipStream_t st);
// device-side binning (bwagpu_align2_device): lists is [kA2Bins][n]
hipError_t launch_align2_bins(const bwagpu_align2_task_t* tasks, int n, int32_t* lists, int32_t* counts,
                              int64_t* boff, unsigned long long* cursor, bwagpu_kswr_t* out, int64_t* stats,
                              hipStream_t st);

}  // namespace bwagpu
