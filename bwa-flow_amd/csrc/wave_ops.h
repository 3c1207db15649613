// wave_ops.h — cross-lane primitives of the gfx950 kernels (sw_kernels.hip,
// align2.hip): DPP-fused max/min steps, group reductions and scans, uniform
// helpers.  Internal; included by the .hip translation units only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace bwagpu {

// ---------------------------------------------------------------- group ops
// Cross-lane primitives restricted to one group.  G = 16 is exactly one DPP
// row, so everything is a DPP-modified VALU op (row_shr / row_ror): no LDS
// crossbar round trip on the per-row critical path.  Wider groups fall back to
// ds_bpermute-based shuffles.
constexpr int DPP_ROW_SHR(int n) { return 0x110 + n; }
constexpr int DPP_ROW_ROR(int n) { return 0x120 + n; }

template <int CTRL>
__device__ __forceinline__ int dpp(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, 0xF, 0xF, false);
}

template <int G>
struct Grp {
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & (G - 1)); }
  static __device__ __forceinline__ int gmax(int v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, G));
    return v;
  }
  static __device__ __forceinline__ int gmin(int v) {
#pragma unroll
    for (int o = G / 2; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, G));
    return v;
  }
  // max over lanes strictly below this one; `ident` for lane 0
  static __device__ __forceinline__ int excl_max(int v, int ident) {
    const int l = lane();
#pragma unroll
    for (int o = 1; o < G; o <<= 1) {
      int y = __shfl_up(v, o, G);
      if (l >= o) v = max(v, y);
    }
    int e = __shfl_up(v, 1, G);
    return l == 0 ? ident : e;
  }
  static __device__ __forceinline__ int up1(int v) { return __shfl_up(v, 1, G); }
  static __device__ __forceinline__ int bcast(int v, int src) { return __shfl(v, src, G); }
};

// DPP max/min steps: `x = op(x, x[DPP source lane])` as ONE v_max_i32_dpp.
// Lanes whose source lies outside the row (or whose row is masked off) keep
// x — the identity for a scan or a reduction.  Inline asm, because the
// update_dpp builtin + max is not folded by the backend's DPP combiner here
// (measured: +23 VALU per CD=1 row); the asm carries its own s_nop for the
// VALU-write -> DPP-read hazard.  BWAGPU_BUILTIN_DPP selects the builtin form.
constexpr int DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_max(int x) {
  return max(x, __builtin_amdgcn_update_dpp(x, x, CTRL, RMASK, 0xF, false));
}
template <int CTRL, int RMASK>
__device__ __forceinline__ int dpp_min(int x) {
  return min(x, __builtin_amdgcn_update_dpp(x, x, CTRL, RMASK, 0xF, false));
}
#ifndef BWAGPU_BUILTIN_DPP
#define BWAGPU_DPP(name, op, ctrl, rmask, fn)                                                         \
  __device__ __forceinline__ int name(int x) {                                                        \
    asm volatile("s_nop 1\n\t" op " %0, %0, %0 " ctrl " row_mask:" rmask " bank_mask:0xf" : "+v"(x)); \
    return x;                                                                                         \
  }
#else
#define BWAGPU_DPP(name, op, ctrl, rmask, fn) \
  __device__ __forceinline__ int name(int x) { return fn(x); }
#endif
BWAGPU_DPP(max_shr1, "v_max_i32_dpp", "row_shr:1", "0xf", (dpp_max<DPP_ROW_SHR(1), 0xF>))
BWAGPU_DPP(max_shr2, "v_max_i32_dpp", "row_shr:2", "0xf", (dpp_max<DPP_ROW_SHR(2), 0xF>))
BWAGPU_DPP(max_shr4, "v_max_i32_dpp", "row_shr:4", "0xf", (dpp_max<DPP_ROW_SHR(4), 0xF>))
BWAGPU_DPP(max_shr8, "v_max_i32_dpp", "row_shr:8", "0xf", (dpp_max<DPP_ROW_SHR(8), 0xF>))
BWAGPU_DPP(max_ror8, "v_max_i32_dpp", "row_ror:8", "0xf", (dpp_max<DPP_ROW_ROR(8), 0xF>))
BWAGPU_DPP(max_ror4, "v_max_i32_dpp", "row_ror:4", "0xf", (dpp_max<DPP_ROW_ROR(4), 0xF>))
BWAGPU_DPP(max_ror2, "v_max_i32_dpp", "row_ror:2", "0xf", (dpp_max<DPP_ROW_ROR(2), 0xF>))
BWAGPU_DPP(max_ror1, "v_max_i32_dpp", "row_ror:1", "0xf", (dpp_max<DPP_ROW_ROR(1), 0xF>))
BWAGPU_DPP(min_ror8, "v_min_i32_dpp", "row_ror:8", "0xf", (dpp_min<DPP_ROW_ROR(8), 0xF>))
BWAGPU_DPP(min_ror4, "v_min_i32_dpp", "row_ror:4", "0xf", (dpp_min<DPP_ROW_ROR(4), 0xF>))
BWAGPU_DPP(min_ror2, "v_min_i32_dpp", "row_ror:2", "0xf", (dpp_min<DPP_ROW_ROR(2), 0xF>))
BWAGPU_DPP(min_ror1, "v_min_i32_dpp", "row_ror:1", "0xf", (dpp_min<DPP_ROW_ROR(1), 0xF>))
// cross-row steps: row_bcast:15 feeds lane 15 of rows 0/2 into rows 1/3,
// row_bcast:31 feeds lane 31 into rows 2/3
BWAGPU_DPP(max_bc15, "v_max_i32_dpp", "row_bcast:15", "0xa", (dpp_max<DPP_BCAST15, 0xA>))
BWAGPU_DPP(max_bc31, "v_max_i32_dpp", "row_bcast:31", "0xc", (dpp_max<DPP_BCAST31, 0xC>))
BWAGPU_DPP(min_bc15, "v_min_i32_dpp", "row_bcast:15", "0xa", (dpp_min<DPP_BCAST15, 0xA>))
BWAGPU_DPP(min_bc31, "v_min_i32_dpp", "row_bcast:31", "0xc", (dpp_min<DPP_BCAST31, 0xC>))
#undef BWAGPU_DPP
constexpr int DPP_WAVE_SHR1 = 0x138;

template <>
struct Grp<16> {
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & 15); }
  static __device__ __forceinline__ int gmax(int v) { return max_ror1(max_ror2(max_ror4(max_ror8(v)))); }
  static __device__ __forceinline__ int gmin(int v) { return min_ror1(min_ror2(min_ror4(min_ror8(v)))); }
  // inclusive row scan, then shift by one with `ident` entering lane 0
  static __device__ __forceinline__ int excl_max(int v, int ident) {
    v = max_shr8(max_shr4(max_shr2(max_shr1(v))));
    return dpp<DPP_ROW_SHR(1)>(ident, v);
  }
  static __device__ __forceinline__ int up1(int v) { return dpp<DPP_ROW_SHR(1)>(v, v); }
  static __device__ __forceinline__ int bcast(int v, int src) { return __shfl(v, src, 16); }
};

// G = 64: one read per wave.  Reductions end in v_readlane, so every
// group-uniform quantity of the DP (band, maxima, break tests) lives in SGPRs
// and the row bookkeeping runs on the scalar unit.
template <>
struct Grp<64> {
  static __device__ __forceinline__ int lane() { return (int)(threadIdx.x & 63); }
  static __device__ __forceinline__ int gmax(int v) {
    v = max_bc31(max_bc15(max_ror1(max_ror2(max_ror4(max_ror8(v))))));
    return __builtin_amdgcn_readlane(v, 63);
  }
  static __device__ __forceinline__ int gmin(int v) {
    v = min_bc31(min_bc15(min_ror1(min_ror2(min_ror4(min_ror8(v))))));
    return __builtin_amdgcn_readlane(v, 63);
  }
  static __device__ __forceinline__ int excl_max(int v, int ident) {
    v = max_bc31(max_bc15(max_shr8(max_shr4(max_shr2(max_shr1(v))))));
    return dpp<DPP_WAVE_SHR1>(ident, v);
  }
  static __device__ __forceinline__ int up1(int v) { return dpp<DPP_WAVE_SHR1>(v, v); }
  static __device__ __forceinline__ int bcast(int v, int src) { return __builtin_amdgcn_readlane(v, src); }
};

// a group-uniform value made visibly uniform to the compiler when a group is
// the whole wave (then it lives in an SGPR)
template <int G>
__device__ __forceinline__ int guni(int x) {
  if constexpr (G == 64) return __builtin_amdgcn_readfirstlane(x);
  else return x;
}
template <int G>
__device__ __forceinline__ int64_t guni64(int64_t x) {
  if constexpr (G == 64) {
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)x);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)((uint64_t)x >> 32));
    return (int64_t)((uint64_t)hi << 32 | lo);
  } else {
    return x;
  }
}

}  // namespace bwagpu
