// stream.hip — bwagpu_sw_stream: the FPGA wire format of bwa-flow's
// seed-extension stage (src/FPGAPipeline.cpp) decoded and extended on the
// device, results in the FPGA's packed record layout.
#include "ksw_dev.h"

namespace bwagpu {

// ============================================================ FPGA wire format
// bwagpu_sw_stream (include/bwagpu.h).  Lane per read record: the record's
// bases unpacked to bytes (4-bit words, first base in the high nibble,
// FPGAPipeline.cpp:262-276), then every chain's window and every task checked
// and written to tasks[task index], binned by read length like the spec
// lists.  Anything that does not parse sets a flag and is not queued.
__device__ __forceinline__ int64_t stream64(const int32_t* b, int64_t at) {
  return (int64_t)((uint64_t)(uint32_t)b[at] | (uint64_t)(uint32_t)b[at + 1] << 32);
}

__global__ void __launch_bounds__(256) stream_decode_kernel(StreamArgs a) {
  const int rd = blockIdx.x * blockDim.x + threadIdx.x;
  if (rd >= a.n_reads) return;
  const int32_t* __restrict__ in = a.buf;
  const int64_t p = a.rstart[rd];
  const int64_t end = in[p];  // the host walk checked p + 2 < end <= words
  const int lq = in[p + 1];   // and 0 <= lq <= BWAGPU_MAX_READ_LEN
  const int nw = (lq + 7) >> 3;
  int err = 0;
  if (p + 3 + nw > end) err |= STR_ERR_RECORD;
  int64_t c = p + 2 + nw;
  if (!err) {
    uint8_t* q = a.qpool + 8 * p;
    for (int k = 0; k < nw; ++k) {
      const uint32_t w = (uint32_t)in[p + 2 + k];
      uint32_t lo4 = 0, hi4 = 0;
      int bad = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t v = w >> (28 - 4 * j) & 15;
        bad |= 8 * k + j < lq && v > 4;
        if (j < 4) lo4 |= v << (8 * j);
        else hi4 |= v << (8 * (j - 4));
      }
      if (bad) err |= STR_ERR_BASE;
      reinterpret_cast<uint2*>(q)[k] = make_uint2(lo4, hi4);  // qpool is 8-byte aligned per word
    }
    const int nch = in[c++];
    for (int ch = 0; ch < nch && !err; ++ch) {
      if (c + 5 > end) {
        err |= STR_ERR_RECORD;
        break;
      }
      const int64_t lo = stream64(in, c), hi = stream64(in, c + 2);
      const int ns = in[c + 4];
      c += 5;
      if (ns < 0 || c + 5 * (int64_t)ns > end) {
        err |= STR_ERR_RECORD;
        break;
      }
      if (ns && (lo < 0 || hi > 2 * a.l_pac || lo > hi || (lo < a.l_pac && a.l_pac < hi))) {
        err |= STR_ERR_SEED;
        break;
      }
      for (int k = 0; k < ns; ++k, c += 5) {
        const int t = in[c];
        StreamTask T;
        T.s.rbeg = stream64(in, c + 1);
        T.s.qbeg = in[c + 3];
        T.s.len = in[c + 4];
        T.s.score = 0;
        T.s.pad_ = 0;
        if (t < 0 || t >= a.cap) {
          err |= STR_ERR_TASK;
          break;
        }
        if (T.s.qbeg < 0 || T.s.len <= 0 || T.s.qbeg + T.s.len > lq || T.s.rbeg < lo || T.s.rbeg + T.s.len > hi) {
          err |= STR_ERR_SEED;
          break;
        }
        if (atomicAdd(&a.seen[t], 1) != 0) {
          err |= STR_ERR_DUP;
          break;
        }
        T.lo = lo;
        T.hi = hi;
        T.qoff = 8 * p;
        T.lq = lq;
        T.pad_ = 0;
        a.tasks[t] = T;
        const int bin = spec_bin(lq);
        a.lists[(size_t)bin * a.cap + atomicAdd(&a.ctr[bin], 1)] = t;
        atomicAdd(&a.ctr[kStrDecoded], 1);
        atomicMax(&a.ctr[kStrMax], t + 1);
      }
    }
    if (!err && c != end) err |= STR_ERR_RECORD;
  }
  if (err) atomicOr(&a.ctr[kStrErr], err);
}

// one wave per task from the bin's sharded queue; the record (5 words of two
// int16 each, little-endian like the FPGA's short[]): t, qb | dqe, drb | dre,
// score | truesc, w
template <int C>
__global__ void __launch_bounds__(kBlock) stream_ext_kernel(DevOpt o, DevRef ref, StreamArgs a, int bin,
                                                            int tb_bytes) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int wib = uni((int)(threadIdx.x >> 6));
  uint8_t* const tbl = lds + wib * 2 * tb_bytes;
  uint8_t* const tbr = tbl + tb_bytes;
  const int n = uni(__hip_atomic_load(&a.ctr[bin], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const int32_t* L = a.lists + (size_t)bin * a.cap;
  ShardQ qq;
  qq.init(a.ctr + kStrHeads + 8 * kQHStride * bin, n);
  int m0, cap;
  while (qq.claim(1, m0, cap)) {
    for (int m = m0; m < m0 + 1 && m < cap; ++m) {
      const int t = uni(L[qq.shard + 8 * m]);
      const StreamTask& T = a.tasks[t];
      const bwagpu_seed_t s = uni_seed(T.s);
      const int lq = uni(T.lq);
      ChainWin cw;
      cw.lo = uni64(T.lo);
      cw.hi = uni64(T.hi);
      const SeedExt e = extend_seed<C>(o, ref, s, lq, a.qpool + uni64(T.qoff), cw, tbl, tbr);
      const int d = (int)(threadIdx.x & 63);
      const uint32_t dqe = (uint16_t)(e.qe - (s.qbeg + s.len)), drb = (uint16_t)(e.rb - s.rbeg),
                     dre = (uint16_t)(e.re - (s.rbeg + s.len));
      uint32_t v = (uint32_t)t;
      v = d == 1 ? (uint16_t)e.qb | dqe << 16 : v;
      v = d == 2 ? drb | dre << 16 : v;
      v = d == 3 ? (uint16_t)e.score | (uint32_t)(uint16_t)e.truesc << 16 : v;
      v = d == 4 ? (uint32_t)(uint16_t)e.w : v;
      if (d < 5) a.out[(size_t)5 * t + d] = (int32_t)v;
    }
  }
}

hipError_t launch_sw_stream(const DevOpt& o, const DevRef& ref, const StreamArgs& a, int tb_bytes, hipStream_t st) {
  if (a.n_reads == 0) return hipSuccess;
  hipLaunchKernelGGL(stream_decode_kernel, dim3((a.n_reads + 255) / 256), dim3(256), 0, st, a);
  const size_t lds = (size_t)(kBlock / 64) * 2 * tb_bytes;
  hipLaunchKernelGGL(stream_ext_kernel<3>, dim3(resident_blocks(stream_ext_kernel<3>, lds)), dim3(kBlock), lds, st,
                     o, ref, a, 0, tb_bytes);
  hipLaunchKernelGGL(stream_ext_kernel<4>, dim3(resident_blocks(stream_ext_kernel<4>, lds)), dim3(kBlock), lds, st,
                     o, ref, a, 1, tb_bytes);
  hipLaunchKernelGGL(stream_ext_kernel<16>, dim3(resident_blocks(stream_ext_kernel<16>, lds)), dim3(kBlock), lds,
                     st, o, ref, a, 2, tb_bytes);
  return hipGetLastError();
}

}  // namespace bwagpu
