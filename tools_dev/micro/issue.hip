// Issue-cost microbenchmark (gfx950): cycles per SIMD per instruction for
// VALU / SALU / DPP / s_nop / mixed streams at W waves per SIMD.
// W blocks of 4 waves per CU (one wave per SIMD per block): W waves per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define REP8(x) x x x x x x x x
constexpr int ITERS = 4096;

template <int MODE>
__global__ void k(int* out, int seed) {
  int v0 = threadIdx.x + seed, v1 = v0 * 3, v2 = v0 * 5, v3 = v0 * 7;
  int s0 = seed, s1 = seed * 3, s2 = seed * 5, s3 = seed * 7;
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0) {  // 32 independent VALU
      REP8(asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %2, %2, %3\n v_xor_b32 %1, %1, %0\n v_xor_b32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 1) {  // 32 SALU
      REP8(asm volatile("s_mul_i32 %0, %0, %1\n s_mul_i32 %2, %2, %3\n s_mul_hi_u32 %1, %1, %0\n s_mul_hi_u32 %3, %3, %2" : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));)
    } else if (MODE == 2) {  // 16 VALU + 16 SALU interleaved
      REP8(asm volatile("v_add_u32 %0, %0, %1\n s_mul_i32 %4, %4, %5\n v_xor_b32 %2, %2, %3\n s_mul_i32 %6, %6, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3));)
    } else if (MODE == 3) {  // 32 DPP max on 4 independent chains, no nops needed (4 chains)
      REP8(asm volatile("v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %1, %1, %1 row_shr:1 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %2, %2, %2 row_shr:1 row_mask:0xf bank_mask:0xf\n v_max_i32_dpp %3, %3, %3 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 4) {  // 16 DPP single chain, s_nop 1 before each (the extension kernel's form)
      REP8(asm volatile("s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n s_nop 1\n v_max_i32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf" : "+v"(v0));)
    } else if (MODE == 5) {  // 32 dependent VALU (one chain)
      REP8(asm volatile("v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_xor_b32 %0, %0, %1" : "+v"(v0) : "v"(v1));)
    } else if (MODE == 6) {  // 32 dependent SALU
      REP8(asm volatile("s_mul_i32 %0, %0, %1\n s_mul_hi_u32 %0, %0, %1\n s_mul_i32 %0, %0, %1\n s_mul_hi_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));)
    } else if (MODE == 7) {  // 8 x (v_readlane -> s_mul -> v_add) round trips
      REP8(asm volatile("v_readlane_b32 %4, %0, 63\n s_mul_i32 %4, %4, %5\n v_add_u32 %1, %1, %4\n v_xor_b32 %0, %0, %1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+s"(s0), "+s"(s1));)
    } else if (MODE == 8) {  // 32 s_nop 0
      REP8(asm volatile("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0");)
    } else if (MODE == 9) {  // 16 VALU + 16 SALU, SALU dependent chain (like band bookkeeping)
      REP8(asm volatile("v_add_u32 %0, %0, %1\n s_mul_i32 %4, %4, %5\n v_xor_b32 %2, %2, %3\n s_mul_hi_u32 %4, %4, %5" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+s"(s0), "+s"(s1));)
    } else if (MODE == 10) {  // 32 packed 16-bit add/max on 4 independent chains (extend_quad's bulk)
      REP8(asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_max_i16 %2, %2, %3\n v_pk_add_u16 %1, %1, %0\n v_pk_max_i16 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 11) {  // 32 packed 16-bit min/sub-saturate on 4 independent chains
      REP8(asm volatile("v_pk_min_u16 %0, %0, %1\n v_pk_sub_u16 %2, %2, %3 clamp\n v_pk_min_u16 %1, %1, %0\n v_pk_sub_u16 %3, %3, %2 clamp" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 12) {  // 32 v_perm / v_bfi / v_bitop3 / v_pk_mad_u16
      REP8(asm volatile("v_perm_b32 %0, %1, %2, %3\n v_bfi_b32 %1, %2, %3, %0\n v_bitop3_b32 %2, %3, %0, %1 bitop3:0xca\n v_pk_mad_u16 %3, %0, %1, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 13) {  // 32 packed 16-bit ops, ONE dependent chain
      REP8(asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_max_i16 %0, %0, %1\n v_pk_sub_u16 %0, %0, %1 clamp\n v_pk_min_u16 %0, %0, %1" : "+v"(v0) : "v"(v1));)
    } else if (MODE == 15) {  // 32 packed f16 add/max on 4 chains
      REP8(asm volatile("v_pk_add_f16 %0, %0, %1\n v_pk_max_f16 %2, %2, %3\n v_pk_add_f16 %1, %1, %0\n v_pk_max_f16 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 16) {  // 32 packed f16 maximum3 / minimum3 on 4 chains
      REP8(asm volatile("v_pk_maximum3_f16 %0, %0, %1, %2\n v_pk_minimum3_f16 %1, %1, %2, %3\n v_pk_maximum3_f16 %2, %2, %3, %0\n v_pk_minimum3_f16 %3, %3, %0, %1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 17) {  // 32 packed f16 fma / mul on 4 chains
      REP8(asm volatile("v_pk_fma_f16 %0, %0, %1, %2\n v_pk_mul_f16 %1, %1, %2\n v_pk_fma_f16 %2, %2, %3, %0\n v_pk_mul_f16 %3, %3, %0" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 18) {  // 32 i32 add / sub on 4 chains
      REP8(asm volatile("v_add_u32 %0, %0, %1\n v_sub_u32 %2, %2, %3\n v_add_u32 %1, %1, %0\n v_sub_u32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 19) {  // 32 i32 max on 4 chains
      REP8(asm volatile("v_max_i32 %0, %0, %1\n v_max_i32 %2, %2, %3\n v_max_i32 %1, %1, %0\n v_max_i32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 20) {  // 32 i32 max3 / add3 on 4 chains
      REP8(asm volatile("v_max3_i32 %0, %0, %1, %2\n v_add3_u32 %1, %1, %2, %3\n v_max3_i32 %2, %2, %3, %0\n v_add3_u32 %3, %3, %0, %1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 21) {  // 32 f32 add / max on 4 chains
      REP8(asm volatile("v_add_f32 %0, %0, %1\n v_max_f32 %2, %2, %3\n v_add_f32 %1, %1, %0\n v_max_f32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 22) {  // 32 v_xor / v_and / v_or / v_not on 4 chains
      REP8(asm volatile("v_xor_b32 %0, %0, %1\n v_and_b32 %2, %2, %3\n v_or_b32 %1, %1, %0\n v_xor_b32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 23) {  // 32 v_pk_add_u16 only on 4 chains
      REP8(asm volatile("v_pk_add_u16 %0, %0, %1\n v_pk_add_u16 %2, %2, %3\n v_pk_add_u16 %1, %1, %0\n v_pk_add_u16 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 24) {  // 32 v_cndmask / v_bfi on 4 chains
      REP8(asm volatile("v_bfi_b32 %0, %0, %1, %2\n v_bfi_b32 %1, %1, %2, %3\n v_bfi_b32 %2, %2, %3, %0\n v_bfi_b32 %3, %3, %0, %1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    } else if (MODE == 14) {  // 32 plain 32-bit max/min/sub on 4 chains (the unpacked form of mode 10)
      REP8(asm volatile("v_max_i32 %0, %0, %1\n v_min_u32 %2, %2, %3\n v_sub_u32 %1, %1, %0\n v_max_i32 %3, %3, %2" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3));)
    }
  }
  if ((v0 ^ v1 ^ v2 ^ v3 ^ s0 ^ s1 ^ s2 ^ s3) == 0x12345) out[threadIdx.x] = 1;
}

int main() {
  int dev = 0, ncu = 0, clk = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);  // kHz
  setvbuf(stdout, nullptr, _IONBF, 0);
  int* out;
  hipMalloc(&out, 4096 * 4);
  const char* names[] = {"VALU indep", "SALU indep", "VALU+SALU mix", "DPP 4 chains", "DPP+s_nop1 1 chain",
                         "VALU dep chain", "SALU dep chain", "readlane rt", "s_nop 0", "VALU + SALU chain",
                         "pk16 add/max 4 chains", "pk16 min/subsat 4 chains", "perm/bfi/bitop3/pk_mad",
                         "pk16 dep chain", "i32 max/min/sub 4 chains", "pk f16 add/max", "pk f16 maximum3/minimum3",
                         "pk f16 fma/mul", "i32 add/sub", "i32 max", "i32 max3/add3", "f32 add/max", "xor/and/or",
                         "pk u16 add only", "bfi"};
  printf("{\"cus\": %d, \"clock_khz\": %d, \"results\": [\n", ncu, clk);
  const int m0 = getenv("ISSUE_MODE0") ? atoi(getenv("ISSUE_MODE0")) : 0;
  for (int mode = m0; mode < 25; ++mode) {
    for (int W : {1, 2, 4, 5, 8}) {
      hipEvent_t a, b;
      hipEventCreate(&a);
      hipEventCreate(&b);
      auto launch = [&]() {
        dim3 g(ncu * W), blk(256);
        switch (mode) {
          case 0: hipLaunchKernelGGL(k<0>, g, blk, 0, 0, out, 1); break;
          case 1: hipLaunchKernelGGL(k<1>, g, blk, 0, 0, out, 1); break;
          case 2: hipLaunchKernelGGL(k<2>, g, blk, 0, 0, out, 1); break;
          case 3: hipLaunchKernelGGL(k<3>, g, blk, 0, 0, out, 1); break;
          case 4: hipLaunchKernelGGL(k<4>, g, blk, 0, 0, out, 1); break;
          case 5: hipLaunchKernelGGL(k<5>, g, blk, 0, 0, out, 1); break;
          case 6: hipLaunchKernelGGL(k<6>, g, blk, 0, 0, out, 1); break;
          case 7: hipLaunchKernelGGL(k<7>, g, blk, 0, 0, out, 1); break;
          case 8: hipLaunchKernelGGL(k<8>, g, blk, 0, 0, out, 1); break;
          case 9: hipLaunchKernelGGL(k<9>, g, blk, 0, 0, out, 1); break;
          case 10: hipLaunchKernelGGL(k<10>, g, blk, 0, 0, out, 1); break;
          case 11: hipLaunchKernelGGL(k<11>, g, blk, 0, 0, out, 1); break;
          case 12: hipLaunchKernelGGL(k<12>, g, blk, 0, 0, out, 1); break;
          case 13: hipLaunchKernelGGL(k<13>, g, blk, 0, 0, out, 1); break;
          case 14: hipLaunchKernelGGL(k<14>, g, blk, 0, 0, out, 1); break;
          case 15: hipLaunchKernelGGL(k<15>, g, blk, 0, 0, out, 1); break;
          case 16: hipLaunchKernelGGL(k<16>, g, blk, 0, 0, out, 1); break;
          case 17: hipLaunchKernelGGL(k<17>, g, blk, 0, 0, out, 1); break;
          case 18: hipLaunchKernelGGL(k<18>, g, blk, 0, 0, out, 1); break;
          case 19: hipLaunchKernelGGL(k<19>, g, blk, 0, 0, out, 1); break;
          case 20: hipLaunchKernelGGL(k<20>, g, blk, 0, 0, out, 1); break;
          case 21: hipLaunchKernelGGL(k<21>, g, blk, 0, 0, out, 1); break;
          case 22: hipLaunchKernelGGL(k<22>, g, blk, 0, 0, out, 1); break;
          case 23: hipLaunchKernelGGL(k<23>, g, blk, 0, 0, out, 1); break;
          case 24: hipLaunchKernelGGL(k<24>, g, blk, 0, 0, out, 1); break;
        }
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(a);
      for (int r = 0; r < 5; ++r) launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double cycles = ms / 5 * 1e-3 * clk * 1e3;
      const int per_iter = (mode == 4) ? 16 : (mode == 7 ? 32 : 32);
      const double per_instr_simd = cycles / ((double)ITERS * per_iter * W);  // SIMD cycles per wave-instruction
      printf("  {\"mode\": \"%s\", \"waves_per_simd\": %d, \"us\": %.1f, \"simd_cycles_per_instr\": %.3f}%s\n", names[mode],
             W, ms / 5 * 1e3, per_instr_simd, (mode == 24 && W == 8) ? "" : ",");
    }
  }
  printf("]}\n");
  return 0;
}
