// micro-test: LDS layout written by global_load_lds of 1/4/16 bytes with 32 active lanes
#include <hip/hip_runtime.h>
#include <stdio.h>
#define GLDS(g, l, S) __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(g), (void __attribute__((address_space(3)))*)(l), S, 0, 0)
__global__ void k(const unsigned char* src, unsigned* out) {
  __shared__ __attribute__((aligned(16))) unsigned char s[4096];
  const int r = threadIdx.x;
  for (int i = r; i < 4096; i += 64) s[i] = 0xEE;
  __syncthreads();
  GLDS(src + r, s + 0, 1);                 // 64 lanes x 1 B
  if (r < 32) GLDS(src + 256 + 4 * r, s + 256, 4);   // 32 lanes x 4 B
  if (r < 32) GLDS(src + 1024 + 16 * r, s + 1024, 16);  // 32 lanes x 16 B
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = r; i < 1024; i += 64) out[i] = ((const unsigned*)s)[i];
}
int main() {
  unsigned char h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = (unsigned char)(i * 7 + 3);
  unsigned char* d; unsigned* o;
  hipMalloc(&d, 4096); hipMalloc(&o, 4096);
  hipMemcpy(d, h, 4096, hipMemcpyHostToDevice);
  k<<<1, 64>>>(d, o);
  unsigned res[1024];
  hipMemcpy(res, o, 4096, hipMemcpyDeviceToHost);
  const unsigned char* rb = (const unsigned char*)res;
  int bad1 = 0, bad4 = 0, bad16 = 0;
  for (int i = 0; i < 64; ++i) bad1 += rb[i] != h[i];
  for (int i = 0; i < 128; ++i) bad4 += rb[256 + i] != h[256 + i];
  for (int i = 0; i < 512; ++i) bad16 += rb[1024 + i] != h[1024 + i];
  printf("glds layout mismatches: 1B %d/64, 4B %d/128, 16B %d/512\n", bad1, bad4, bad16);
  printf("first bytes 1B region: %02x %02x %02x %02x (want %02x %02x %02x %02x)\n", rb[0], rb[1], rb[2], rb[3], h[0], h[1], h[2], h[3]);
  printf("byte 64..67 (should be untouched 0xEE): %02x %02x %02x %02x\n", rb[64], rb[65], rb[66], rb[67]);
  return 0;
}
