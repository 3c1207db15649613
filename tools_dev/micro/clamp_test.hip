// What the clamp bit does on gfx950 packed 16-bit integer multiplies:
// v_pk_mul_lo_u16 a, b clamp  for a few (a, b) pairs, low and high halves.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const unsigned* a, const unsigned* b, unsigned* o, int n) {
  const int i = threadIdx.x;
  if (i >= n) return;
  unsigned r, s;
  asm volatile("v_pk_mul_lo_u16 %0, %1, %2 clamp" : "=v"(r) : "v"(a[i]), "v"(b[i]));
  asm volatile("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(s) : "v"(a[i]), "v"(b[i]));
  o[2 * i] = r;
  o[2 * i + 1] = s;
}
int main() {
  const unsigned A[] = {0x00000000u, 0x00010000u, 0x00000001u, 0x00020003u, 0x7fff0100u, 0x01000001u, 0xffffffffu};
  const unsigned B[] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu, 0x01000001u, 0x00010001u};
  const int n = 7;
  unsigned *da, *db, *dout, out[2 * n];
  hipMalloc(&da, sizeof A); hipMalloc(&db, sizeof B); hipMalloc(&dout, sizeof out);
  hipMemcpy(da, A, sizeof A, hipMemcpyHostToDevice); hipMemcpy(db, B, sizeof B, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, da, db, dout, n);
  hipMemcpy(out, dout, sizeof out, hipMemcpyDeviceToHost);
  for (int i = 0; i < n; ++i) printf("a=%08x b=%08x clamp=%08x plain=%08x\n", A[i], B[i], out[2 * i], out[2 * i + 1]);
  return 0;
}
