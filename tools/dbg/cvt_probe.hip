// Probe (development): fp32 -> fp16 rounding of v_cvt_f16_f32 vs v_cvt_pk_f16_f32 on ties.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
__global__ void k(const float* x, unsigned* o) {
  int i = threadIdx.x;
  float a = x[i];
  unsigned r1, r2;
  asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(r1) : "v"(a));
  asm volatile("v_cvt_pk_f16_f32 %0, %1, %1" : "=v"(r2) : "v"(a));
  o[2 * i] = r1 & 0xffff; o[2 * i + 1] = r2 & 0xffff;
}
int main() {
  // ties: fp16 mantissa 10 bits; fp32 23 bits; tie when low 13 bits = 0x1000
  float h[64]; unsigned bits[64];
  for (int i = 0; i < 64; ++i) {
    unsigned b = 0x3f800000u | ((unsigned)(i * 37 % 1024) << 13) | 0x1000u;  // 1.xxx + half ulp
    if (i & 1) b |= 0x80000000u;
    if (i >= 32) b = (b & ~0x1fffu) | 0x1001u;  // just above the tie
    bits[i] = b; memcpy(&h[i], &b, 4);
  }
  float* dx; unsigned* dout; unsigned ho[128];
  hipMalloc(&dx, sizeof h); hipMalloc(&dout, sizeof ho);
  hipMemcpy(dx, h, sizeof h, hipMemcpyHostToDevice);
  k<<<1, 64>>>(dx, dout);
  hipMemcpy(ho, dout, sizeof ho, hipMemcpyDeviceToHost);
  int diff = 0;
  for (int i = 0; i < 64; ++i) {
    // RNE reference
    unsigned b = bits[i], sign = (b >> 16) & 0x8000, m = (b >> 13) & 0x3ff, rest = b & 0x1fff;
    unsigned e = ((b >> 23) & 0xff) - 127 + 15;
    unsigned r = sign | (e << 10) | m;
    if (rest > 0x1000 || (rest == 0x1000 && (m & 1))) r += 1;
    if (i < 6 || ho[2 * i] != ho[2 * i + 1] || ho[2 * i] != r)
      printf("i=%2d in %08x cvt %04x cvt_pk %04x rne %04x\n", i, b, ho[2 * i], ho[2 * i + 1], r);
    diff += ho[2 * i] != ho[2 * i + 1];
  }
  printf("differences cvt vs cvt_pk: %d of 64\n", diff);
  return 0;
}
