// tr_probe.hip — prints what ds_read_b64_tr_b8 / ds_read_b64_tr_b4 return per lane when lane l
// supplies LDS address 8·l over a 512-byte buffer holding byte i = i (development tool).
// Build: hipcc --offload-arch=gfx950 -O2 tr_probe.hip -o tr_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x2 __attribute__((ext_vector_type(2)));
__global__ void probe(unsigned* out) {
  __shared__ unsigned char buf[1024];
  for (int i = threadIdx.x; i < 1024; i += 64) buf[i] = (unsigned char)i;
  __syncthreads();
  const int l = threadIdx.x;
  auto* p = (__attribute__((address_space(3))) i32x2*)(buf + 8 * l);
  const i32x2 a = __builtin_amdgcn_ds_read_tr8_b64_v2i32(p);
  const i32x2 b = __builtin_amdgcn_ds_read_tr4_b64_v2i32(p);
  out[l * 4 + 0] = a[0]; out[l * 4 + 1] = a[1];
  out[l * 4 + 2] = b[0]; out[l * 4 + 3] = b[1];
}
int main() {
  unsigned* d;
  hipMalloc(&d, 64 * 16);
  probe<<<1, 64>>>(d);
  unsigned h[256];
  hipMemcpy(h, d, 64 * 16, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d tr8:", l);
    for (int k = 0; k < 8; ++k) printf(" %3u", (h[l * 4 + k / 4] >> (8 * (k % 4))) & 255);
    printf("   tr4 nibbles:");
    for (int k = 0; k < 16; ++k) printf(" %2u", (h[l * 4 + 2 + k / 8] >> (4 * (k % 8))) & 15);
    printf("\n");
  }
  return 0;
}
