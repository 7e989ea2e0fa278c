// aw_trace.hip — per-step row state of the AGPR-owning forward, workgroup 0 lane 0
// (development tool).  Build: make -C tools/diag aw_trace
#define AW_DEBUG_TRACE 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_aw.hip"
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
__global__ void fill_g(uint16_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = mfa::F16::from_f32(((h & 0xffff) / 65535.f * 2.f - 1.f) * 2.f);
  }
}
int main(int argc, char** argv) {
  const int S = argc > 1 ? atoi(argv[1]) : 512, D = 128, H = 1, B = 1;
  const size_t n = (size_t)S * D;
  uint16_t *q, *k, *v, *l; float* o;
  hipMalloc(&q, n * 2); hipMalloc(&k, n * 2); hipMalloc(&v, n * 2); hipMalloc(&o, n * 4); hipMalloc(&l, S * 2);
  fill_g<<<64, 256>>>(q, n, 1); fill_g<<<64, 256>>>(k, n, 2); fill_g<<<64, 256>>>(v, n, 3);
  mfa::FwdParams p; memset(&p, 0, sizeof(p));
  auto op = [&](const void* ptr) { mfa::Operand x; memset(&x, 0, sizeof(x)); x.ptr = ptr; x.ss = D; x.sh = (int64_t)S * D; x.sb = (int64_t)H * S * D; x.sd = 1; x.prec = mfa::P_FP16; x.vec = 1; x.scale = 1.f; x.cols = D; return x; };
  p.q = op(q); p.k = op(k); p.v = op(v); p.o = o; p.o_ss = D; p.o_sh = (int64_t)S * D; p.o_sb = (int64_t)S * D;
  p.l = l; p.l_f16 = 1; p.B = B; p.H = H; p.Hkv = H; p.R = S; p.C = S; p.D = D;
  p.c_log2 = 1.442695041f / sqrtf((float)D); p.o_mul = 1.f; p.mask.causal = 1; p.mask.skip_ok = 1;
  mfa::fwd_aw_dispatch(p, mfa::P_FP16, D, nullptr);
  hipDeviceSynchronize();
  float tr[256]; void* sym; hipGetSymbolAddress(&sym, HIP_SYMBOL(mfa::g_aw_trace));
  hipMemcpy(tr, sym, sizeof(tr), hipMemcpyDeviceToHost);
  printf("u: m0 lh0 corr0 | m1 lh1 corr1 | O0[a0] O1[a64] after B\n");
  for (int u = 0; u < 16; ++u)
    printf("%2d: %9.4f %10.4f %8.5f | %9.4f %10.4f %8.5f | %10.5f %10.5f\n", u, tr[u*8], tr[u*8+1], tr[u*8+2], tr[u*8+3], tr[u*8+4], tr[u*8+5], tr[u*8+6], tr[u*8+7]);
  return 0;
}
