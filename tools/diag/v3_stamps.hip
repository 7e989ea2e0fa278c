// v3_stamps.hip — diagnostic build of the v3 forward with per-wave segment cycle totals
// (development tool; not part of libmfa_amd.so).  Build: make -C tools/diag v3_stamps
// Run: tools/diag/v3_stamps [H] [S] [causal] [reps]
#define V3_STAMPS 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_v3.hip"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void fill_rand(uint16_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    float f = ((h & 0xffff) / 65535.f * 2.f - 1.f) * 0.25f;
    x[i] = mfa::F16::from_f32(f);
  }
}

int main(int argc, char** argv) {
  const int H = argc > 1 ? atoi(argv[1]) : 16;
  const int S = argc > 2 ? atoi(argv[2]) : 8192;
  const int causal = argc > 3 ? atoi(argv[3]) : 0;
  const int reps = argc > 4 ? atoi(argv[4]) : 50;
  const int B = 1, D = 128;
  const size_t n = (size_t)B * H * S * D;
  uint16_t *q, *k, *v, *l;
  float* o;
  CK(hipMalloc(&q, n * 2)); CK(hipMalloc(&k, n * 2)); CK(hipMalloc(&v, n * 2));
  CK(hipMalloc(&o, n * 4)); CK(hipMalloc(&l, (size_t)B * H * S * 2));
  fill_rand<<<1024, 256>>>(q, n, 1); fill_rand<<<1024, 256>>>(k, n, 2);
  fill_rand<<<1024, 256>>>(v, n, 3);
  mfa::FwdParams p;
  memset(&p, 0, sizeof(p));
  auto op = [&](const void* ptr) {
    mfa::Operand x;
    memset(&x, 0, sizeof(x));
    x.ptr = ptr; x.ss = D; x.sh = (int64_t)S * D; x.sb = (int64_t)H * S * D; x.sd = 1;
    x.prec = mfa::P_FP16; x.vec = 1; x.scale = 1.f; x.cols = D;
    return x;
  };
  p.q = op(q); p.k = op(k); p.v = op(v);
  p.o = o; p.o_ss = D; p.o_sh = (int64_t)S * D; p.o_sb = (int64_t)H * S * D;
  p.l = l; p.l_f16 = 1;
  p.B = B; p.H = H; p.Hkv = H; p.R = S; p.C = S; p.D = D;
  p.c_log2 = 1.442695041f / sqrtf((float)D);
  p.o_mul = 1.f;
  p.mask.causal = causal; p.mask.skip_ok = 1;
  setenv("MFA_FWD3", "1", 1);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 20; ++i) CK(mfa::fwd3_dispatch(p, mfa::P_FP16, 128, st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < reps; ++i) CK(mfa::fwd3_dispatch(p, mfa::P_FP16, 128, st));
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  const int nb128 = (S + 127) / 128;
  const int nwg = (causal ? (nb128 + 1) / 2 : (S + 255) / 256) * B * H;
  std::vector<unsigned long long> st_h((size_t)nwg * 4 * 8);
  CK(hipMemcpyFromSymbol(st_h.data(), HIP_SYMBOL(mfa::fwd3::g_v3_stamps), st_h.size() * 8));
  double sum[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int w = 0; w < nwg * 4; ++w)
    for (int k2 = 0; k2 < 8; ++k2) sum[k2] += (double)st_h[(size_t)w * 8 + k2];
  double tot = 0;
  for (int k2 = 0; k2 < 8; ++k2) tot += sum[k2];
  const double flop = 4.0 * D * (causal ? S * (S + 1) / 2.0 : (double)S * S) * B * H;
  printf("H%d S%d causal=%d: %.4f ms = %.1f TFLOP/s (stamped build)\n", H, S, causal, ms,
         flop / ms / 1e9);
  const char* names[8] = {"M2", "wait+barrier", "rescale A", "M4", "rescale B",
                          "outside loop", "M1", "M3"};
  const int iters_per_wg = causal ? (nb128 + 1) : (S / 64);
  for (int k2 = 0; k2 < 8; ++k2)
    printf("  %-14s %6.1f%%  %8.0f cycles per wave per iteration\n", names[k2],
           100.0 * sum[k2] / tot, sum[k2] / (nwg * 4.0) / iters_per_wg * (causal ? 1.0 : 1.0));
  return 0;
}
