// aw_stamps.hip — diagnostic build of the AGPR-owning forward (attention_fwd_aw.hip) with
// per-phase shader-cycle totals per wave (development tool; not part of libmfa_amd.so).
// Build: make -C tools/diag aw_stamps     Run: tools/diag/aw_stamps [H] [S] [causal] [reps]
// Prints the median over waves of each phase's cycles per loop iteration.
#define MFA_STAMPS 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_aw.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void fill_rand(uint16_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = mfa::F16::from_f32(((h & 0xffff) / 65535.f * 2.f - 1.f) * 0.25f);
  }
}

int main(int argc, char** argv) {
  const int H = argc > 1 ? atoi(argv[1]) : 16;
  const int S = argc > 2 ? atoi(argv[2]) : 8192;
  const int causal = argc > 3 ? atoi(argv[3]) : 0;
  const int reps = argc > 4 ? atoi(argv[4]) : 200;
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
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < reps; ++i) CK(mfa::fwd_aw_dispatch(p, mfa::P_FP16, D, st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < 50; ++i) CK(mfa::fwd_aw_dispatch(p, mfa::P_FP16, D, st));
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double us = ms * 1e3 / 50;
  const double fl = 4.0 * D * (causal ? (double)S * (S + 1) / 2 : (double)S * S) * B * H;
  printf("H=%d S=%d causal=%d: %.2f us/launch -> %.1f TFLOP/s (stamped build)\n", H, S, causal, us,
         fl / (us * 1e-6) / 1e12);
  std::vector<unsigned long long> stamps(1 << 20, 0);
  void* dsym;
  CK(hipGetSymbolAddress(&dsym, HIP_SYMBOL(mfa::g_mfa_stamps)));
  CK(hipMemset(dsym, 0, sizeof(unsigned long long) << 20));
  CK(mfa::fwd_aw_dispatch(p, mfa::P_FP16, D, st));
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(stamps.data(), dsym, sizeof(unsigned long long) << 20, hipMemcpyDeviceToHost));
  const int iters = causal ? 0 : S / 64;  // unmasked: one 64-key tile per iteration
  const char* names[8] = {"QK_0 | sm_1", "mask+decide_1", "PV_1 | sm_0", "QK_1 | sm_0",
                          "mask+decide_0", "PV_0 | sm_1", "wait_vm", "barrier"};
  double tot = 0;
  for (int s = 0; s < 8; ++s) {
    std::vector<double> x;
    for (int w = 0; w < (1 << 17); ++w)
      if (stamps[w * 8 + 6]) x.push_back((double)stamps[w * 8 + s]);
    if (x.empty()) continue;
    std::sort(x.begin(), x.end());
    const double med = x[x.size() / 2];
    tot += med;
    printf("%-16s med %10.0f cyc  p90 %10.0f", names[s], med, x[(size_t)(0.9 * (x.size() - 1))]);
    if (iters) printf("  per iteration %7.1f", med / iters);
    printf("\n");
  }
  if (iters) printf("total per iteration %.1f cycles for 64 MFMAs per wave (%.1f per MFMA)\n", tot / iters, tot / iters / 64);
  return 0;
}
