// i8_abl.hip — timing-only ablations of the INT8 integer-MFMA forward at C3 (development tool;
// not part of libmfa_amd.so).  Build: make -C tools/diag i8_abl
// Run: tools/diag/i8_abl [H] [S] [codes, e.g. s,0,1,2,3,4,8,12,15]
//   s: the product kernel (attention_fwd_i8.hip, mfa_fwd_i8_kernel<F16,128,128,2,2>)
//   ABL bits of the diagnostic copy (i8_abl_kernel.hip): 1 no LDS-DMA in the loop, 2 no vmcnt
//   wait / barrier, 4 no softmax VALU, 8 no LDS fragment reads.  Wrong results but for s / 0.
// Also reports the clock each variant holds (s_memtime / s_memrealtime around the launch, one
// wave per workgroup, after ~1.5 s of back-to-back launches).
#include "i8_abl_kernel.hip"
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_i8.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

__global__ void fill_f16(uint16_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = mfa::F16::from_f32(((h & 0xffff) / 65535.f * 2.f - 1.f) * 0.25f);
  }
}
__global__ void fill_i8(int8_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = (int8_t)((int)(h % 255) - 127);
  }
}

__device__ unsigned long long g_clk[4096 * 4];
__global__ void clk_kernel(int slot) {
  if (threadIdx.x == 0) {
    g_clk[blockIdx.x * 4 + 2 * slot] = __builtin_amdgcn_s_memtime();
    g_clk[blockIdx.x * 4 + 2 * slot + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

int main(int argc, char** argv) {
  const int H = argc > 1 ? atoi(argv[1]) : 16;
  const int S = argc > 2 ? atoi(argv[2]) : 8192;
  const char* var = argc > 3 ? argv[3] : "s,0,1,2,3,4,8,12,15";
  const int B = 1, D = 128;
  const size_t n = (size_t)B * H * S * D;
  uint16_t *q, *l;
  int8_t *k, *v;
  float* o;
  CK(hipMalloc(&q, n * 2)); CK(hipMalloc(&k, n)); CK(hipMalloc(&v, n));
  CK(hipMalloc(&o, n * 4)); CK(hipMalloc(&l, (size_t)B * H * S * 2));
  fill_f16<<<1024, 256>>>(q, n, 1); fill_i8<<<1024, 256>>>(k, n, 2); fill_i8<<<1024, 256>>>(v, n, 3);
  mfa::FwdParams p;
  memset(&p, 0, sizeof(p));
  auto op = [&](const void* ptr, int prec) {
    mfa::Operand x;
    memset(&x, 0, sizeof(x));
    x.ptr = ptr; x.ss = D; x.sh = (int64_t)S * D; x.sb = (int64_t)H * S * D; x.sd = 1;
    x.prec = prec; x.vec = 1; x.scale = 1.f; x.cols = D;
    return x;
  };
  p.q = op(q, mfa::P_FP16); p.k = op(k, mfa::P_INT8); p.v = op(v, mfa::P_INT8);
  p.o = o; p.o_ss = D; p.o_sh = (int64_t)S * D; p.o_sb = (int64_t)H * S * D;
  p.l = l; p.l_f16 = 1;
  p.B = B; p.H = H; p.Hkv = H; p.R = S; p.C = S; p.D = D;
  p.nblk = (S + 127) / 128;
  p.c_log2 = 1.442695041f / sqrtf((float)D) * (0.25f / 127.f);
  p.o_mul = 0.25f / 127.f;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  std::vector<std::string> vars;
  {
    std::string all(var);
    size_t a = 0;
    while (a <= all.size()) {
      size_t e = all.find(',', a);
      if (e == std::string::npos) e = all.size();
      vars.push_back(all.substr(a, e - a));
      a = e + 1;
    }
  }
  constexpr int LDS = 2 * 128 * (128 * 4 + 16);
  const dim3 grid((p.nblk + 1) / 2 * B * H);
  auto run = [&](const std::string& vv) -> hipError_t {
    if (vv == "s") return mfa::fwd_i8mma_dispatch(p, mfa::P_FP16, st);
    switch (atoi(vv.c_str())) {
#define C_(k) case k: return mfa::launch(mfa::diag::mfa_fwd_i8_abl_kernel<k>, grid, dim3(512), LDS, st, p);
      C_(0) C_(1) C_(2) C_(3) C_(4) C_(5) C_(7) C_(8) C_(11) C_(12) C_(15)
#undef C_
      default: fprintf(stderr, "unknown code %s\n", vv.c_str()); exit(1);
    }
  };
  const double fl = 4.0 * D * (double)S * S * B * H;
  for (int i = 0; i < 200; ++i) CK(run(vars[i % vars.size()]));
  const int timed = 30;
  std::vector<std::vector<float>> res(vars.size());
  for (int r = 0; r < 7; ++r)
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < timed; ++i) CK(run(vars[vi]));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[vi].push_back(ms * 1e3f / timed);
    }
  // Clock under each variant: stamps just before and just after one launch that follows
  // ~1.5 s of back-to-back launches (256 one-wave workgroups, one per CU, 100 MHz reference).
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    for (int i = 0; i < 3000; ++i) CK(run(vars[vi]));
    clk_kernel<<<256, 64, 0, st>>>(0);
    for (int i = 0; i < 20; ++i) CK(run(vars[vi]));
    clk_kernel<<<256, 64, 0, st>>>(1);
    CK(hipStreamSynchronize(st));
    std::vector<unsigned long long> hc(256 * 4);
    CK(hipMemcpyFromSymbol(hc.data(), HIP_SYMBOL(g_clk), hc.size() * 8));
    std::vector<double> f;
    for (int w = 0; w < 256; ++w) {
      const double dc = (double)(hc[w * 4 + 2] - hc[w * 4 + 0]);
      const double dr = (double)(hc[w * 4 + 3] - hc[w * 4 + 1]);
      if (dr > 0) f.push_back(dc / dr * 0.1);
    }
    std::sort(f.begin(), f.end());
    std::vector<float> x = res[vi];
    std::sort(x.begin(), x.end());
    printf("H=%d S=%d code=%-3s us/launch min %8.2f med %8.2f -> %7.1f TOPS (med), clock %.3f GHz\n",
           H, S, vars[vi].c_str(), x.front(), x[x.size() / 2],
           fl / (x[x.size() / 2] * 1e-6) / 1e12, f.empty() ? 0.0 : f[f.size() / 2]);
  }
  return 0;
}
