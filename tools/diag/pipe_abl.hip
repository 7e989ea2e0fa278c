// pipe_abl.hip — timing-only ablations of the software-pipelined forward (development tool;
// not part of libmfa_amd.so).  Build: make -C tools/diag pipe_abl
// Run: tools/diag/pipe_abl [H] [S] [codes, e.g. s,0,1,2,3,4,8,12,15]
//   s: the shipped shared-tile kernel (mfa_fwd2_share_kernel, adjacent pairs)
//   ABL bits of mfa_fwd_pipe_kernel<ABL>: 1 no LDS-DMA in the loop, 2 no vmcnt wait and no
//   barrier in the loop, 4 no exp / row-sum / pack, 8 no LDS fragment reads (MFMAs on stale
//   registers), 16 the step's LDS-DMA pieces inside the X block's MFMA gaps (correct results).
//   Results are wrong for every code but 0, 16 and s.
#define MFA_PIPE_ABL 1
#include "fwd_pipe_asm_abl.h"
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_pipe.hip"
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_v2.hip"

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

__global__ void fill_rand(uint16_t* x, size_t n, uint32_t seed) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    float f = ((h & 0xffff) / 65535.f * 2.f - 1.f) * 0.25f;
    x[i] = mfa::F16::from_f32(f);
  }
}

template <int A>
static hipError_t run_abl(const mfa::FwdParams& p0, hipStream_t st) {
  mfa::FwdParams q = p0;
  q.nblk = (p0.R + 127) / 128;
  q.xcd_heads = 1;
  const int npairs = (q.nblk + 1) / 2;
  constexpr int LDS = 2 * 128 * (128 * 4 + 16);
  return mfa::launch(mfa::mfa_fwd_pipe_abl_kernel<A>, dim3(npairs * p0.B * p0.H), dim3(512), LDS, st, q);
}

int main(int argc, char** argv) {
  const int H = argc > 1 ? atoi(argv[1]) : 16;
  const int S = argc > 2 ? atoi(argv[2]) : 8192;
  const char* var = argc > 3 ? argv[3] : "s,0,1,2,3,4,8,12,15";
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
  p.nblk = (S + 127) / 128;
  p.c_log2 = 1.442695041f / sqrtf((float)D);
  p.o_mul = 1.f;
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
  auto run = [&](const std::string& v) -> hipError_t {
    if (v == "s") return mfa::fwd2_dispatch(p, mfa::P_FP16, D, st);
    switch (atoi(v.c_str())) {
      case 0: return run_abl<0>(p, st);
      case 1: return run_abl<1>(p, st);
      case 2: return run_abl<2>(p, st);
      case 3: return run_abl<3>(p, st);
      case 4: return run_abl<4>(p, st);
      case 5: return run_abl<5>(p, st);
      case 7: return run_abl<7>(p, st);
      case 8: return run_abl<8>(p, st);
      case 11: return run_abl<11>(p, st);
      case 12: return run_abl<12>(p, st);
      case 15: return run_abl<15>(p, st);
      case 16: return run_abl<16>(p, st);
      case 18: return run_abl<18>(p, st);
      default: fprintf(stderr, "unknown code %s\n", v.c_str()); exit(1);
    }
  };
  const double fl = 4.0 * D * (double)S * S * B * H;
  for (int i = 0; i < 300; ++i) CK(run(vars[i % vars.size()]));
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
  // Clock held during each pipe variant: back-to-back launches for ~1.5 s, then one stamped
  // launch; median over waves of (shader cycles) / (100 MHz ticks) over the wave's lifetime.
  std::vector<double> clk(vars.size(), 0.0);
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    if (vars[vi] == "s") continue;
    for (int i = 0; i < 3000; ++i) CK(run(vars[vi]));
    CK(hipStreamSynchronize(st));
    const int nwg = (p.R + 255) / 256 * H;
    std::vector<unsigned long long> hc((size_t)4096 * 8 * 4);
    CK(hipMemcpyFromSymbol(hc.data(), HIP_SYMBOL(mfa::g_pipe_clk), hc.size() * 8));
    std::vector<double> f;
    for (int w = 0; w < std::min(nwg, 4096) * 8; ++w) {
      const double dc = (double)(hc[w * 4 + 2] - hc[w * 4 + 0]);
      const double dr = (double)(hc[w * 4 + 3] - hc[w * 4 + 1]);
      if (dr > 0) f.push_back(dc / dr * 0.1);
    }
    std::sort(f.begin(), f.end());
    clk[vi] = f.empty() ? 0 : f[f.size() / 2];
  }
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    std::vector<float> x = res[vi];
    std::sort(x.begin(), x.end());
    printf("H=%d S=%d code=%-3s us/launch min %8.2f med %8.2f -> %7.1f TFLOP/s (med), clock %.3f GHz\n",
           H, S, vars[vi].c_str(), x.front(), x[x.size() / 2], fl / (x[x.size() / 2] * 1e-6) / 1e12,
           clk[vi]);
  }
  // Bit-identity of the correct variants (0, 16) against the first listed correct one.
  std::vector<float> ref, cur;
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    const std::string& v = vars[vi];
    if (v != "0" && v != "16" && v != "s") continue;
    CK(hipMemset(o, 0, n * 4));
    CK(run(v));
    CK(hipStreamSynchronize(st));
    cur.resize(n);
    CK(hipMemcpy(cur.data(), o, n * 4, hipMemcpyDeviceToHost));
    if (ref.empty()) {
      ref = cur;
      printf("reference for bit checks: code %s\n", v.c_str());
      continue;
    }
    double md = 0;
    size_t nd = 0;
    for (size_t i = 0; i < n; ++i) {
      const double d = fabs((double)cur[i] - (double)ref[i]);
      if (d > 0) ++nd;
      md = d > md ? d : md;
    }
    printf("code %s vs reference: max |diff| %.3g, %zu differing elements\n", v.c_str(), md, nd);
  }
  return 0;
}
