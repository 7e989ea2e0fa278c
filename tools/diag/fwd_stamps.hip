// fwd_stamps.hip — diagnostic build of the v2 forward with per-wave phase stamps
// (development tool; not part of libmfa_amd.so).  Build: make -C tools/diag
// Run: tools/diag/fwd_stamps [H] [S] [causal] [variants, e.g. s,p,3] [reps] [D]
// Prints, per stamp slot, the spread over waves of (slot time − kernel's first start), µs.
#define MFA_STAMPS 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_v2.hip"
// The adjacent fp16 pairs route to the pipelined kernel (attention_fwd_pipe.hip), which this
// build does not link: report it as not covered so the dispatcher takes the shared-tile kernel.
namespace mfa {
hipError_t fwd_pipe_dispatch(const FwdParams&, int, int, hipStream_t) { return hipErrorNotSupported; }
}  // namespace mfa

#include <algorithm>
#include <cstring>
#include <cmath>
#include <cstdio>
#include <cstdlib>
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

int main(int argc, char** argv) {
  setenv("MFA_DEV", "1", 1);  // the library reads its A/B switches only under MFA_DEV=1
  const int H = argc > 1 ? atoi(argv[1]) : 16;
  const int S = argc > 2 ? atoi(argv[2]) : 4096;
  const int causal = argc > 3 ? atoi(argv[3]) : 1;
  const char* var = argc > 4 ? argv[4] : "p";
  const int reps = argc > 5 ? atoi(argv[5]) : 400;
  const int B = 1;
  const int D = argc > 6 ? atoi(argv[6]) : 128;
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
  p.mask.causal = causal; p.mask.skip_ok = 1;
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  // Variants: comma-separated MFA_FWD_VARIANT[MFA_FWD_PAIR] codes, e.g. "p,p4,s" — timed in
  // interleaved rounds (the chip's clock drifts between calls), stamped with the first.
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
  auto set_var = [&](const std::string& v) {
    if (v[0] == 't') {  // single-block kernel with MFA_FWD2_TUNE=<digit>
      setenv("MFA_FWD_VARIANT", "s", 1);
      setenv("MFA_FWD2_TUNE", v.substr(1).c_str(), 1);
      unsetenv("MFA_FWD_PAIR");
      return;
    }
    unsetenv("MFA_FWD2_TUNE");
    setenv("MFA_FWD_VARIANT", v.substr(0, 1).c_str(), 1);
    if (v.size() > 1) setenv("MFA_FWD_PAIR", v.substr(1).c_str(), 1);
    else unsetenv("MFA_FWD_PAIR");
  };
  double fl = 4.0 * D * (causal ? (double)S * (S + 1) / 2 : (double)S * S) * B * H;
  for (int i = 0; i < reps; ++i) {
    set_var(vars[i % vars.size()]);
    CK(mfa::fwd2_dispatch(p, mfa::P_FP16, D, st));
  }
  const int timed = 50;
  std::vector<std::vector<float>> res(vars.size());
  for (int r = 0; r < 5; ++r)
    for (size_t vi = 0; vi < vars.size(); ++vi) {
      set_var(vars[vi]);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < timed; ++i) CK(mfa::fwd2_dispatch(p, mfa::P_FP16, D, st));
      CK(hipEventRecord(e1, st));
      CK(hipStreamSynchronize(st));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      res[vi].push_back(ms * 1e3f / timed);
    }
  for (size_t vi = 0; vi < vars.size(); ++vi) {
    std::vector<float> x = res[vi];
    std::sort(x.begin(), x.end());
    printf("H=%d S=%d causal=%d variant=%s: us/launch min %.2f med %.2f max %.2f -> %.1f TFLOP/s (med)\n",
           H, S, causal, vars[vi].c_str(), x.front(), x[x.size() / 2], x.back(),
           fl / (x[x.size() / 2] * 1e-6) / 1e12);
  }
  set_var(vars[0]);
  std::vector<unsigned long long> stamps(1 << 20, 0);
  void* dsym;
  CK(hipGetSymbolAddress(&dsym, HIP_SYMBOL(mfa::g_mfa_stamps)));
  CK(hipMemset(dsym, 0, sizeof(unsigned long long) << 20));
  CK(mfa::fwd2_dispatch(p, mfa::P_FP16, D, st));
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(stamps.data(), dsym, sizeof(unsigned long long) << 20, hipMemcpyDeviceToHost));
  {
    // Held clock: shader cycles over s_memrealtime (100 MHz) between each wave's first and
    // last stamp, median over waves (MI355X_MICROARCH.md, DVFS item 6).
    std::vector<unsigned long long> cyc(1 << 18, 0);
    void* csym;
    CK(hipGetSymbolAddress(&csym, HIP_SYMBOL(mfa::g_mfa_cyc)));
    CK(hipMemcpy(cyc.data(), csym, sizeof(unsigned long long) << 18, hipMemcpyDeviceToHost));
    const int last = (var[0] == 'p') ? 7 : 4;
    std::vector<double> mhz;
    for (int w = 0; w < (1 << 17); ++w) {
      const unsigned long long r0 = stamps[w * 8], r1 = stamps[w * 8 + last];
      if (!r0 || !r1 || r1 <= r0 || !cyc[2 * w] || !cyc[2 * w + 1]) continue;
      mhz.push_back((double)(cyc[2 * w + 1] - cyc[2 * w]) / ((double)(r1 - r0) / 100.0));
    }
    if (!mhz.empty()) {
      std::sort(mhz.begin(), mhz.end());
      printf("held clock: median %.0f MHz (p10 %.0f, p90 %.0f, %zu waves)\n", mhz[mhz.size() / 2],
             mhz[mhz.size() / 10], mhz[mhz.size() * 9 / 10], mhz.size());
    }
  }
  unsigned long long t0 = ~0ull, tend = 0;
  int nw = 0;
  for (int w = 0; w < (1 << 17); ++w) {
    if (!stamps[w * 8]) continue;
    ++nw;
    t0 = std::min(t0, stamps[w * 8]);
    for (int s = 0; s < 8; ++s) if (stamps[w * 8 + s]) tend = std::max(tend, stamps[w * 8 + s]);
  }
  printf("waves stamped %d, span %.2f us\n", nw, (tend - t0) / 100.0);
  for (int s = 0; s < 8; ++s) {
    std::vector<double> x, d;
    for (int w = 0; w < (1 << 17); ++w) {
      if (!stamps[w * 8] || !stamps[w * 8 + s]) continue;
      x.push_back((stamps[w * 8 + s] - t0) / 100.0);
      if (s > 0) {
        int pr = s - 1;
        while (pr > 0 && !stamps[w * 8 + pr]) --pr;
        d.push_back((double)(stamps[w * 8 + s] - stamps[w * 8 + pr]) / 100.0);
      }
    }
    if (x.empty()) continue;
    std::sort(x.begin(), x.end());
    std::sort(d.begin(), d.end());
    auto q = [](const std::vector<double>& a, double f) { return a.empty() ? 0.0 : a[(size_t)(f * (a.size() - 1))]; };
    printf("slot %d: at  min %7.2f p10 %7.2f med %7.2f p90 %7.2f max %7.2f | since prev: p10 %6.2f med %6.2f p90 %6.2f max %6.2f\n",
           s, x.front(), q(x, .1), q(x, .5), q(x, .9), x.back(), q(d, .1), q(d, .5), q(d, .9),
           q(d, 1.0));
  }
  // Per XCD (blockIdx % 8): median and max of the main-loop time (slot 1 -> 2) and of the
  // loop end time (slot 2), µs.
  const int wpb = (var[0] == 'p') ? 8 : 4;  // waves per workgroup of the stamped variant  // waves per workgroup of the stamped variant
  for (int x = 0; x < 8; ++x) {
    std::vector<double> lt, le;
    for (int w = 0; w < (1 << 17); ++w) {
      if (!stamps[w * 8] || !stamps[w * 8 + 2]) continue;
      if ((w / wpb) % 8 != x) continue;
      lt.push_back((stamps[w * 8 + 2] - stamps[w * 8 + 1]) / 100.0);
      le.push_back((stamps[w * 8 + 2] - t0) / 100.0);
    }
    if (lt.empty()) continue;
    std::sort(lt.begin(), lt.end());
    std::sort(le.begin(), le.end());
    printf("xcd %d: loop med %7.2f max %7.2f | loop end med %7.2f max %7.2f (n=%zu)\n", x,
           lt[lt.size() / 2], lt.back(), le[le.size() / 2], le.back(), lt.size());
  }
  if (var[0] == 'p' && causal) {
    // Shared-tile mirrored pairs: per pair index pi (workgroup / (B·H)), the median over its
    // workgroups' waves of phase 1 (slot 1 -> 2: the nA shared steps) and phase 2 (slot 2 -> 3:
    // the switch step and the rest of B's tiles) per step, and the loop end (slot 3).
    const int nb = (S + 127) / 128, np = (nb + 1) / 2;
    for (int pi = 0; pi < np; ++pi) {
      const int nA = 2 * (pi + 1), nBt = 2 * (nb - pi), h0 = (nBt - nA + 1) / 2;
      std::vector<double> p1, p2, le;
      for (int w = 0; w < (1 << 17); ++w) {
        if (!stamps[w * 8] || !stamps[w * 8 + 3]) continue;
        if ((w / 8) / (B * H) != pi) continue;
        if (stamps[w * 8 + 2]) {
          p1.push_back((stamps[w * 8 + 2] - stamps[w * 8 + 1]) / 100.0 / nA);
          if (h0 > 0) p2.push_back((stamps[w * 8 + 3] - stamps[w * 8 + 2]) / 100.0 / h0);
        }
        le.push_back((stamps[w * 8 + 3] - t0) / 100.0);
      }
      auto med = [](std::vector<double> a) { if (a.empty()) return 0.0; std::sort(a.begin(), a.end()); return a[a.size() / 2]; };
      printf("pair %2d: nA %2d phase-2 steps %2d | us/step phase 1 %.3f phase 2 %.3f | loop end med %.2f\n",
             pi, nA, h0, med(p1), med(p2), med(le));
    }
  }
  if (wpb == 4) {
    // Single-block kernel: shader-cycle totals per wave of DMA issue / tile / wait+barrier.
    double a[3] = {0, 0, 0};
    int nw2 = 0;
    for (int w = 0; w < (1 << 17); ++w) {
      if (!stamps[w * 8]) continue;
      ++nw2;
      for (int k = 0; k < 3; ++k) a[k] += (double)stamps[w * 8 + 5 + k];
    }
    const int nt = causal ? 1 : S / 64;
    const double tot = a[0] + a[1] + a[2];
    printf("per wave per tile (shader cycles%s): DMA issue %.0f (%.1f%%), tile %.0f (%.1f%%), wait+barrier %.0f (%.1f%%)\n",
           causal ? ", totals: causal" : "", a[0] / nw2 / nt, 100 * a[0] / tot, a[1] / nw2 / nt,
           100 * a[1] / tot, a[2] / nw2 / nt, 100 * a[2] / tot);
  }
  return 0;
}
