// stream_stamps.hip — diagnostic build of the stream-split causal forward with per-wave phase
// stamps (development tool; not part of libmfa_amd.so).  Build: make -C tools/diag stream_stamps
// Run: tools/diag/stream_stamps [H] [S] [D] [W]
// Slots: 0 start, then per segment k < 2: 1+3k prologue done, 2+3k loop done, 3+3k epilogue
// done (store / publish / merge); 7 end.  Prints the per-slot spread, the per-step time of
// each segment, the held clock, and the workgroups that end last.
#define MFA_STAMPS 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_fwd_stream.hip"

#include <algorithm>
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
  const int S = argc > 2 ? atoi(argv[2]) : 4096;
  const int D = argc > 3 ? atoi(argv[3]) : 128;
  if (argc > 4) setenv("MFA_FWD_STREAM_WGS", argv[4], 1);
  setenv("MFA_DEV", "1", 1);  // the library reads its A/B switches only under MFA_DEV=1
  setenv("MFA_FWD_STREAM", "1", 1);
  const int B = 1;
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
  p.mask.causal = 1; p.mask.skip_ok = 1;
  size_t zb = 0;
  const size_t wsb = mfa::fwd_stream_workspace_bytes(p, mfa::P_FP16, D, &zb);
  if (!wsb) { fprintf(stderr, "shape not taken by the stream kernel\n"); return 1; }
  CK(hipMalloc(&p.ws, wsb));
  CK(hipMemset(p.ws, 0, zb));
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 400; ++i) CK(mfa::fwd_stream_dispatch(p, mfa::P_FP16, D, st));
  std::vector<float> res;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < 50; ++i) CK(mfa::fwd_stream_dispatch(p, mfa::P_FP16, D, st));
    CK(hipEventRecord(e1, st));
    CK(hipStreamSynchronize(st));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    res.push_back(ms * 1e3f / 50);
  }
  std::sort(res.begin(), res.end());
  const double fl = 4.0 * D * (double)S * (S + 1) / 2 * B * H;
  printf("H=%d S=%d D=%d: us/launch med %.2f -> %.1f TFLOP/s\n", H, S, D, res[2], fl / (res[2] * 1e-6) / 1e12);
  std::vector<unsigned long long> stamps(1 << 20, 0), cyc(1 << 18, 0);
  void *dsym, *csym;
  CK(hipGetSymbolAddress(&dsym, HIP_SYMBOL(mfa::g_mfa_stamps)));
  CK(hipGetSymbolAddress(&csym, HIP_SYMBOL(mfa::g_mfa_cyc)));
  CK(hipMemset(dsym, 0, sizeof(unsigned long long) << 20));
  CK(mfa::fwd_stream_dispatch(p, mfa::P_FP16, D, st));
  CK(hipStreamSynchronize(st));
  CK(hipMemcpy(stamps.data(), dsym, sizeof(unsigned long long) << 20, hipMemcpyDeviceToHost));
  CK(hipMemcpy(cyc.data(), csym, sizeof(unsigned long long) << 18, hipMemcpyDeviceToHost));
  std::vector<double> mhz;
  unsigned long long t0 = ~0ull;
  int nw = 0;
  for (int w = 0; w < (1 << 17); ++w) {
    if (!stamps[w * 8]) continue;
    ++nw;
    t0 = std::min(t0, stamps[w * 8]);
    const unsigned long long r0 = stamps[w * 8], r1 = stamps[w * 8 + 7];
    if (r1 > r0 && cyc[2 * w + 1] > cyc[2 * w])
      mhz.push_back((double)(cyc[2 * w + 1] - cyc[2 * w]) / ((double)(r1 - r0) / 100.0));
  }
  std::sort(mhz.begin(), mhz.end());
  if (!mhz.empty()) printf("held clock: median %.0f MHz, waves %d\n", mhz[mhz.size() / 2], nw);
  auto qt = [](std::vector<double> a, double f) { if (a.empty()) return 0.0; std::sort(a.begin(), a.end()); return a[(size_t)(f * (a.size() - 1))]; };
  for (int s = 0; s < 8; ++s) {
    std::vector<double> x, d;
    for (int w = 0; w < (1 << 17); ++w) {
      if (!stamps[w * 8] || !stamps[w * 8 + s]) continue;
      x.push_back((stamps[w * 8 + s] - t0) / 100.0);
      int pr = s - 1;
      while (pr > 0 && !stamps[w * 8 + pr]) --pr;
      if (s > 0) d.push_back((double)(stamps[w * 8 + s] - stamps[w * 8 + pr]) / 100.0);
    }
    if (x.empty()) continue;
    printf("slot %d: at med %7.2f p90 %7.2f max %7.2f | since prev: p10 %6.2f med %6.2f p90 %6.2f max %6.2f (n=%zu)\n",
           s,qt(x, .5),qt(x, .9),qt(x, 1.0),qt(d, .1),qt(d, .5),qt(d, .9),qt(d, 1.0), x.size());
  }
  // Per workgroup: segments (from the same split), loop time per step, end time.
  mfa::FwdParams pp = p;
  int W, L, T, Th, nb;
  mfa::stream_split(pp, mfa::P_FP16, D, &W, &L, &T, &Th, &nb);
  std::vector<double> step0, step1, end2, end1;
  for (int bid = 0; bid < W; ++bid) {
    const int v = (W & 7) == 0 ? (bid & 7) * (W >> 3) + (bid >> 3) : bid;
    const int g0 = v * L, g1 = std::min(g0 + L, T);
    std::vector<int> segl;
    for (int gpos = g0; gpos < g1;) {
      const int bh = gpos / Th;
      int blk, toff, ntb;
      mfa::stream_locate(gpos - bh * Th, nb, p.C, 64, &blk, &toff, &ntb);
      const int th = std::min(ntb, toff + (g1 - gpos));
      segl.push_back(th - toff);
      gpos += th - toff;
    }
    const int w = bid * 8;  // wave 0 of the workgroup
    if (!stamps[w * 8]) continue;
    step0.push_back((stamps[w * 8 + 2] - stamps[w * 8 + 1]) / 100.0 / segl[0]);
    if (segl.size() > 1 && stamps[w * 8 + 5]) step1.push_back((stamps[w * 8 + 5] - stamps[w * 8 + 4]) / 100.0 / segl[1]);
    (segl.size() > 1 ? end2 : end1).push_back((stamps[w * 8 + 7] - t0) / 100.0);
  }
  printf("us/step seg0 med %.3f p90 %.3f | seg1 med %.3f p90 %.3f\n",qt(step0, .5),qt(step0, .9),qt(step1, .5),qt(step1, .9));
  printf("end: 1-segment WGs med %.2f max %.2f (n=%zu) | 2+-segment WGs med %.2f max %.2f (n=%zu)\n",
        qt(end1, .5),qt(end1, 1.0), end1.size(),qt(end2, .5),qt(end2, 1.0), end2.size());
  return 0;
}
