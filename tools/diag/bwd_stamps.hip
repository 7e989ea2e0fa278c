// bwd_stamps.hip — diagnostic build of the fast backward with per-wave phase cycle totals of
// backwardKeyValue (development tool; not part of libmfa_amd.so).  Build: make -C tools/diag
// Run: tools/diag/bwd_stamps [B] [H] [S] [D] [band] [phase]   (fp16, non-causal; band > 0:
// sparse ranges of `band` 128-key blocks per 128-row block, as bench.py's buildBlockSparse row,
// which runs the mask instantiation; phase 0 = backwardKeyValue (default), 1 = backwardQuery.
// At most 16384 waves: B·H·S/32 for either phase)
#define MFA_BSTAMPS 1
#include "../../metal-flash-attention-plus_amd/csrc/attention_bwd_fast.hip"

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

__global__ void fill_rand16(uint16_t* x, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    x[i] = mfa::F16::from_f32(((h & 0xffff) / 65535.f * 2.f - 1.f) * 0.25f);
  }
}
__global__ void fill_const32(float* x, size_t n, float v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) x[i] = v;
}

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 4;
  const int H = argc > 2 ? atoi(argv[2]) : 32;
  const int S = argc > 3 ? atoi(argv[3]) : 4096;
  const int D = argc > 4 ? atoi(argv[4]) : 128;
  const int band = argc > 5 ? atoi(argv[5]) : 0;
  const int qphase = argc > 6 ? atoi(argv[6]) : 0;
  const int kind = qphase ? 0 : 1;  // bwd_fast_dispatch: 0 = backwardQuery, 1 = backwardKeyValue
  if ((size_t)B * H * S / 32 > (1u << 14)) { fprintf(stderr, "too many waves for the stamp buffer\n"); return 1; }
  const size_t n = (size_t)B * H * S * D;
  uint16_t *q, *k, *v, *dO;
  float *l, *dd, *o, *dq, *dk, *dv;
  CK(hipMalloc(&q, n * 2)); CK(hipMalloc(&k, n * 2)); CK(hipMalloc(&v, n * 2)); CK(hipMalloc(&dO, n * 2));
  CK(hipMalloc(&o, n * 4)); CK(hipMalloc(&dq, n * 4)); CK(hipMalloc(&dk, n * 4)); CK(hipMalloc(&dv, n * 4));
  CK(hipMalloc(&l, (size_t)B * H * S * 4)); CK(hipMalloc(&dd, (size_t)B * H * S * 4));
  fill_rand16<<<1024, 256>>>(q, n, 1); fill_rand16<<<1024, 256>>>(k, n, 2);
  fill_rand16<<<1024, 256>>>(v, n, 3); fill_rand16<<<1024, 256>>>(dO, n, 4);
  fill_const32<<<1024, 256>>>(l, (size_t)B * H * S, 12.f);
  fill_const32<<<1024, 256>>>(dd, (size_t)B * H * S, 0.01f);
  mfa::BwdParams p;
  memset(&p, 0, sizeof(p));
  auto op = [&](const void* ptr) {
    mfa::Operand x;
    memset(&x, 0, sizeof(x));
    x.ptr = ptr; x.ss = D; x.sh = (int64_t)S * D; x.sb = (int64_t)H * S * D; x.sd = 1;
    x.prec = mfa::P_FP16; x.vec = 1; x.scale = 1.f; x.cols = D;
    return x;
  };
  p.q = op(q); p.k = op(k); p.v = op(v); p.dO_op = op(dO);
  p.o = o; p.l = l; p.l_f16 = 0; p.dD = dd; p.d_bf16 = 0;
  p.dq = dq; p.dk = dk; p.dv = dv;
  p.B = B; p.H = H; p.Hkv = H; p.R = S; p.C = S; p.D = D; p.group = 1;
  const float scale = 1.f / sqrtf((float)D);
  p.c_log2 = 1.442695041f * scale; p.scale = scale; p.dscale = scale; p.dq_mul = 1.f; p.dk_mul = 1.f;
  if (band > 0) {
    // Row q of every head keeps keys [128·c0, 128·(c0 + band)) with c0 centred on its block.
    const int nb = S / 128;
    std::vector<uint32_t> rg((size_t)B * H * S * 2);
    for (int bh = 0; bh < B * H; ++bh)
      for (int q = 0; q < S; ++q) {
        const int i = q / 128;
        const int c0 = std::min(std::max(0, i - band / 2), nb - band);
        rg[((size_t)bh * S + q) * 2] = 128u * c0;
        rg[((size_t)bh * S + q) * 2 + 1] = 128u * (c0 + band);
      }
    uint32_t* drg;
    CK(hipMalloc(&drg, rg.size() * 4));
    CK(hipMemcpy(drg, rg.data(), rg.size() * 4, hipMemcpyHostToDevice));
    p.mask.ranges = drg;
  }
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) CK(mfa::bwd_fast_dispatch(p, kind, mfa::P_FP16, D, st));
  CK(hipEventRecord(e0, st));
  for (int i = 0; i < 5; ++i) CK(mfa::bwd_fast_dispatch(p, kind, mfa::P_FP16, D, st));
  CK(hipEventRecord(e1, st));
  CK(hipStreamSynchronize(st));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  ms /= 5;
  const double fl = (qphase ? 6.0 : 8.0) * D * (double)S * S * B * H;  // 3 or 4 GEMMs
  printf("%s B=%d H=%d S=%d D=%d band=%d: %.3f ms, %.1f TFLOP/s executed\n", qphase ? "bwd_q" : "bwd_kv", B, H, S,
         D, band, ms, fl / (ms * 1e-3) / 1e12);
  std::vector<unsigned long long> st8(1 << 18);
  void* dsym;
  CK(hipGetSymbolAddress(&dsym, HIP_SYMBOL(mfa::g_mfa_bstamps)));
  CK(hipMemcpy(st8.data(), dsym, sizeof(unsigned long long) << 18, hipMemcpyDeviceToHost));
  const char* names_kv[8] = {"L/D + DMA issue", "S(+dP) chain", "dP chain|P", "dV chain+dS", "dK chain", "wait_vm", "barrier+ld", "prologue"};
  const char* names_q[8] = {"DMA issue", "S chain+mask", "dP chain+P", "dQ chain+dS", "wait_vm", "barrier", "dQ store", "prologue"};
  const char* const* names = qphase ? names_q : names_kv;
  double tot[8] = {0};
  int nw = 0;
  for (size_t w = 0; w < (1 << 14); ++w) {  // (the second half holds the prologue points)
    bool any = false;
    for (int s = 0; s < 8; ++s) any |= st8[w * 8 + s] != 0;
    if (!any) continue;
    ++nw;
    for (int s = 0; s < 8; ++s) tot[s] += (double)st8[w * 8 + s];
  }
  double all = 0;
  for (int s = 0; s < 8; ++s) all += tot[s];
  const int nsteps = band > 0 ? 1 : S / (D >= 256 ? 32 : 64);  // (BT and BQ agree per D)
  printf("waves %d; per wave %s (shader cycles); per-wave total %.0f cycles:\n", nw,
         band > 0 ? "in all" : "per step", all / nw);
  for (int s = 0; s < 8; ++s)
    printf("  %-14s %8.0f  (%.1f%%)\n", names[s], tot[s] / nw / (s == 7 || (qphase && s == 6) ? 1 : nsteps),
           100.0 * tot[s] / all);
  // Prologue points, cycles from the wave's first stamp (medians over waves): 0 pre-pass loads
  // and interval stores done, 1 row-range reduction done, 2 step flags done, 3 first tiles and
  // L/D issued, 4 their wait done.
  const char* pn_kv[7] = {"pre-pass rows", "reduction", "step flags", "first tiles issued", "first tiles landed",
                          "chunk 0 loads issued", "chunk 0 used"};
  // backwardQuery: 0 Q/dO fragment loads issued, 1 first K/V tile issued, 2 D summed (O read),
  // 3 L/D stored, 4 wait_vm done, 5 barrier before the loop done.
  const char* pn_q[7] = {"Q/dO loads issued", "first tile issued", "D summed", "L/D stored", "wait_vm done",
                         "loop entry", ""};
  const char* const* pn = qphase ? pn_q : pn_kv;
  for (int k = 0; k < 7; ++k) {
    std::vector<double> x;
    for (size_t w = 0; w < (1 << 14); ++w)
      if (st8[(1 << 17) + w * 8 + k]) x.push_back((double)st8[(1 << 17) + w * 8 + k]);
    if (x.empty()) continue;
    std::sort(x.begin(), x.end());
    printf("  prologue point %-20s med %8.0f  p90 %8.0f cycles\n", pn[k], x[x.size() / 2], x[x.size() * 9 / 10]);
  }
  return 0;
}
