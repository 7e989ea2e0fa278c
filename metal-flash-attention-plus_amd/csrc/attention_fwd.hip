// attention_fwd.hip — fused attention forward for gfx950 (AttentionKernelType.forward).
//
// Semantics follow the reference generated kernel (AttentionKernel+Source.swift:372-416,
// AttentionKernel+Softmax.swift, AttentionKernel+Accumulate.swift:550-625,
// AttentionKernel+Caching.swift:318-400):
//   S = Q·K^T (+ additive mask); masked elements = (0.875/log2e)·(-FLT_MAX)
//   m_new = log2e·scale·max_j S_ij ; if m_new > m: corr = exp2(m - m_new), m = m_new
//   P = exp2(S·log2e·scale - m) ; l = l·corr + Σ P (l = FLT_MIN if !(l > 0))
//   O = O·corr + P·V ; O /= l at the end ; L = m + log2(l)        (m0 = -FLT_MAX, l0 = FLT_MIN)
//
// Structure (MI355X-native, not a translation of the Metal codegen): one workgroup = NW waves,
// each wave owns 32 queries.  Q stays in registers for the whole kernel; K/V tiles of BK keys
// are staged global->registers->LDS (double buffered, one barrier per tile).  Per tile a wave
// computes S^T = K·Q^T on MFMA (query on the lane, keys in registers), runs the online softmax
// in registers, and accumulates O^T += V^T·P^T directly from the S^T accumulator registers;
// V^T is read with ds_read_b64_tr_b16 from the row-major LDS image.  Causal and sliding-window
// tiles that are entirely masked are skipped (the reference computes and discards them,
// SURVEY.md §8a quirk 4 — results are identical because their P is exactly 0).
#include "mfa_stage.h"

namespace mfa {

template <class A, int DP, int BK, int NW, int KSRC, int VSRC>
__global__ void __launch_bounds__(NW * 64) mfa_fwd_kernel(FwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NW * 64;
  constexpr int BQ = NW * 32;
  constexpr int NJ = BK / 32;
  constexpr int TILEB = A::is_f32 ? BK * (DP + 1) * 4 : BK * DP * 2;
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int rb = p.nblk - 1 - bid / BH;  // heaviest (causal) query blocks dispatch first
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;

  typename A::frag qf[A::DSTEPS];
  load_row_frags<A, DP>(qf, p.q, b, h, qi, qvalid, hh, p.D);

  uint2 range = make_uint2(0u, 0u);
  if (p.mask.ranges && qvalid) {
    const uint32_t* rp = p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + qi);
    range = make_uint2(rp[0], rp[1]);
  }

  int kend = p.C;
  if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
  int kbeg = 0;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
    kbeg = lo > 0 ? (int)(lo / BK) * BK : 0;
  }

  f32x16 o[DP / 32];
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt) o[dt] = zero16();
  float m = -kFltMax, l = kFltMin;
  const float c = p.c_log2;

  Stager<A, BK, DP, NT, KSRC> sk;
  Stager<A, BK, DP, NT, VSRC> sv;
  if (kbeg < kend) {
    sk.load(p.k, b, kvh, kbeg, p.C, p.D);
    sv.load(p.v, b, kvh, kbeg, p.C, p.D);
    sk.store(kb0, p.k, b, kvh, kbeg, p.C, p.D);
    sv.store(vb0, p.v, b, kvh, kbeg, p.C, p.D);
  }
  __syncthreads();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool has_next = t + BK < kend;
    if (has_next) {
      sk.load(p.k, b, kvh, t + BK, p.C, p.D);
      sv.load(p.v, b, kvh, t + BK, p.C, p.D);
    }
    const char* kt = kb0 + cur * TILEB;
    const char* vt = vb0 + cur * TILEB;

    // S^T = K·Q^T : query on the lane, 32 keys per accumulator.
    f32x16 s[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) s[j] = zero16();
#pragma unroll
    for (int ds = 0; ds < A::DSTEPS; ++ds) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        s[j] = A::mma(A::read_row(kt, j * 32 + l32, ds, hh), qf[ds], s[j]);
    }

    const bool need_mask = (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) ||
                           p.mask.window || p.mask.ranges || p.mask.amask;
    if (need_mask) apply_masks<NJ>(s, t, qi, hh, p, b, h, range);

    // Online softmax (base 2).
    float mx = s[0][0];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[j][i]);
    mx = xhalf_max(mx);
    const float m_new = mx * c;
    float corr = 1.f;
    if (m_new > m) {
      corr = __builtin_amdgcn_exp2f(m - m_new);
      m = m_new;
    }
    float rs = 0.f;
    if (__any(m < kMaskLevel)) {
      // A row still masked everywhere: m = round(mask·c), so P must use the same rounded
      // product (a fused multiply-add leaves a ~1e31 residual and exp2 overflows).
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(mul_rn(s[j][i], c) - m);
          s[j][i] = pv;
          rs += pv;
        }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(s[j][i] * c - m);
          s[j][i] = pv;
          rs += pv;
        }
    }
    rs = xhalf_sum(rs);
    l = l * corr + rs;
    if (!(l > 0.f)) l = kFltMin;
    if (__any(corr != 1.f)) {
#pragma unroll
      for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= corr;
    }

    // O^T += V^T · P^T
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag pb = A::pack(s[j], ks);
#pragma unroll
        for (int dt = 0; dt < DP / 32; ++dt)
          o[dt] = A::mma(A::read_tr(vt, j * 32, ks, dt * 32, lane), pb, o[dt]);
      }
    }

    if (has_next) {
      sk.store(kb0 + (cur ^ 1) * TILEB, p.k, b, kvh, t + BK, p.C, p.D);
      sv.store(vb0 + (cur ^ 1) * TILEB, p.v, b, kvh, t + BK, p.C, p.D);
    }
    __syncthreads();
    cur ^= 1;
  }

  // Epilogue: O = O / l (fast::divide(1, l) on the last iteration), L = m + log2(l).
  if (qvalid) {
    const float inv = p.o_mul / l;
    float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
    const bool ovec = p.o_sd == 1 && (p.o_ss & 3) == 0 && (p.D & 3) == 0;
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        const float4 val = make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv,
                                       o[dt][4 * g + 2] * inv, o[dt][4 * g + 3] * inv);
        if (p.o_sd != 1) {  // transposed O: element (qi, d) at d * o_sd
          if (d < p.D) orow[(int64_t)d * p.o_sd] = val.x;
          if (d + 1 < p.D) orow[(int64_t)(d + 1) * p.o_sd] = val.y;
          if (d + 2 < p.D) orow[(int64_t)(d + 2) * p.o_sd] = val.z;
          if (d + 3 < p.D) orow[(int64_t)(d + 3) * p.o_sd] = val.w;
        } else if (d + 4 <= p.D && ovec) {
          *reinterpret_cast<float4*>(orow + d) = val;
        } else {
          if (d < p.D) orow[d] = val.x;
          if (d + 1 < p.D) orow[d + 1] = val.y;
          if (d + 2 < p.D) orow[d + 2] = val.z;
          if (d + 3 < p.D) orow[d + 3] = val.w;
        }
      }
    }
    if (hh == 0) {
      const float L = m + __log2f(l);
      const int64_t li = (int64_t)(b * p.H + h) * p.R + qi;
      if (p.l_f16)
        reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
      else
        reinterpret_cast<float*>(p.l)[li] = L;
    }
  }
}

// ---------------------------------------------------------------------------------------
// Host-visible launcher table.  Each (element type, padded head dim, K/V source) pair is one
// instantiation; block sizes per instantiation are fixed here and reported to the plan.
template <class A, int DP, int BK, int NW, int KSRC, int VSRC>
static hipError_t launch_fwd(const FwdParams& p, hipStream_t stream) {
  constexpr int TILEB = A::is_f32 ? BK * (DP + 1) * 4 : BK * DP * 2;
  constexpr int LDS = 4 * TILEB;
  auto kern = mfa_fwd_kernel<A, DP, BK, NW, KSRC, VSRC>;
  const int grid = p.nblk * p.B * p.H;
  return launch(kern, dim3(grid), dim3(NW * 64), LDS, stream, p);
}

}  // namespace mfa

#include "mfa_dispatch.h"

namespace mfa {

// Block configuration per (element kind, padded head dim): see mfa_dispatch.h.
hipError_t fwd_dispatch(const FwdParams& p, int elem, int DP, int ksrc, int vsrc,
                        hipStream_t stream) {
#define MFA_FWD_CASE(ELEM, DPV, KS, VS)                                                   \
  if (elem == ELEM && DP == DPV && ksrc == KS && vsrc == VS)                              \
    return launch_fwd<typename ArithOf<ELEM, DPV>::type, DPV, FwdCfg<ELEM, DPV>::BK,        \
                      FwdCfg<ELEM, DPV>::NW, KS, VS>(p, stream);
#define MFA_FWD_DPS(ELEM, KS, VS)                                                         \
  MFA_FWD_CASE(ELEM, 32, KS, VS)                                                          \
  MFA_FWD_CASE(ELEM, 64, KS, VS)                                                          \
  MFA_FWD_CASE(ELEM, 128, KS, VS)                                                         \
  MFA_FWD_CASE(ELEM, 256, KS, VS)
  MFA_FWD_DPS(P_FP16, SRC_SAME, SRC_SAME)
  MFA_FWD_DPS(P_FP16, SRC_I8, SRC_I8)
  MFA_FWD_DPS(P_FP16, SRC_I4, SRC_I4)
  MFA_FWD_DPS(P_BF16, SRC_SAME, SRC_SAME)
  MFA_FWD_DPS(P_BF16, SRC_I8, SRC_I8)
  MFA_FWD_DPS(P_BF16, SRC_I4, SRC_I4)
  MFA_FWD_DPS(P_FP32, SRC_SAME, SRC_SAME)
#undef MFA_FWD_DPS
#undef MFA_FWD_CASE
  return hipErrorInvalidValue;
}

}  // namespace mfa
