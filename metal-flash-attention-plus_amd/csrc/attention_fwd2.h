// attention_fwd2.h — building blocks of the 16-bit tuned forwards (attention_fwd_v2.hip):
// per-wave row state, the three parts of one K/V tile (QK^T, softmax,
// PV), Q fragments and the O / L epilogue.  Semantics: attention_fwd_v2.hip's header.
#pragma once
#include <type_traits>

#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

// Diagnostic build only (tools/diag/fwd_stamps.hip defines MFA_STAMPS): per-wave s_memrealtime
// stamps (100 MHz) at phase boundaries, into a buffer no kernel output is computed from.
#ifdef MFA_STAMPS
__device__ unsigned long long g_mfa_stamps[1 << 20];
#define MFA_STAMP(slot)                                                                     \
  do {                                                                                      \
    const unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                          \
    if ((threadIdx.x & 63) == 0)                                                            \
      g_mfa_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + (slot)] = t_; \
  } while (0)
#define MFA_STAMP_DRAIN() asm volatile("s_waitcnt vmcnt(0)" ::: "memory")
// Shader-cycle counter at the kernel's start (slot 0) and end (slot 1) of each wave: with the
// s_memrealtime stamps this gives the clock the chip held during the kernel.
__device__ unsigned long long g_mfa_cyc[1 << 18];
#define MFA_CYC(slot)                                                                        \
  do {                                                                                       \
    const unsigned long long c_ = __builtin_amdgcn_s_memtime();                              \
    if ((threadIdx.x & 63) == 0)                                                             \
      g_mfa_cyc[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 2 + (slot)] = c_; \
  } while (0)
// Shader-cycle phase totals (slots 5..7 of the wave's record).
#define MFA_ACC_DECL() unsigned long long acc_[3] = {0, 0, 0}, acct_ = __builtin_amdgcn_s_memtime()
#define MFA_ACC(k)                                                  \
  do {                                                              \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();     \
    acc_[k] += t_ - acct_;                                          \
    acct_ = t_;                                                     \
  } while (0)
#define MFA_ACC_END()                                                                      \
  do {                                                                                     \
    if ((threadIdx.x & 63) == 0)                                                           \
      for (int k_ = 0; k_ < 3; ++k_)                                                       \
        g_mfa_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + 5 + k_] = acc_[k_]; \
  } while (0)
#else
#define MFA_CYC(slot) do {} while (0)
#define MFA_ACC_DECL() do {} while (0)
#define MFA_ACC(k) do {} while (0)
#define MFA_ACC_END() do {} while (0)
#define MFA_STAMP(slot) do {} while (0)
#define MFA_STAMP_DRAIN() do {} while (0)
#endif

// Scheduling knobs (development A/B; the defaults are the shipped configuration): fragment
// read-ahead for the QK^T and PV chains, MFMA-cluster priority, order pinning.
template <int AHK_ = 4, int AHV_ = 3, bool PRIO_ = false, bool PIN_ = true, bool SPREAD_ = false>
struct Tune {
  static constexpr int AHK = AHK_, AHV = AHV_;
  static constexpr bool PRIO = PRIO_, PIN = PIN_;
  static constexpr bool SPREAD = SPREAD_;  // next tile's DMA pieces between the QK^T MFMAs
};
using TuneDefault = Tune<>;

// Per-wave running state of 32 query rows (one per lane, halves split the head dimension).
template <int DP>
struct RowState {
  f32x16 o[DP / 32];
  f32x16 negm;   // −moff in every register (fp16 path): the QK^T chain's initial accumulator
  float m;       // running max (log2 units, reference convention)
  float moff;    // the max subtracted inside S' (== m once the row has seen an unmasked key)
  float lh;      // partial row sum of this half-wave's keys
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt) o[dt] = zero16();
    negm = zero16();
    m = -kFltMax;
    moff = 0.f;
    lh = 0.f;
  }
};

// One BK-key tile for one wave: S^T = K·Q^T (key in registers, query on the lane), masks,
// online softmax, O^T += V^T·P^T.
struct NoHook {
  __device__ __forceinline__ void operator()(int) const {}
};

// One tile in three parts: fwd2_qk (S^T = K·Q^T; S·c − moff on the fp16 path), fwd2_softmax
// (masks, online softmax, P packed as the PV B operand) and fwd2_pv (O^T += V^T·P^T).
// qk_hook(i) runs after QK^T MFMA i (e.g. staging the next tile piece by piece).
template <class E, int DP, int BK, class TU = TuneDefault, class QKHook = NoHook>
__device__ __forceinline__ void fwd2_qk(const char* kt, const int (&rbase)[2],
                                        const i16x8 (&qf)[DP / 16], const RowState<DP>& st,
                                        f32x16 (&s)[BK / 32], QKHook&& qk_hook = QKHook()) {
  using A = Arith16<E, DP>;
  // Pre-scaled Q, S' = S·c − moff from the MFMA (fp16 up to D=128: at D=256 the −m tile's
  // registers are worth more than the per-element multiply-add, which halves per MFMA there).
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, DS = DP / 16;
  constexpr int NM = DS * NJ;
  constexpr int AH = DP > 128 ? 2 : TU::AHK;
  i16x8 kf[AH];
#pragma unroll
  for (int i = 0; i < AH; ++i) kf[i] = A::read_row_a(kt, rbase, i % NJ, i / NJ);
  if constexpr (TU::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int ds = i / NJ, j = i % NJ;
    if (ds == 0)
      s[j] = A::mma(kf[i % AH], qf[0], PS ? st.negm : zero16());
    else
      s[j] = A::mma(kf[i % AH], qf[ds], s[j]);
    if (i + AH < NM) kf[i % AH] = A::read_row_a(kt, rbase, (i + AH) % NJ, (i + AH) / NJ);
    qk_hook(i);
    if constexpr (TU::PIN) __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (TU::PRIO) __builtin_amdgcn_s_setprio(0);
}

// fwd2_softmax in two parts, so a caller can place the exp / sum / pack work of one row block
// beside another block's MFMAs: fwd2_max (edge / causal / window masks, row max, the lazy
// rescale of O and l — a rarely taken branch) and fwd2_exp (P = exp2(S'), row sum, P packed
// as the PV B operand; straight-line code).
template <class E, int DP, int BK>
__device__ __forceinline__ void fwd2_max(RowState<DP>& st, f32x16 (&s)[BK / 32], int t,
                                         bool mask_tile, int qi, const FwdParams& p, float c,
                                         int wsz, int hh, int rlo = -0x40000000,
                                         int rhi = 0x3fffffff) {
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, ND = DP / 32;
  constexpr float THR = 8.0f;
  if (mask_tile) {
    MFA_KEEP_BRANCH();
    // Keys t + 4hh + kk stay for lo <= kk <= hi: below C, at most qi (causal), at least
    // qi - wsz (window), inside the row's sparse range [rlo, rhi].
    const int base = t + 4 * hh;
    int hi = min(p.C - 1, rhi) - base;
    if (p.mask.causal) hi = min(hi, qi - base);
    int lo = max(p.mask.window ? qi - wsz : -0x40000000, rlo);
    lo = lo <= -0x40000000 ? -0x40000000 : lo - base;
    mask_outside<NJ>(s, lo, hi, -__builtin_inff());
  }

  float mx = s[0][0];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[j][i]);
  mx = cross_half_max(mx);
  // Tile max in absolute log2 units.
  const float mt = PS ? mx + st.moff : mx * c;
  if (__any(mt > st.m + THR)) {
    MFA_KEEP_BRANCH();
    const float m_new = fmaxf(st.m, mt);
    const float corr = __builtin_amdgcn_exp2f(st.m - m_new);
    st.m = m_new;
    st.lh *= corr;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) st.o[dt][i] *= corr;
    if constexpr (PS) {
      // Rows still at the initial max saw only masked keys (S' = −inf): keep their offset.
      const float moff_new = m_new > kMaskLevel ? m_new : st.moff;
      const float shift = moff_new - st.moff;
      st.moff = moff_new;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) s[j][i] -= shift;
#pragma unroll
      for (int i = 0; i < 16; ++i) st.negm[i] = -moff_new;
    }
  }
}

template <class E, int DP, int BK>
__device__ __forceinline__ void fwd2_exp(RowState<DP>& st, f32x16 (&s)[BK / 32],
                                         i16x8 (&pb)[BK / 16], float c) {
  using A = Arith16<E, DP>;
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32;
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float x = PS ? s[j][i] : __builtin_fmaf(s[j][i], c, -st.m);
      const float pv = __builtin_amdgcn_exp2f(x);
      s[j][i] = pv;
      rs[i & 3] += pv;
    }
  st.lh += (rs[0] + rs[1]) + (rs[2] + rs[3]);
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) pb[j * 2 + ks] = A::pack(s[j], ks);
}

template <class E, int DP, int BK>
__device__ __forceinline__ void fwd2_softmax(RowState<DP>& st, f32x16 (&s)[BK / 32],
                                             i16x8 (&pb)[BK / 16], int t, bool mask_tile, int qi,
                                             const FwdParams& p, float c, int wsz, int hh,
                                             int rlo = -0x40000000, int rhi = 0x3fffffff) {
  fwd2_max<E, DP, BK>(st, s, t, mask_tile, qi, p, c, wsz, hh, rlo, rhi);
  fwd2_exp<E, DP, BK>(st, s, pb, c);
}

template <class E, int DP, int BK, class TU = TuneDefault, class PVHook = NoHook>
__device__ __forceinline__ void fwd2_pv(const char* vt, const int (&trb)[2],
                                        const i16x8 (&pb)[BK / 16], RowState<DP>& st,
                                        PVHook&& pv_hook = PVHook()) {
  using A = Arith16<E, DP>;
  constexpr int NJ = BK / 32, ND = DP / 32;
  constexpr int NM = NJ * 2 * ND;
  constexpr int AH = DP > 128 ? 2 : TU::AHV;
  i16x8 vf[AH];
#pragma unroll
  for (int i = 0; i < AH; ++i) {
    const int jk = i / ND, dt = i % ND;
    vf[i] = A::read_tr_a(vt, trb, (jk >> 1) * 32, jk & 1, dt * 32);
  }
  if constexpr (TU::PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int jk = i / ND, dt = i % ND;
    st.o[dt] = A::mma(vf[i % AH], pb[jk], st.o[dt]);
    if (i + AH < NM) {
      const int jn = (i + AH) / ND, dn = (i + AH) % ND;
      vf[i % AH] = A::read_tr_a(vt, trb, (jn >> 1) * 32, jn & 1, dn * 32);
    }
    pv_hook(i);
    if constexpr (TU::PIN) __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (TU::PRIO) __builtin_amdgcn_s_setprio(0);
}

template <class E, int DP, int BK, class TU = TuneDefault, class QKHook = NoHook>
__device__ __forceinline__ void fwd2_tile(const char* kt, const char* vt, const int (&rbase)[2],
                                          const int (&trb)[2], const i16x8 (&qf)[DP / 16],
                                          RowState<DP>& st, int t, bool mask_tile, int qi,
                                          const FwdParams& p, float c, int wsz, int hh,
                                          QKHook&& qk_hook = QKHook(), int rlo = -0x40000000,
                                          int rhi = 0x3fffffff) {
  f32x16 s[BK / 32];
  i16x8 pb[BK / 16];
  fwd2_qk<E, DP, BK, TU>(kt, rbase, qf, st, s, qk_hook);
  fwd2_softmax<E, DP, BK>(st, s, pb, t, mask_tile, qi, p, c, wsz, hh, rlo, rhi);
  fwd2_pv<E, DP, BK, TU>(vt, trb, pb, st);
}

// Q fragments of the lane's query row, pre-scaled by c (rounded to the element type) on the
// fp16 path.
// Q fragments in two halves so a caller can issue the loads early and scale them later
// (the pair kernel overlaps the next block's Q with the current block's merge and stores).
template <int DP>
__device__ __forceinline__ void load_q2_raw(i16x8 (&qf)[DP / 16], const FwdParams& p, int b,
                                            int h, int qi, bool qvalid, int hh) {
  const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh +
                         (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    const int d0 = 16 * s + 8 * hh;
    i16x8 v = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (qvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
    qf[s] = v;
  }
}

template <class E, int DP>
__device__ __forceinline__ void prescale_q2(i16x8 (&qf)[DP / 16], float c) {
  if constexpr (E::prec == P_FP16 && DP <= 128) {
#pragma unroll
    for (int s = 0; s < DP / 16; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[s][j] = (short)E::from_f32(E::to_f32((uint16_t)qf[s][j]) * c);
  }
}

template <class E, int DP>
__device__ __forceinline__ void load_q2(i16x8 (&qf)[DP / 16], const FwdParams& p, int b, int h,
                                        int qi, bool qvalid, int hh, float c) {
  load_q2_raw<DP>(qf, p, b, h, qi, qvalid, hh);
  prescale_q2<E, DP>(qf, c);
}

__device__ __forceinline__ void store_l(const FwdParams& p, float L, int b, int h, int qi) {
  const int64_t li = (int64_t)(b * p.H + h) * p.R + qi;
  if (p.l_f16)
    reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
  else
    reinterpret_cast<float*>(p.l)[li] = L;
}

// 16 bytes of O; NT: a non-temporal (streaming) store.  Only for whole-row stores (the O row
// image): O is written once, and the final drain of every CU at once is the mirrored kernel's
// tail (C2 +2.4-2.8 %).  Row-per-lane stores (16-32 B per row and instruction) lose with NT
// (C3 -4.9 %, C5 forward -11.5 %): their partial lines are no longer merged in L2.
template <bool NT>
__device__ __forceinline__ void st_o4(float* dst, float a, float b, float c, float d) {
  typedef float f4v __attribute__((ext_vector_type(4)));
  if constexpr (NT)
    __builtin_nontemporal_store(f4v{a, b, c, d}, reinterpret_cast<f4v*>(dst));
  else
    *reinterpret_cast<f4v*>(dst) = f4v{a, b, c, d};
}

// Rows [q0, q0 + NR) of an O row image (rows of DP floats at a pitch of ORS bytes) leave as
// 16-byte chunks from all NTH threads, thread t taking chunk t % CPR of rows t / CPR + k·NTH/CPR.
// Every image read is issued before the first store and, for a full block (all rows below R,
// D = DP), the stores are unguarded with the row address advanced by a constant: the guarded
// per-store form compiles to one read -> wait -> store round trip per chunk (~300 cycles each
// at the mirrored kernel's switch).
template <int DP, int NR, int NTH, bool NT>
__device__ __forceinline__ void store_o_image(const FwdParams& p, float* obase, const char* img,
                                              int ors, int q0, int tid, bool full) {
  constexpr int CPR = DP / 4, OST = NR * CPR / NTH, RPK = NTH / CPR;
  static_assert(NTH % CPR == 0 && NR * CPR % NTH == 0, "O image store geometry");
  const int r0 = tid / CPR, d = (tid % CPR) * 4;
  float4 v[OST];
#pragma unroll
  for (int k = 0; k < OST; ++k)
    v[k] = *reinterpret_cast<const float4*>(img + (k * RPK + r0) * ors + d * 4);
  if (full) {
    float* dst = obase + (int64_t)(q0 + r0) * p.o_ss + d;
    const int64_t step = (int64_t)RPK * p.o_ss;
#pragma unroll
    for (int k = 0; k < OST; ++k) st_o4<NT>(dst + k * step, v[k].x, v[k].y, v[k].z, v[k].w);
  } else {
#pragma unroll
    for (int k = 0; k < OST; ++k) {
      const int r = k * RPK + r0;
      if (q0 + r < p.R && d < p.D)
        st_o4<NT>(obase + (int64_t)(q0 + r) * p.o_ss + d, v[k].x, v[k].y, v[k].z, v[k].w);
    }
  }
}

template <int DP, bool NT = false>
__device__ __forceinline__ void store_o_l(const FwdParams& p, const f32x16 (&o)[DP / 32],
                                          float m, float l, int b, int h, int qi, int hh) {
  const float inv = p.o_mul / l;
  float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = dt * 32 + 8 * g + 4 * hh;
      if (d < p.D)
        st_o4<NT>(orow + d, o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
                  o[dt][4 * g + 3] * inv);
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

__device__ __forceinline__ void key_range(const FwdParams& p, int q0, int BQ, int BK, int* kbeg,
                                          int* kend) {
  *kend = p.C;
  if (p.mask.causal) *kend = min(*kend, q0 + BQ);
  *kbeg = 0;
  if (p.mask.window) {
    const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
    *kbeg = lo > 0 ? (int)(lo / BK) * BK : 0;
  }
}

}  // namespace mfa
