// attention_fwd_v2.hip — second-generation forward for 16-bit operands on gfx950.
//
// Same algorithm and numerics contract as attention_fwd.hip (the reference forward,
// AttentionKernel+Source.swift:372-416: S = QK^T, base-2 online softmax, O = PV / l,
// L = m + log2 l), restricted to fp16/bf16 Q/K/V with contiguous 16-byte aligned rows,
// D % 8 == 0, D <= DP ∈ {64, 128, 256}, a positive softmax scale, and at most causal /
// sliding-window masks whose fully masked tiles may be skipped (so no row is masked
// everywhere).  The host routes everything else to the other kernels.
//
// What is different from attention_fwd_fast.hip, all aimed at the VALU work per MFMA (the
// binding limit of that kernel):
//   * K/V tiles land by LDS-DMA in the sub-tiled TileA image, so every fragment read is a base
//     register plus an immediate (no per-read address arithmetic);
//   * fp16: Q is pre-scaled by c = scale·log2(e) in registers and the first QK^T MFMA of each
//     chain accumulates onto a register tile holding −m (the running row max), so the MFMA
//     output already is S·c − m and P = exp2(S') needs no subtract or multiply per element.
//     (bf16 keeps the fused multiply-add: pre-scaling would round Q·c to 8 bits.);
//   * built with MFMA accumulators in VGPRs (Makefile): the in-loop O rescale would otherwise
//     make hipcc copy all of O between AGPRs and VGPRs every iteration; D=256 then fits in
//     244 registers and runs two waves per SIMD;
//   * masked scores are −inf: with no fully masked row the reference's finite mask value and
//     −inf give the same P (exactly 0) and the same O and L.
// Lazy rescaling (threshold 8 in log2 units, cdna_hip_programming.md T13) is kept: the running
// max and the −m tile change only when a tile's max exceeds m + 8.
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

template <class E, int DP, int BK>
__device__ __forceinline__ void fwd2_softmax(RowState<DP>& st, f32x16 (&s)[BK / 32],
                                             i16x8 (&pb)[BK / 16], int t, bool mask_tile, int qi,
                                             const FwdParams& p, float c, int wsz, int hh) {
  using A = Arith16<E, DP>;
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, ND = DP / 32;
  constexpr float THR = 8.0f;
  if (mask_tile) {
    MFA_KEEP_BRANCH();
    // Keys t + 4hh + kk stay for lo <= kk <= hi: below C, at most qi (causal), at least
    // qi - wsz (window).
    const int base = t + 4 * hh;
    int hi = p.C - 1 - base;
    if (p.mask.causal) hi = min(hi, qi - base);
    const int lo = p.mask.window ? qi - wsz - base : -0x40000000;
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

template <class E, int DP, int BK, class TU = TuneDefault>
__device__ __forceinline__ void fwd2_pv(const char* vt, const int (&trb)[2],
                                        const i16x8 (&pb)[BK / 16], RowState<DP>& st) {
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
    if constexpr (TU::PIN) __builtin_amdgcn_sched_barrier(0);
  }
  if constexpr (TU::PRIO) __builtin_amdgcn_s_setprio(0);
}

template <class E, int DP, int BK, class TU = TuneDefault, class QKHook = NoHook>
__device__ __forceinline__ void fwd2_tile(const char* kt, const char* vt, const int (&rbase)[2],
                                          const int (&trb)[2], const i16x8 (&qf)[DP / 16],
                                          RowState<DP>& st, int t, bool mask_tile, int qi,
                                          const FwdParams& p, float c, int wsz, int hh,
                                          QKHook&& qk_hook = QKHook()) {
  f32x16 s[BK / 32];
  i16x8 pb[BK / 16];
  fwd2_qk<E, DP, BK, TU>(kt, rbase, qf, st, s, qk_hook);
  fwd2_softmax<E, DP, BK>(st, s, pb, t, mask_tile, qi, p, c, wsz, hh);
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

// ---------------------------------------------------------------------------------------
// One 128-row query block per workgroup (4 waves x 32 rows); WPS workgroups' waves per SIMD.
template <class E, int DP, int BK, int WPS, class TU = TuneDefault>
__global__ void __launch_bounds__(256, WPS) mfa_fwd2_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128;
  constexpr int TILEB = BK * DP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  // Causal: heaviest blocks first over the whole grid (balance); otherwise each head's blocks
  // together on one XCD (L2 reuse of its K/V).
  int bh, blk;
  if (p.mask.causal) {
    bh = blockIdx.x % (p.B * p.H);
    blk = blockIdx.x / (p.B * p.H);
  } else {
    xcd_unit_block(blockIdx.x, p.B * p.H, p.nblk, &bh, &blk);
  }
  const int rb = p.nblk - 1 - blk;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  MFA_STAMP(0);
  MFA_CYC(0);
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  int kbeg, kend;
  key_range(p, q0, BQ, BK, &kbeg, &kend);
  DmaA<DP, BK, NT> kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;
  if (kbeg < kend) {
    kd.issue(khead, kbeg, kb0);
    vd.issue(vhead, kbeg, vb0);
  }
  i16x8 qf[DP / 16];
  load_q2<E, DP>(qf, p, b, h, qi, qvalid, hh, c);
  RowState<DP> st;
  st.init();
  wait_vm();
  __syncthreads();
  MFA_STAMP(1);
  MFA_ACC_DECL();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool nxt = t + BK < kend;
    if (!TU::SPREAD && nxt) {
      kd.issue(khead, t + BK, kb0 + (cur ^ 1) * TILEB);
      vd.issue(vhead, t + BK, vb0 + (cur ^ 1) * TILEB);
    }
    MFA_ACC(0);
    auto hook = [&](int i) {
      if constexpr (TU::SPREAD) {
        constexpr int PPW = DmaA<DP, BK, NT>::PPW;
        if ((i & 1) == 0 && i / 2 < 2 * PPW && nxt) {
          const int k = i / 2;
          if (k < PPW)
            kd.issue_piece(khead, t + BK, kb0 + (cur ^ 1) * TILEB, k);
          else
            vd.issue_piece(vhead, t + BK, vb0 + (cur ^ 1) * TILEB, k - PPW);
        }
      }
    };
    const bool mask_tile = (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) || p.mask.window;
    fwd2_tile<E, DP, BK, TU>(kb0 + cur * TILEB, vb0 + cur * TILEB, rbase, trb, qf, st, t, mask_tile,
                         qi, p, c, wsz, hh, hook);
    MFA_ACC(1);
    wait_vm();
    __syncthreads();
    MFA_ACC(2);
    cur ^= 1;
  }
  MFA_ACC_END();

  MFA_STAMP(2);
  float l = cross_half_sum(st.lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if (qvalid) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
  MFA_STAMP(3);
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(4);
}

// ---------------------------------------------------------------------------------------
// Causal balance: two groups of NWG waves.  A workgroup owns the mirrored pair of query
// blocks (i, nblk-1-i) of NWG*32 rows (equal causal work per workgroup); inside each block
// group 0 takes the first half of the key tiles and group 1 the second half, and the two
// partial softmax states (O, m, l) merge through LDS before group 0 stores the block.
// NWG = 4: one 512-thread workgroup per CU; NWG = 2 (64-row blocks, BK = 32): two
// independent 256-thread workgroups per CU, whose waves are not tied by a shared barrier.

// OVL: the seam between the two blocks overlaps.  The staging ring is laid out slot-major
// (slot 0 of both groups in [0, 4*TILEB), slot 1 in [4*TILEB, 8*TILEB)), so once the first
// block's loop ends, the second block's first K/V tiles and its Q fragments are issued into
// slot 0 and registers before the merge, which runs over slot 1 and beyond; block two then
// waits with a counted vmcnt that leaves block one's O stores in flight.
template <class E, int DP, int BK, int NWG, bool OVL>
__global__ void __launch_bounds__(NWG * 128, 2) mfa_fwd2_pair_kernel(FwdParams p) {
  constexpr int NT = NWG * 64, BQ = NWG * 32, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int CPR = DP / 4;                        // 16-byte O chunks per row
  constexpr int OST = BQ * CPR / (2 * NT);           // O stores per thread per block
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / NT);
  const int gt = tid % NT;
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  // K of ring slot s at kb0 + s * SLOT, V at vb0 + s * SLOT.
  constexpr int SLOT = OVL ? 4 * TILEB : TILEB;
  char* const kb0 = smem + (OVL ? g * 2 * TILEB : g * 4 * TILEB);
  char* const vb0 = kb0 + (OVL ? TILEB : 2 * TILEB);
  char* const mbase = smem + (OVL ? 4 * TILEB : 0);  // merge area / O row image

  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int pi = bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;
  MFA_STAMP(0);
  MFA_CYC(0);

  DmaA<DP, BK, NT> kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, gt);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, gt);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;

  // This group's key range [t0, t1) of query block rb and the shared step count nA.
  auto range = [&](int rb, int& t0, int& t1, int& nA) {
    int kbeg, kend;
    key_range(p, rb * BQ, BQ, BK, &kbeg, &kend);
    const int ntile = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    nA = (ntile + 1) / 2;
    t0 = g == 0 ? kbeg : kbeg + nA * BK;
    t1 = g == 0 ? min(kend, kbeg + nA * BK) : kend;
  };

  const int rbA = pi, rbB = p.nblk - 1 - pi;
  i16x8 qf[DP / 16];
  int t0, t1, nA;
  range(rbB, t0, t1, nA);
  if (t0 < t1) {
    kd.issue(khead, t0, kb0);
    vd.issue(vhead, t0, vb0);
  }
  load_q2_raw<DP>(qf, p, b, h, rbB * BQ + wg * 32 + l32, rbB * BQ + wg * 32 + l32 < p.R, hh);
  bool counted = false;  // this block's loads were issued before the previous block's stores
  for (int which = 0; which < 2; ++which) {
    const int rb = which == 0 ? rbB : rbA;
    if (which == 1 && rbA >= rbB) break;  // odd middle block handled once
    const int q0 = rb * BQ;
    const int qi = q0 + wg * 32 + l32;
    const bool qvalid = qi < p.R;
    if (!OVL && which == 1) {
      if (t0 < t1) {
        kd.issue(khead, t0, kb0);
        vd.issue(vhead, t0, vb0);
      }
      load_q2_raw<DP>(qf, p, b, h, qi, qvalid, hh);
    }
    // Older than the (at most OST + 1) stores the previous block left in flight.
    if (OVL && counted)
      __builtin_amdgcn_s_waitcnt(0x0F70 | (OST & 15) | ((OST >> 4) << 14));
    else
      wait_vm();
    prescale_q2<E, DP>(qf, c);
    RowState<DP> st;
    st.init();
    __syncthreads();
    MFA_STAMP(1 + 3 * which);
    int cur = 0;
    for (int step = 0; step < nA; ++step) {
      const int t = t0 + step * BK;
      if (t < t1) {
        if (t + BK < t1) {
          kd.issue(khead, t + BK, kb0 + (cur ^ 1) * SLOT);
          vd.issue(vhead, t + BK, vb0 + (cur ^ 1) * SLOT);
        }
        const bool mask_tile =
            (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) || p.mask.window;
        fwd2_tile<E, DP, BK>(kb0 + cur * SLOT, vb0 + cur * SLOT, rbase, trb, qf, st, t,
                             mask_tile, qi, p, c, wsz, hh);
        wait_vm();
      }
      __syncthreads();
      cur ^= 1;
    }

    MFA_STAMP(2 + 3 * which);
    if (which == 0) {
      range(rbA, t0, t1, nA);
      if (OVL && rbA < rbB) {
        // Every wave passed the loop's last barrier: slot 0 is free for the next block.
        if (t0 < t1) {
          kd.issue(khead, t0, kb0);
          vd.issue(vhead, t0, vb0);
        }
        const int nqi = rbA * BQ + wg * 32 + l32;
        load_q2_raw<DP>(qf, p, b, h, nqi, nqi < p.R, hh);
        // Full block: every wave issues exactly OST O stores after these loads (and group 0
        // one L store before them), so a counted wait covers the loads.
        counted = q0 + BQ <= p.R && p.D == DP;
        __asm__ __volatile__("" ::: "memory");  // keep the loads ahead of the stores
      }
    }
    // Merge group 1's partial state into group 0 through LDS.
    float* mrg = reinterpret_cast<float*>(mbase);       // [NWG waves][ND*16][64]
    float* mml = mrg + NWG * ND * 16 * 64;              // [NWG waves][2][64]
    if (g == 1) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mrg[((wg * ND + dt) * 16 + i) * 64 + lane] = st.o[dt][i];
      mml[(wg * 2 + 0) * 64 + lane] = st.m;
      mml[(wg * 2 + 1) * 64 + lane] = st.lh;
    }
    __syncthreads();
    float inv = 0.f;
    if (g == 0) {
      const float mb = mml[(wg * 2 + 0) * 64 + lane];
      const float lb = mml[(wg * 2 + 1) * 64 + lane];
      const float mf = fmaxf(st.m, mb);
      const float ca = __builtin_amdgcn_exp2f(st.m - mf);
      const float cb = __builtin_amdgcn_exp2f(mb - mf);
      float l = cross_half_sum(st.lh * ca + lb * cb) + kFltMin;
      if (!(l > 0.f)) l = kFltMin;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          st.o[dt][i] = st.o[dt][i] * ca + mrg[((wg * ND + dt) * 16 + i) * 64 + lane] * cb;
      inv = p.o_mul / l;
      if (hh == 0 && qvalid) store_l(p, mf + __log2f(l), b, h, qi);
    }
    __syncthreads();
    // O leaves through LDS as whole rows (T21): group 0 writes its lanes' rows into a padded
    // [BQ][DP] fp32 image over the (now free) merge area, then all 2·NT threads store 16-byte
    // chunks along the rows, one wave instruction covering 1 KiB of consecutive O bytes
    // instead of 64 rows x 16 B.
    constexpr int ORS = DP * 4 + 16;  // padded row stride (bytes): conflict-free b128 writes
    if (g == 0) {
      char* orow = mbase + (wg * 32 + l32) * ORS;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
              make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                          st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
    }
    __syncthreads();
    {
      float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
      for (int k = 0; k < OST; ++k) {
        const int idx = k * 2 * NT + tid;
        const int r = idx / CPR, d = (idx % CPR) * 4;
        if (q0 + r < p.R && d < p.D)
          *reinterpret_cast<float4*>(obase + (int64_t)(q0 + r) * p.o_ss + d) =
              *reinterpret_cast<const float4*>(mbase + r * ORS + d * 4);
      }
    }
    __syncthreads();
    MFA_STAMP(3 + 3 * which);
  }
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(7);
}

// ---------------------------------------------------------------------------------------
// Causal balance with shared K/V tiles ("share" schedule, no window).  The workgroup owns the
// mirrored pair of 128-row blocks A (light, pi: nA key tiles) and B (heavy, nblk-1-pi: nB
// tiles).  A's keys are the first nA of B's, so:
//   phase 1 (steps 0..nA-1): one tile per step, staged by all 8 waves and read by both
//     groups — group 0 (waves 0-3) with A's rows, group 1 (waves 4-7) with B's rows.  Half
//     the K/V bytes and DMA instructions of the pair kernel for these steps;
//   phase 2: B's remaining nB - nA tiles, split between the groups (each with its own ring,
//     one tile each per step, as in the pair kernel).  Group 0 enters it with B's rows: it
//     stores A's O and L from registers at the switch and takes B's Q from LDS, where it
//     staged them by DMA during the last shared step.
// Steps: nA + ceil((nB - nA) / 2) — 33 for every workgroup at C2, as in the pair kernel.  B's
// two partial states merge through LDS at the end.  LDS: ring 0 (shared, then group 0's),
// ring 1 (group 1's), group 0's Q staging: 160 KiB at D = 128.
// MIRROR = false (no mask): the pair is two adjacent blocks (2·pi, 2·pi + 1) with the same key
// range, so every step is a shared one (256 query rows per K/V tile).
// IMG: adjacent pairs — both blocks' O through LDS row images; mirrored pairs — A's O at the
// switch through the wave's Q staging region.
// DV (mirrored pairs with nA >= 2): the prologue waits for K0 and Q only — Q arrives by
// LDS-DMA like the tiles (group 0 into the Q staging, group 1 into ring 1, unused before
// phase 2) so that every prologue load is counted by hand — and step 0 waits for V0 between
// its softmax and its PV.
template <class E, int DP, int BK, bool MIRROR, bool NTS = false, bool IMG = false, bool DV = false>
__global__ void __launch_bounds__(512, 2) mfa_fwd2_share_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int QW = 32 * DP * 2;                    // one wave's 32 Q rows
  constexpr int CPR = DP / 4;                        // 16-byte O chunks per row
  constexpr int OST = BQ * CPR / (2 * NT);           // O stores per thread (final block)
  constexpr int NSW = 4 * ND + 1;                    // stores per wave at the switch (O + L)
  static_assert(NSW < 64, "counted vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / NT);
  const int gt = tid % NT;
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  char* const sk = smem;                  // ring 0: K slots 0, 1, then V slots 0, 1
  char* const sv = smem + 2 * TILEB;
  char* const kb0 = smem + g * 4 * TILEB; // this group's ring in phase 2
  char* const vb0 = kb0 + 2 * TILEB;
  char* const qstg = smem + 8 * TILEB + wg * QW;

  const int BH = p.B * p.H;
  const int pi = blockIdx.x / BH;
  const int bh = blockIdx.x % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = 0x3fffffff;

  DmaA<DP, BK, NT> kd, vd;         // a group's own tiles
  DmaA<DP, BK, 2 * NT> ksh, vsh;   // shared tiles, staged by all 8 waves
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, gt);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, gt);
  ksh.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vsh.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;

  // Adjacent pairs: an odd last block leaves group 1 without rows (it still stages tiles).
  const int rbA = MIRROR ? pi : 2 * pi;
  const int rbB = MIRROR ? p.nblk - 1 - pi : 2 * pi + 1;
  int a0, a1, b0, b1;
  key_range(p, rbA * BQ, BQ, BK, &a0, &a1);
  key_range(p, MIRROR ? rbB * BQ : rbA * BQ, BQ, BK, &b0, &b1);
  const int nB = b1 > b0 ? (b1 - b0 + BK - 1) / BK : 0;
  // Mirrored: the odd middle block is B only.
  const int nA = !MIRROR ? nB : rbA < rbB && a1 > a0 ? (a1 - a0 + BK - 1) / BK : 0;
  const int n2 = nB - nA;            // phase-2 tiles
  const int h0 = (n2 + 1) / 2;       // group 0's share of them
  const int S = nA + h0;
  // Tile index of this group at step s (group 0: s; group 1: s, then s + h0); false past its
  // range.
  auto tile = [&](int s, int& t) -> bool {
    const int i = (g == 1 && s >= nA) ? s + h0 : s;
    t = b0 + i * BK;
    return s < S && i < nB;
  };

  int q0 = (g == 0 && nA > 0 ? rbA : rbB) * BQ;
  int qi = q0 + wg * 32 + l32;
  i16x8 qf[DP / 16];
  DmaA<DP, 32, 64> qd;  // this wave's 32 Q rows (group 0: B's, staged for the switch)
  qd.init((int)p.q.ss * 2, p.R, p.D * 2, lane);
  const char* qhead = (const char*)p.q.ptr + ((int64_t)b * p.q.sb + (int64_t)h * p.q.sh) * 2;
  RowState<DP> st;
  st.init();
  const bool dv = DV && nA >= 2;
  if (dv) {
    char* const qdst = g == 0 ? qstg : smem + 4 * TILEB + wg * QW;
    ksh.issue(khead, b0, sk);
    qd.issue(qhead, q0 + wg * 32, qdst);
    vsh.issue(vhead, b0, sv);
    constexpr int PV0 = DmaA<DP, BK, 2 * NT>::PPW;  // V0 pieces per wave (the youngest)
    __builtin_amdgcn_s_waitcnt(0x0F70 | PV0);
    __syncthreads();
    using A = Arith16<E, DP>;
#pragma unroll
    for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(qdst, rbase, 0, ds);
    prescale_q2<E, DP>(qf, c);
  } else {
    if (nA > 0) {
      ksh.issue(khead, b0, sk);
      vsh.issue(vhead, b0, sv);
    } else {
      int t;
      if (tile(0, t)) {
        kd.issue(khead, t, kb0);
        vd.issue(vhead, t, vb0);
      }
    }
    load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
    wait_vm();
    prescale_q2<E, DP>(qf, c);
    __syncthreads();
  }

  const bool full_sw = rbA * BQ + BQ <= p.R && p.D == DP;  // every switch store is issued
  auto step = [&](int s, bool sw, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;  // step 0 of the deferred-V prologue
    // Stage the next step's tile(s) into the slot read two steps ago.
    const int nx = (s + 1) & 1;
    if (s + 1 < nA) {
      ksh.issue(khead, b0 + (s + 1) * BK, sk + nx * TILEB);
      vsh.issue(vhead, b0 + (s + 1) * BK, sv + nx * TILEB);
    } else {
      int tn;
      if (tile(s + 1, tn)) {
        kd.issue(khead, tn, kb0 + nx * TILEB);
        vd.issue(vhead, tn, vb0 + nx * TILEB);
      }
    }
    if (sw) {
      // A is complete: its O and L leave from registers (the next tiles' DMA is older than
      // these stores, so the step's counted wait below leaves them in flight).
      float l = cross_half_sum(st.lh) + kFltMin;
      if (!(l > 0.f)) l = kFltMin;
      using A = Arith16<E, DP>;
      if constexpr (MIRROR && IMG) {
        // B's Q rows first (this wave's staging region is then free), then A's O leaves
        // through that region in two column halves: the wave writes its 32 rows (row per
        // lane, 16-byte chunks XOR-swizzled by row) and reads them back as whole half-rows,
        // so each store instruction covers 4 rows x DP*2 contiguous bytes (row-per-lane stores
        // touched 32 rows x 32 B); wave-private, so no barrier.  Same store count (NSW).
        char* const wreg = qstg;  // this wave's staging region
#pragma unroll
        for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(wreg, rbase, 0, ds);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): Q is in registers
        constexpr int HB = DP * 2, NCH = DP / 8;  // bytes and 16-byte chunks per half-row
        const float inv = p.o_mul / l;
        const int qa0 = q0 + wg * 32;
        float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int dt = 0; dt < ND / 2; ++dt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
              const int cch = dt * 8 + 2 * gq + hh;
              const f32x16& o = st.o[half * (ND / 2) + dt];
              *reinterpret_cast<float4*>(wreg + l32 * HB + ((cch ^ (l32 & (NCH - 1))) * 16)) =
                  make_float4(o[4 * gq] * inv, o[4 * gq + 1] * inv, o[4 * gq + 2] * inv,
                              o[4 * gq + 3] * inv);
            }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          constexpr int RPI = 64 / NCH;  // rows per read instruction
#pragma unroll
          for (int k = 0; k < 32 / RPI; ++k) {
            const int r = k * RPI + lane / NCH, j = lane % NCH;
            const float4 v =
                *reinterpret_cast<const float4*>(wreg + r * HB + ((j ^ (r & (NCH - 1))) * 16));
            const int col = half * (DP / 2) + 4 * j;
            if (qa0 + r < p.R && col < p.D)
              st_o4<NTS>(obase + (int64_t)(qa0 + r) * p.o_ss + col, v.x, v.y, v.z, v.w);
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);  // reads done before the next half's writes
        }
        if (hh == 0 && qi < p.R) store_l(p, st.m + __log2f(l), b, h, qi);
        __asm__ __volatile__("" ::: "memory");
        q0 = rbB * BQ;
        qi = q0 + wg * 32 + l32;
      } else {
        if (qi < p.R) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
        __asm__ __volatile__("" ::: "memory");
        q0 = rbB * BQ;
        qi = q0 + wg * 32 + l32;
#pragma unroll
        for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(qstg, rbase, 0, ds);
      }
      prescale_q2<E, DP>(qf, c);
      st.init();
    }
    int tc;
    if (tile(s, tc)) {
      const bool shared = s < nA;
      const char* kt = (shared ? sk : kb0) + (s & 1) * TILEB;
      const char* vt = (shared ? sv : vb0) + (s & 1) * TILEB;
      const bool mask_tile = (tc + BK > p.C) || (p.mask.causal && tc + BK - 1 > q0);
      if constexpr (FIRST) {
        // V0 is older than the next shared tile's pieces issued above.
        constexpr int NPN = 2 * DmaA<DP, BK, 2 * NT>::PPW;
        f32x16 sc[BK / 32];
        i16x8 pb[BK / 16];
        fwd2_qk<E, DP, BK>(kt, rbase, qf, st, sc);
        fwd2_softmax<E, DP, BK>(st, sc, pb, tc, mask_tile, qi, p, c, wsz, hh);
        __builtin_amdgcn_s_waitcnt(0x0F70 | NPN);
        __syncthreads();
        fwd2_pv<E, DP, BK>(vt, trb, pb, st);
      } else {
        fwd2_tile<E, DP, BK>(kt, vt, rbase, trb, qf, st, tc, mask_tile, qi, p, c, wsz, hh);
      }
    }
    if (sw && full_sw)
      __builtin_amdgcn_s_waitcnt(0x0F70 | (NSW & 15) | ((NSW >> 4) << 14));
    else
      wait_vm();
    __syncthreads();
  };
  // Phase 1 up to its last step, which also stages B's Q rows; group 0 switches at step nA.
  int s = 0;
  using F0 = std::false_type;
  if (dv) step(s++, false, std::true_type());
  for (; s < nA - 1; ++s) step(s, false, F0());
  if (nA > 0 && n2 > 0) {
    if (g == 0) qd.issue(qhead, rbB * BQ + wg * 32, qstg);
    step(s++, false, F0());
    step(s++, g == 0, F0());
  }
  for (; s < S; ++s) step(s, false, F0());

  char* const mbase = smem;  // the rings are free: merge area, then the O row image
  if (n2 == 0) {
    // Group 0 holds all of A (if any), group 1 all of B: no merge.
    float l = cross_half_sum(st.lh) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    if constexpr (!MIRROR && IMG) {
      // Adjacent pairs: both blocks leave through O row images (one per group, over the free
      // ring) as whole rows from all 8 waves.
      constexpr int ORS = DP * 4 + 16;
      const float inv = p.o_mul / l;
      char* orow = smem + (g * 128 + wg * 32 + l32) * ORS;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
              make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                          st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
      if (hh == 0 && qi < p.R) store_l(p, st.m + __log2f(l), b, h, qi);
      __syncthreads();
      float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
      for (int blk = 0; blk < 2; ++blk) {
        const int qb = (blk ? rbB : rbA) * BQ;
#pragma unroll
        for (int k = 0; k < OST; ++k) {
          const int idx = k * 2 * NT + tid;
          const int r = idx / CPR, d = (idx % CPR) * 4;
          if (qb + r < p.R && d < p.D) {
            const float4 v = *reinterpret_cast<const float4*>(smem + (blk * 128 + r) * ORS + d * 4);
            st_o4<NTS>(obase + (int64_t)(qb + r) * p.o_ss + d, v.x, v.y, v.z, v.w);
          }
        }
      }
      return;
    }
    if (qi < p.R && (g == 1 || nA > 0)) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
    return;
  }
  // Merge group 1's partial state of B into group 0 through LDS.
  float* mrg = reinterpret_cast<float*>(mbase);       // [4 waves][ND*16][64]
  float* mml = mrg + 4 * ND * 16 * 64;                // [4 waves][2][64]
  if (g == 1) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mrg[((wg * ND + dt) * 16 + i) * 64 + lane] = st.o[dt][i];
    mml[(wg * 2 + 0) * 64 + lane] = st.m;
    mml[(wg * 2 + 1) * 64 + lane] = st.lh;
  }
  __syncthreads();
  float inv = 0.f;
  if (g == 0) {
    const float mb = mml[(wg * 2 + 0) * 64 + lane];
    const float lb = mml[(wg * 2 + 1) * 64 + lane];
    const float mf = fmaxf(st.m, mb);
    const float ca = __builtin_amdgcn_exp2f(st.m - mf);
    const float cb = __builtin_amdgcn_exp2f(mb - mf);
    float l = cross_half_sum(st.lh * ca + lb * cb) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        st.o[dt][i] = st.o[dt][i] * ca + mrg[((wg * ND + dt) * 16 + i) * 64 + lane] * cb;
    inv = p.o_mul / l;
    if (hh == 0 && qi < p.R) store_l(p, mf + __log2f(l), b, h, qi);
  }
  __syncthreads();
  // O leaves through LDS as whole rows (T21), as in the pair kernel.
  constexpr int ORS = DP * 4 + 16;
  if (g == 0) {
    char* orow = mbase + (wg * 32 + l32) * ORS;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
            make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                        st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
  }
  __syncthreads();
  float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
  for (int k = 0; k < OST; ++k) {
    const int idx = k * 2 * NT + tid;
    const int r = idx / CPR, d = (idx % CPR) * 4;
    if (q0 + r < p.R && d < p.D) {
      const float4 v = *reinterpret_cast<const float4*>(mbase + r * ORS + d * 4);
      float4* dst = reinterpret_cast<float4*>(obase + (int64_t)(q0 + r) * p.o_ss + d);
      st_o4<NTS>(reinterpret_cast<float*>(dst), v.x, v.y, v.z, v.w);
    }
  }
}

template <class E, int DP, int BK, bool MIRROR = true>
static hipError_t launch_fwd2_share(const FwdParams& p, hipStream_t stream) {
  // Adjacent pairs use ring 0 only (every step is shared, no merge).
  constexpr int RING = MIRROR ? 8 * BK * DP * 2 + 4 * 32 * DP * 2 : 4 * BK * DP * 2;
  constexpr int MERGE = 4 * (DP / 32) * 16 * 64 * 4 + 4 * 2 * 64 * 4;
  constexpr int OIMG = 128 * (DP * 4 + 16);
  constexpr int LDS = !MIRROR ? RING
                      : RING > MERGE ? (RING > OIMG ? RING : OIMG) : (MERGE > OIMG ? MERGE : OIMG);
  constexpr int LDS_IMG = 2 * OIMG > RING ? 2 * OIMG : RING;  // adjacent pairs, two O images
  static_assert(LDS <= 160 * 1024, "LDS");
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  // Mirrored pairs store the final O image non-temporally; MFA_SHARE_NT=0 keeps plain stores
  // (A/B).
  // Mirrored pairs: deferred V0 (+1.2 % at C2 in one-process A/B) and non-temporal O image
  // stores by default; MFA_SHARE_DV=0 / MFA_SHARE_NT=0 turn them off (A/B).
  const char* dvv = getenv("MFA_SHARE_DV");
  const char* nt = getenv("MFA_SHARE_NT");
  // ... and A's O at the switch leaves through the wave's Q staging region as whole
  // half-rows (+0.8 % at C2; MFA_SHARE_SWI=0 keeps row-per-lane stores there).
  const char* swi = getenv("MFA_SHARE_SWI");
  if (MIRROR && !(dvv && dvv[0] == '0') && !(nt && nt[0] == '0')) {
    if (swi && swi[0] == '0')
      return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, false, true>,
                    dim3(npairs * p.B * p.H), dim3(512), LDS, stream, q);
    return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, true, true>,
                  dim3(npairs * p.B * p.H), dim3(512), LDS, stream, q);
  }
  if constexpr (!MIRROR && LDS_IMG <= 160 * 1024) {
    // Adjacent pairs (D <= 128): both blocks leave through O row images by non-temporal
    // whole-row stores (C3 +0.8 %, C4's attention +1.9 % in one-process A/B; plain stores
    // from the images: +0.5 / +0.9 %).  MFA_SHARE_IMG=0 keeps row-per-lane stores (A/B).
    const char* im = getenv("MFA_SHARE_IMG");
    if (!(im && im[0] == '0'))
      return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, true>,
                    dim3(npairs * p.B * p.H), dim3(512), LDS_IMG, stream, q);
  }
  if (MIRROR && !(nt && nt[0] == '0'))
    return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true>, dim3(npairs * p.B * p.H),
                  dim3(512), LDS, stream, q);
  return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR>, dim3(npairs * p.B * p.H), dim3(512),
                LDS, stream, q);
}

template <class E, int DP, int BK, int WPS, class TU = TuneDefault>
static hipError_t launch_fwd2(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = 4 * BK * DP * 2;
  auto kern = mfa_fwd2_kernel<E, DP, BK, WPS, TU>;
  return launch(kern, dim3(p.nblk * p.B * p.H), dim3(256), LDS, stream, p);
}

template <class E, int DP, int BK, int NWG, bool OVL = true>
static hipError_t launch_fwd2_pair(const FwdParams& p, hipStream_t stream) {
  constexpr int MERGE = NWG * (DP / 32) * 16 * 64 * 4 + NWG * 2 * 64 * 4;
  constexpr int OIMG = NWG * 32 * (DP * 4 + 16);
  constexpr int MB = OVL ? 4 * BK * DP * 2 : 0;  // merge area / O image base
  constexpr int RING = 8 * BK * DP * 2;
  constexpr int LDS = RING > MB + MERGE && RING > MB + OIMG ? RING
                      : (MERGE > OIMG ? MB + MERGE : MB + OIMG);
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(NWG * 32 * (DP / 4) % (NWG * 128) == 0 && NWG * 32 * (DP / 4) / (NWG * 128) < 64,
                "O stores per thread (counted vmcnt)");
  auto kern = mfa_fwd2_pair_kernel<E, DP, BK, NWG, OVL>;
  FwdParams q = p;
  q.nblk = (p.R + NWG * 32 - 1) / (NWG * 32);
  const int npairs = (q.nblk + 1) / 2;
  return launch(kern, dim3(npairs * p.B * p.H), dim3(NWG * 128), LDS, stream, q);
}

// hipErrorNotSupported when the configuration is not covered (the caller falls back).
hipError_t fwd2_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream) {
  const char* var = getenv("MFA_FWD_VARIANT");
  const int blocks = p.nblk * p.B * p.H;
  // Causal: mirrored pairs while they fill at most ~1.5 rounds of the chip, or up to 3 rounds
  // for long rows (S >= 8192: 64 blocks; one-process A/B: H16 S8192 1057 vs 987 TF single,
  // B2 H16 S8192 1027 vs 1043, B2 H16 S4096 881 vs 889).
  bool single = !p.mask.causal || DP > 128 || (blocks > 768 && !(p.nblk >= 64 && blocks <= 1536));
  if (var && var[0] == 's') single = true;
  if (var && var[0] == 'p') single = false;
  // Development A/B of the scheduling knobs on the fp16 D=128 single-block kernel.
  if (const char* tv = getenv("MFA_FWD2_TUNE")) {
    if (elem == P_FP16 && DP == 128 && single) {
      switch (tv[0]) {
        case '1': return launch_fwd2<F16, 128, 64, 2, Tune<8, 4>>(p, stream);
        case '2': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, false, false>>(p, stream);
        case '3': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, true, true>>(p, stream);
        case '4': return launch_fwd2<F16, 128, 128, 2>(p, stream);
        case '5': return launch_fwd2<F16, 128, 64, 2, Tune<2, 2>>(p, stream);
        case '6': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, false, true, true>>(p, stream);
        default: break;
      }
    }
  }
  const char* pv = getenv("MFA_FWD_PAIR");
  const bool pair64 = pv && pv[0] == '2';
  // Causal pairs run the shared-tile schedule; MFA_FWD_PAIR=o keeps the pair kernel (A/B).
  const bool share = !(pv && (pv[0] == 'o' || pv[0] == '2' || pv[0] == 'n')) && !p.mask.window;
  if (pv && pv[0] == 'n' && elem == P_FP16 && DP == 128 && !single)  // A/B: serial seam
    return launch_fwd2_pair<F16, 128, 64, 4, false>(p, stream);
  // Unmasked forwards with at least a full wave of pairs: adjacent block pairs share every
  // K/V tile (256 query rows per staged tile; +6.5 % at C3 over the single-block kernel).
  // MFA_FWD_SHARE=0 keeps the single-block kernel (A/B), =1 takes the shared-tile kernel at
  // any size (tests).
  const char* sv = getenv("MFA_FWD_SHARE");
  // (An odd block count leaves group 1 of the last pair without rows: not for nblk < 8 odd.)
  const bool adj = !p.mask.causal && !p.mask.window && !var &&
                   (sv ? sv[0] == '1'
                       : (p.nblk % 2 == 0 || p.nblk >= 8) &&
                             (int64_t)((p.nblk + 1) / 2) * p.B * p.H >= 256);
#define MFA_F2(ELEM, EE, DPV, BKV, WPS)                                          \
  if (elem == ELEM && DP == DPV && adj)                                         \
    return launch_fwd2_share<EE, DPV, BKV, false>(p, stream);                   \
  if (elem == ELEM && DP == DPV)                                                \
    return single  ? launch_fwd2<EE, DPV, BKV, WPS>(p, stream)                  \
           : share ? launch_fwd2_share<EE, DPV, BKV>(p, stream)                  \
                   : (pair64 ? launch_fwd2_pair<EE, DPV, 32, 2>(p, stream)       \
                             : launch_fwd2_pair<EE, DPV, BKV, 4>(p, stream));
  MFA_F2(P_FP16, F16, 64, 64, 2)
  MFA_F2(P_FP16, F16, 128, 64, 2)
  MFA_F2(P_BF16, BF16, 64, 64, 2)
  MFA_F2(P_BF16, BF16, 128, 64, 2)
#undef MFA_F2
  if (elem == P_FP16 && DP == 256)
    return adj ? launch_fwd2_share<F16, 256, 32, false>(p, stream) : launch_fwd2<F16, 256, 32, 2>(p, stream);
  if (elem == P_BF16 && DP == 256)
    return adj ? launch_fwd2_share<BF16, 256, 32, false>(p, stream) : launch_fwd2<BF16, 256, 32, 2>(p, stream);
  return hipErrorNotSupported;
}

#define MFA_F2_INST(EE, DPV, BKV, WPS)                                        \
  template __global__ void mfa_fwd2_kernel<EE, DPV, BKV, WPS>(FwdParams);     \
  template __global__ void mfa_fwd2_pair_kernel<EE, DPV, BKV, 4, true>(FwdParams);  \
  template __global__ void mfa_fwd2_pair_kernel<EE, DPV, 32, 2, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, true, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, false>(FwdParams);
MFA_F2_INST(F16, 64, 64, 2)
MFA_F2_INST(F16, 128, 64, 2)
MFA_F2_INST(BF16, 64, 64, 2)
MFA_F2_INST(BF16, 128, 64, 2)
#undef MFA_F2_INST
template __global__ void mfa_fwd2_pair_kernel<F16, 128, 64, 4, false>(FwdParams);
template __global__ void mfa_fwd2_kernel<F16, 256, 32, 2>(FwdParams);
template __global__ void mfa_fwd2_share_kernel<F16, 256, 32, false>(FwdParams);
template __global__ void mfa_fwd2_share_kernel<BF16, 256, 32, false>(FwdParams);
template __global__ void mfa_fwd2_kernel<BF16, 256, 32, 2>(FwdParams);

}  // namespace mfa
