// attention_fwd_pp.hip — 16-bit forward with one wave per SIMD and two 32-row query
// sub-blocks per wave, whose softmax passes run between each other's MFMAs.
//
// Same algorithm and numerics contract as attention_fwd_v2.hip (the reference forward,
// AttentionKernel+Source.swift:372-416: S = QK^T, base-2 online softmax with the lazy rescale,
// O = PV / l, L = m + log2 l), for fp16/bf16 Q/K/V with contiguous 16-byte rows, D <= DP = 128,
// a positive scale, and either no mask or a causal mask with no fully masked row.
//
// Why a different skeleton.  The v2 kernels run two 4-wave groups per CU (two waves per SIMD):
// a wave's softmax of one key tile (exp2, row max, row sum, pack: ~5 VALU per MFMA) can only
// hide behind its SIMD partner's MFMAs, and the partner is usually doing the same thing at the
// same time.  Here a wave owns 64 query rows as two independent sub-blocks X0 and X1 and the
// whole 512-register file; the MFMA chains of one sub-block carry the other's softmax in their
// gaps (one exp2 and two or three other VALU per 32-cycle MFMA, cdna_hip_programming.md
// "4-wave, one-wave-per-SIMD" structure):
//
//   iteration u:   QK_0(u)   | softmax_1(u-1), second half of its 32 values
//                  decide_1(u-1)                      (lazy rescale; rare branch)
//                  PV_1(u-1) | softmax_0(u), first half
//                  QK_1(u)   | softmax_0(u), second half
//                  decide_0(u)
//                  PV_0(u)   | softmax_1(u), first half
//                  barrier
//
// X1 runs half an iteration behind X0, so its PV reads the previous step's V tile: the V ring
// has three slots, K two.  The next step's K/V tiles arrive by LDS-DMA, one piece every few
// MFMA gaps.  The softmax pass is speculative: P = exp2(S'), the running row max and the row
// sum are computed in one pass with the current offset, and only when the tile's max exceeds
// m + 8 (the lazy threshold, T13) does the rare branch rescale O and l and recompute P from the
// kept S' — so no exponential waits for the row max.
//
// Work units.  Unmasked: a workgroup owns 256 consecutive query rows (wave w: rows 32w and
// 128 + 32w of the two 128-row blocks), every staged K/V tile serves all of them.  Causal
// (MIRROR): the mirrored pair of 128-row blocks A (light) and B (heavy) as in the shared-tile
// kernel of attention_fwd_v2.hip; X0 holds A's rows and X1 B's rows while the keys are A's
// (phase 1, one tile per step serving 256 rows); then A is stored from registers, X0 takes B's
// rows too, and each step stages two tiles, X1 continuing B's state on the even one and X0 a
// second state of B's rows on the odd one (phase 2); the two states merge in registers at the
// end (same lanes, same rows).  Steps per workgroup: nA + ceil((nB - nA) / 2), 33 at C2.
#include "attention_fwd2.h"

namespace mfa {

template <class E>
__device__ __forceinline__ i16x8 pp_pack8(const float (&x)[8]) {
  i16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (short)E::from_f32(x[j]);
  return f;
}

// Softmax working set of one sub-block's tile: running max of the raw S' values, row-sum
// partials, the packed P (the PV B operand) and eight P values awaiting their pack.
template <int BK>
struct PPSoft {
  float mx;
  float rs[4];
  float pt[8];
  i16x8 pb[BK / 16];
  __device__ __forceinline__ void reset() {
    mx = -__builtin_inff();
    rs[0] = rs[1] = rs[2] = rs[3] = 0.f;
  }
};

template <class E, int DP, int BK, bool MIRROR>
__global__ void __launch_bounds__(256, 1) mfa_fwd_pp_kernel(FwdParams p) {
  using A = Arith16<E, DP>;
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, ND = DP / 32;
  constexpr int NV = NJ * 16;                  // S values of a tile per lane (half its keys)
  constexpr int HV = NV / 2;                   // values per half pass (one per MFMA of a chain)
  constexpr int TILEB = BK * DP * 2;
  constexpr int SLOT = (MIRROR ? 2 : 1) * TILEB;  // phase 2 stages two tiles per step
  constexpr float THR = 8.0f;
  static_assert(HV == 2 * NJ * ND && HV == NJ * (DP / 16), "one value per MFMA of each chain");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kring = smem;                    // K slots 0, 1
  char* const vring = smem + 2 * SLOT;         // V slots 0, 1, 2

  const int tid = threadIdx.x;
  const int lane = tid & 63, w = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};

  const int BH = p.B * p.H;
  const int npairs = (p.nblk + 1) / 2;
  int bh, pi;
  if constexpr (MIRROR) {
    pi = blockIdx.x / BH;  // equal causal work per workgroup: no order to keep
    bh = blockIdx.x % BH;
  } else {
    xcd_unit_block(blockIdx.x, BH, npairs, &bh, &pi);  // a head's blocks on one XCD
  }
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;

  const int rbA = MIRROR ? pi : 2 * pi;
  const int rbB = MIRROR ? p.nblk - 1 - pi : 2 * pi + 1;
  int a0, a1, kb0, kb1;
  key_range(p, rbA * 128, 128, BK, &a0, &a1);
  key_range(p, (MIRROR ? rbB : rbA) * 128, 128, BK, &kb0, &kb1);
  const int nB = kb1 > kb0 ? (kb1 - kb0 + BK - 1) / BK : 0;
  // Mirrored: the odd middle block is B only (X0 joins B from the start).
  const int nA = !MIRROR ? nB : (rbA < rbB && a1 > a0 ? (a1 - a0 + BK - 1) / BK : 0);
  const int n2 = nB - nA;
  const int U = nA + (n2 + 1) / 2;

  // Query rows of the two sub-blocks (X1: always B's; X0: A's, or B's in phase 2).
  const int qB0 = rbB * 128 + 32 * w;
  int q00 = (nA > 0 ? rbA * 128 : rbB * 128) + 32 * w;

  DmaA<DP, BK, 256> kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;

  // First key of X1's / X0's tile at step u.
  auto key1 = [&](int u) __attribute__((always_inline)) { return kb0 + (u < nA ? u : nA + 2 * (u - nA)) * BK; };
  auto key0 = [&](int u) __attribute__((always_inline)) { return kb0 + (u < nA ? u : nA + 2 * (u - nA) + 1) * BK; };

  // Prologue: step 0's tiles, then both sub-blocks' Q rows into registers.
  kd.issue(khead, key1(0), kring);
  vd.issue(vhead, key1(0), vring);
  if (nA == 0) {
    kd.issue(khead, key0(0), kring + TILEB);
    vd.issue(vhead, key0(0), vring + TILEB);
  }
  i16x8 qf0[DP / 16], qf1[DP / 16];
  load_q2_raw<DP>(qf0, p, b, h, q00 + l32, q00 + l32 < p.R, hh);
  load_q2_raw<DP>(qf1, p, b, h, qB0 + l32, qB0 + l32 < p.R, hh);
  RowState<DP> st0, st1;
  st0.init();
  st1.init();
  PPSoft<BK> sm0, sm1;
  f32x16 s0[NJ], s1[NJ];
  wait_vm();
  prescale_q2<E, DP>(qf0, c);
  prescale_q2<E, DP>(qf1, c);
  __syncthreads();

  // Value k of a sub-block's tile: P = exp2(S') with the current offset, running max, row-sum
  // partial, pack by k-steps of 8 (the order of Arith16::pack).
  auto smv = [&](f32x16 (&s)[NJ], PPSoft<BK>& sm, const RowState<DP>& st, int k) __attribute__((always_inline)) {
    const int j = k >> 4, i = k & 15;
    const float v = s[j][i];
    sm.mx = __builtin_fmaxf(sm.mx, v);
    const float pv = __builtin_amdgcn_exp2f(PS ? v : __builtin_fmaf(v, c, -st.m));
    sm.rs[k & 3] += pv;
    sm.pt[k & 7] = pv;
    if ((k & 7) == 7) sm.pb[k >> 3] = pp_pack8<E>(sm.pt);
  };
  // After the pass: the lazy-rescale decision (wave-uniform, rarely taken), then l += Σ P.
  auto decide = [&](f32x16 (&s)[NJ], PPSoft<BK>& sm, RowState<DP>& st) __attribute__((always_inline)) {
    const float mx = cross_half_max(sm.mx);
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
      sm.rs[0] = sm.rs[1] = sm.rs[2] = sm.rs[3] = 0.f;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int j = k >> 4, i = k & 15;
        const float pv = __builtin_amdgcn_exp2f(PS ? s[j][i] : __builtin_fmaf(s[j][i], c, -st.m));
        sm.rs[k & 3] += pv;
        sm.pt[k & 7] = pv;
        if ((k & 7) == 7) sm.pb[k >> 3] = pp_pack8<E>(sm.pt);
      }
    }
    st.lh += (sm.rs[0] + sm.rs[1]) + (sm.rs[2] + sm.rs[3]);
  };
  // Causal diagonal / key-edge masks of a sub-block's tile (keys t..t+BK-1, rows q0 + l32).
  auto mask = [&](f32x16 (&s)[NJ], int t, int q0) __attribute__((always_inline)) {
    if ((t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0)) {
      MFA_KEEP_BRANCH();
      const int base = t + 4 * hh;
      int hi = p.C - 1 - base;
      if (p.mask.causal) hi = min(hi, q0 + l32 - base);
      mask_outside<NJ>(s, -0x40000000, hi, -__builtin_inff());
    }
  };

  int vcur = 0;  // V slot of step u (u % 3)
  auto iteration = [&](int u, auto first_c, auto dma2_c) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr bool DMA2 = decltype(dma2_c)::value;  // step u + 1 stages two tiles
    const bool ph2 = u >= nA;
    if (MIRROR && u == nA && nA > 0) {
      // A is complete (its last PV ran in iteration u - 1): store it from registers, then X0
      // becomes a second state of B's rows.
      float l = cross_half_sum(st0.lh) + kFltMin;
      if (!(l > 0.f)) l = kFltMin;
      if (q00 + l32 < p.R) store_o_l<DP>(p, st0.o, st0.m, l, b, h, q00 + l32, hh);
      st0.init();
#pragma unroll
      for (int ds = 0; ds < DP / 16; ++ds) qf0[ds] = qf1[ds];
      q00 = qB0;
    }
    const char* kt1 = kring + (u & 1) * SLOT;
    const char* kt0 = kt1 + (ph2 ? TILEB : 0);
    const int vprev = vcur == 0 ? 2 : vcur - 1;
    const char* vt1 = vring + vprev * SLOT;                     // X1's tile of step u - 1
    const char* vt0 = vring + vcur * SLOT + (ph2 ? TILEB : 0);  // X0's tile of step u
    const int vnext = vcur == 2 ? 0 : vcur + 1;
    char* const kn = kring + ((u + 1) & 1) * SLOT;
    char* const vn = vring + vnext * SLOT;
    const int tn1 = key1(u + 1), tn0 = key0(u + 1);
    // The next step's tiles: 4 pieces per wave per tile, one every few MFMA gaps.
    constexpr int NP = DMA2 ? 16 : 8;
    constexpr int STRIDE = 4 * NJ * 2 * ND / NP;  // gaps per piece over the 4 chains
    auto dma = [&](int chain, int i) __attribute__((always_inline)) {
      const int g = chain * (2 * NJ * ND) + i;
      if (g % STRIDE == STRIDE / 2) {
        const int pc = g / STRIDE, which = pc / 4, k = pc % 4;
        if (which == 0) kd.issue_piece(khead, tn1, kn, k);
        else if (which == 1) vd.issue_piece(vhead, tn1, vn, k);
        else if (which == 2) kd.issue_piece(khead, tn0, kn + TILEB, k);
        else vd.issue_piece(vhead, tn0, vn + TILEB, k);
      }
    };
    const int t0 = key0(u), t1 = key1(u);

    // QK_0(u) | second half of softmax_1(u - 1).
    fwd2_qk<E, DP, BK>(kt0, rbase, qf0, st0, s0, [&](int i) {
      if constexpr (!FIRST) smv(s1, sm1, st1, HV + i);
      dma(0, i);
    });
    mask(s0, t0, q00);
    sm0.reset();
    if constexpr (!FIRST) {
      decide(s1, sm1, st1);
      // PV_1(u - 1) | first half of softmax_0(u).
      fwd2_pv<E, DP, BK>(vt1, trb, sm1.pb, st1, [&](int i) {
        smv(s0, sm0, st0, i);
        dma(1, i);
      });
    } else {
#pragma unroll
      for (int k = 0; k < HV; ++k) smv(s0, sm0, st0, k);
    }
    // QK_1(u) | second half of softmax_0(u).
    fwd2_qk<E, DP, BK>(kt1, rbase, qf1, st1, s1, [&](int i) {
      smv(s0, sm0, st0, HV + i);
      dma(2, i);
    });
    mask(s1, t1, qB0);
    decide(s0, sm0, st0);
    sm1.reset();
    // PV_0(u) | first half of softmax_1(u).
    fwd2_pv<E, DP, BK>(vt0, trb, sm0.pb, st0, [&](int i) {
      smv(s1, sm1, st1, i);
      dma(3, i);
    });
    if constexpr (FIRST) {
      // No PV_1(u - 1) chain carried its pieces.
#pragma unroll
      for (int i = 0; i < 2 * NJ * ND; ++i) dma(1, i);
    }
    wait_vm();
    __syncthreads();
    vcur = vnext;
  };

  using T_ = std::true_type;
  using F_ = std::false_type;
  if (U > 0) {
    // u + 1 stages two tiles once u + 1 >= nA (phase 2).
    if (1 >= nA && MIRROR) iteration(0, T_(), T_());
    else iteration(0, T_(), F_());
    int u = 1;
    if constexpr (MIRROR) {
      for (; u < nA - 1 && u < U; ++u) iteration(u, F_(), F_());
      for (; u < U; ++u) iteration(u, F_(), T_());
    } else {
      for (; u < U; ++u) iteration(u, F_(), F_());
    }
    // Drain: the rest of softmax_1(U - 1) and PV_1(U - 1).
#pragma unroll
    for (int k = HV; k < NV; ++k) smv(s1, sm1, st1, k);
    decide(s1, sm1, st1);
    const int vprev = vcur == 0 ? 2 : vcur - 1;
    fwd2_pv<E, DP, BK>(vring + vprev * SLOT, trb, sm1.pb, st1);
  }

  // Epilogue.  Mirrored with a phase 2: X0 holds a second state of B's rows, merged into X1.
  bool store0 = !MIRROR || (nA > 0 && n2 == 0);
  if (MIRROR && n2 > 0) {
    const float mf = fmaxf(st1.m, st0.m);
    const float ca = __builtin_amdgcn_exp2f(st1.m - mf);
    const float cb = __builtin_amdgcn_exp2f(st0.m - mf);
    st1.lh = st1.lh * ca + st0.lh * cb;
    st1.m = mf;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) st1.o[dt][i] = st1.o[dt][i] * ca + st0.o[dt][i] * cb;
  }
  // O leaves through LDS row images (the rings are free) as whole rows, non-temporal.
  constexpr int ORS = DP * 4 + 16;
  auto img = [&](const RowState<DP>& st, int x, int q0) __attribute__((always_inline)) {
    float l = cross_half_sum(st.lh) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    const float inv = p.o_mul / l;
    char* orow = smem + (x * 128 + 32 * w + l32) * ORS;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
            make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                        st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
    if (hh == 0 && q0 + l32 < p.R) store_l(p, st.m + __log2f(l), b, h, q0 + l32);
  };
  __syncthreads();  // every wave's last LDS reads are done before the images overwrite them
  if (store0) img(st0, 0, q00);
  img(st1, 1, qB0);
  __syncthreads();
  constexpr int CPR = DP / 4;
  constexpr int OST = 128 * CPR / 256;
  float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    if (x == 0 && !store0) continue;
    const int qb = (x == 0 ? rbA : rbB) * 128;
#pragma unroll
    for (int k = 0; k < OST; ++k) {
      const int idx = k * 256 + tid;
      const int r = idx / CPR, d = (idx % CPR) * 4;
      if (qb + r < p.R && d < p.D) {
        const float4 v = *reinterpret_cast<const float4*>(smem + (x * 128 + r) * ORS + d * 4);
        st_o4<true>(obase + (int64_t)(qb + r) * p.o_ss + d, v.x, v.y, v.z, v.w);
      }
    }
  }
}

template <class E, int DP, int BK, bool MIRROR>
static hipError_t launch_fwd_pp(const FwdParams& p, hipStream_t stream) {
  constexpr int TILEB = BK * DP * 2;
  constexpr int RING = 5 * (MIRROR ? 2 : 1) * TILEB;
  constexpr int OIMG = 2 * 128 * (DP * 4 + 16);
  constexpr int LDS = RING > OIMG ? RING : OIMG;
  static_assert(LDS <= 160 * 1024, "LDS");
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  return launch(mfa_fwd_pp_kernel<E, DP, BK, MIRROR>, dim3(npairs * p.B * p.H), dim3(256), LDS,
                stream, q);
}

// hipErrorNotSupported when the configuration is not covered.  Causal problems run the
// mirrored schedule (no window, no ranges); unmasked ones 256-row blocks.
hipError_t fwd_pp_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream) {
  if (DP != 128 || p.mask.window || p.mask.ranges || p.mask.amask) return hipErrorNotSupported;
  if (p.mask.causal && !p.mask.skip_ok) return hipErrorNotSupported;
  const bool mir = p.mask.causal;
  if (elem == P_FP16)
    return mir ? launch_fwd_pp<F16, 128, 64, true>(p, stream) : launch_fwd_pp<F16, 128, 64, false>(p, stream);
  if (elem == P_BF16)
    return mir ? launch_fwd_pp<BF16, 128, 64, true>(p, stream) : launch_fwd_pp<BF16, 128, 64, false>(p, stream);
  return hipErrorNotSupported;
}

template __global__ void mfa_fwd_pp_kernel<F16, 128, 64, true>(FwdParams);
template __global__ void mfa_fwd_pp_kernel<F16, 128, 64, false>(FwdParams);
template __global__ void mfa_fwd_pp_kernel<BF16, 128, 64, true>(FwdParams);
template __global__ void mfa_fwd_pp_kernel<BF16, 128, 64, false>(FwdParams);

}  // namespace mfa
