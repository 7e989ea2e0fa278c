// attention_fwd_aw.hip — 16-bit forward with one wave per SIMD, two 32-row query sub-blocks
// per wave, and the O accumulators in accumulator registers (AGPRs) the kernel owns.
//
// Same algorithm and numerics contract as attention_fwd_v2.hip (the reference forward,
// AttentionKernel+Source.swift:372-416: S = QK^T, base-2 online softmax with the lazy rescale,
// O = PV / l, L = m + log2 l), for fp16/bf16 Q/K/V with contiguous 16-byte rows, D <= DP = 128,
// a positive scale, and either no mask or a causal mask with no fully masked row.
//
// Schedule (cdna_hip_programming.md, "4-wave, one-wave-per-SIMD" structure).  A workgroup is
// 4 waves, one per SIMD, each owning the whole 512-entry register file.  A wave holds 64 query
// rows as two independent sub-blocks X0 and X1; the MFMA chains of one sub-block carry the
// other's softmax in their gaps (one exp2 and one to three other VALU per 32-cycle MFMA):
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
// MFMA gaps.  The softmax pass is speculative: P = exp2(S'), the tile's row max and the row sum
// come from one pass against the current offset; only when the tile max exceeds m + 8 (the
// lazy threshold) does the rare branch rescale O and l and recompute P from the kept S'.
//
// Registers.  The two sub-blocks' O (2 x 32 rows x 128 columns, fp32) is 128 registers per
// lane.  A compiler-allocated kernel keeps MFMA accumulators in the 256 arch
// VGPRs, where O, Q, S, the -m tiles and the packed P do not fit together (round-3 experiment
// in DESIGN.md: the compiler parked Q in AGPRs and copied fragments back before every MFMA).
// Here the PV MFMAs are written as inline assembly that accumulates straight into fixed AGPRs
// a[0:63] (X0) and a[64:127] (X1); the compiler sees them only as clobbers, allocates
// everything else in arch VGPRs, and the rare rescale, the phase switch and the epilogue move
// O through v_accvgpr_read/write.  The hazards the compiler cannot see in inline assembly are
// covered by hand: s_nop before a PV chain (VALU-written P read by the MFMA) and before any
// read of an AGPR an MFMA wrote (XDL write -> VALU read), after AGPR writes before the next
// MFMA reads them as accumulators.
//
// Work units.  Unmasked: a workgroup owns 256 consecutive query rows (wave w: rows 32w and
// 128 + 32w of the two 128-row blocks); every staged K/V tile serves all of them.  Causal
// (MIRROR): the mirrored pair of 128-row blocks A (light) and B (heavy); X0 holds A's rows and
// X1 B's rows while the keys are A's (phase 1, one tile per step serving 256 rows); then A is
// stored, X0 takes B's rows too, and each step stages two tiles, X1 continuing B's state on the
// even one and X0 a second state of B's rows on the odd one (phase 2); the two states merge at
// the end (same lanes, same rows).
#include <utility>

#include "attention_fwd2.h"

// Development knobs (the defaults are the shipped configuration): fragment read-ahead of the
// QK^T and PV chains, and how many of an iteration's four chains carry the next tiles' DMA.
#ifndef AW_AHK
#define AW_AHK 4
#endif
#ifndef AW_AHV
#define AW_AHV 3
#endif
#ifndef AW_DMA_CHAINS
#define AW_DMA_CHAINS 4
#endif

namespace mfa {
namespace aw {

// Every O register, named as a clobber of each inline-assembly statement that writes O: the
// compiler then keeps none of its own values in them across those statements.
#define AW_O_CLOBBERS \
  "a0", "a1", "a2", "a3", "a4", "a5", "a6", "a7", "a8", "a9", "a10", "a11", "a12", "a13", "a14", "a15", \
  "a16", "a17", "a18", "a19", "a20", "a21", "a22", "a23", "a24", "a25", "a26", "a27", "a28", "a29", "a30", "a31", \
  "a32", "a33", "a34", "a35", "a36", "a37", "a38", "a39", "a40", "a41", "a42", "a43", "a44", "a45", "a46", "a47", \
  "a48", "a49", "a50", "a51", "a52", "a53", "a54", "a55", "a56", "a57", "a58", "a59", "a60", "a61", "a62", "a63", \
  "a64", "a65", "a66", "a67", "a68", "a69", "a70", "a71", "a72", "a73", "a74", "a75", "a76", "a77", "a78", "a79", \
  "a80", "a81", "a82", "a83", "a84", "a85", "a86", "a87", "a88", "a89", "a90", "a91", "a92", "a93", "a94", "a95", \
  "a96", "a97", "a98", "a99", "a100", "a101", "a102", "a103", "a104", "a105", "a106", "a107", "a108", "a109", "a110", "a111", \
  "a112", "a113", "a114", "a115", "a116", "a117", "a118", "a119", "a120", "a121", "a122", "a123", "a124", "a125", "a126", "a127"
// Compile-time loop: f(integral_constant<int, B>) ... f(<B + N - 1>).
template <int B, int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  if constexpr (N > 0) {
    f(std::integral_constant<int, B>());
    sfor<B + 1, N - 1>(f);
  }
}

template <int R>
__device__ __forceinline__ float aread() {
  float x;
  asm volatile("v_accvgpr_read_b32 %0, a[%1]" : "=v"(x) : "n"(R));
  return x;
}
template <int R>
__device__ __forceinline__ void awrite(float x) {
  asm volatile("v_accvgpr_write_b32 a[%0], %1" ::"n"(R), "v"(x) : AW_O_CLOBBERS);
}
template <int R>
__device__ __forceinline__ void azero() {
  asm volatile("v_accvgpr_write_b32 a[%0], 0" ::"n"(R) : AW_O_CLOBBERS);
}
// XDL write -> VALU read of the same register (v_accvgpr_read): 11 wait states for the
// 8-pass 32x32x16 MFMA; 24 here.
__device__ __forceinline__ void drain_mfma() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }
// VALU / v_accvgpr_write -> MFMA read of the same register.
__device__ __forceinline__ void settle_writes() { asm volatile("s_nop 4" ::: "memory"); }

// O^T tile (rows of the head dimension, query on the lane) += V^T · P^T into a[R:R+15].
// NOP: the chain's first MFMA, whose P operand the VALU may have written just before.
template <class E, int R, bool NOP>
__device__ __forceinline__ void pv_mfma(i16x8 a, i16x8 b) {
  if constexpr (E::prec == P_FP16) {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a),
                   "v"(b), "n"(R) : AW_O_CLOBBERS);
    else
      asm volatile("v_mfma_f32_32x32x16_f16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a), "v"(b),
                   "n"(R) : AW_O_CLOBBERS);
  } else {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a),
                   "v"(b), "n"(R) : AW_O_CLOBBERS);
    else
      asm volatile("v_mfma_f32_32x32x16_bf16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a), "v"(b),
                   "n"(R) : AW_O_CLOBBERS);
  }
}

// Two P values rounded to the element type (round to nearest even, as E::from_f32) in one
// word, low half first: one v_cvt_pk_{f16,bf16}_f32.
template <class E>
__device__ __forceinline__ unsigned pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  if constexpr (E::prec == P_FP16) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, h2));
  } else {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(unsigned, __builtin_convertvector((f2){a, b}, b2));
  }
}

// Row state of one sub-block (O lives in AGPRs).
struct Row {
  float m;   // running max (log2 units, reference convention)
  float lh;  // partial row sum of this half-wave's keys
  __device__ __forceinline__ void init() {
    m = -kFltMax;
    lh = 0.f;
  }
};

// Softmax working set of one sub-block's tile: row-sum partials and the packed P (the PV B
// operand).
template <int BK>
struct Soft {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  float rs[4];
  float pe;            // the even value of the pair being packed
  u32x4 pw[BK / 16];   // packed P, two 16-bit values per word (Arith16::pack order)
  __device__ __forceinline__ i16x8 pb(int ks) const { return __builtin_bit_cast(i16x8, pw[ks]); }
  __device__ __forceinline__ void reset() { rs[0] = rs[1] = rs[2] = rs[3] = 0.f; }
};

template <int OB, int N>
__device__ __forceinline__ void zero_o() {
  sfor<0, N>([&](auto ic) { azero<OB + decltype(ic)::value>(); });
}

template <int OB>
__device__ __forceinline__ void scale_o(float corr) {
  drain_mfma();
  sfor<0, 64>([&](auto ic) {
    constexpr int r = OB + decltype(ic)::value;
    awrite<r>(aread<r>() * corr);
  });
  settle_writes();
}

}  // namespace aw

// Diagnostic build only (tools/diag/aw_stamps.hip defines MFA_STAMPS): shader cycles per phase
// of the tile loop, summed per wave into slots 0..7 of its stamp record.
#ifdef MFA_STAMPS
#define AW_ACC_DECL() unsigned long long awacc_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, awt_ = __builtin_amdgcn_s_memtime()
#define AW_ACC(k)                                               \
  do {                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    awacc_[k] += t_ - awt_;                                     \
    awt_ = t_;                                                  \
  } while (0)
#define AW_ACC_END()                                                                         \
  do {                                                                                       \
    if ((threadIdx.x & 63) == 0)                                                             \
      for (int k_ = 0; k_ < 8; ++k_)                                                         \
        g_mfa_stamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + k_] = awacc_[k_]; \
  } while (0)
#else
#define AW_ACC_DECL() do {} while (0)
#define AW_ACC(k) do {} while (0)
#define AW_ACC_END() do {} while (0)
#endif

template <class E, int DP, int BK, bool MIRROR>
__global__ void __launch_bounds__(256, 1) mfa_fwd_aw_kernel(FwdParams p) {
  using A = Arith16<E, DP>;
  using aw::aread;
  using aw::sfor;
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, ND = DP / 32, DS = DP / 16;
  constexpr int NV = NJ * 16;                  // S values of a tile per lane (half its keys)
  constexpr int HV = NV / 2;                   // values per half pass (one per MFMA of a chain)
  constexpr int TILEB = BK * DP * 2;
  constexpr int SLOT = (MIRROR ? 2 : 1) * TILEB;  // phase 2 stages two tiles per step
  constexpr float THR = 8.0f;
  constexpr int NQK = DS * NJ, NPV = NJ * 2 * ND;
  static_assert(DP == 128 && HV == NQK && HV == NPV, "one value per MFMA of each chain");
  constexpr int OB0 = 0, OB1 = 64;             // AGPR bases of X0's and X1's O
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
  i16x8 qf0[DS], qf1[DS];
  load_q2_raw<DP>(qf0, p, b, h, q00 + l32, q00 + l32 < p.R, hh);
  load_q2_raw<DP>(qf1, p, b, h, qB0 + l32, qB0 + l32 < p.R, hh);
  aw::Row st0, st1;
  st0.init();
  st1.init();
  aw::zero_o<0, 128>();
  aw::Soft<BK> sm0, sm1;
  f32x16 s0[NJ], s1[NJ];
  wait_vm();
  prescale_q2<E, DP>(qf0, c);
  prescale_q2<E, DP>(qf1, c);
  aw::settle_writes();
  __syncthreads();
  AW_ACC_DECL();

  // Fragment rings of the two chain kinds.  A chain's last read-ahead slots prefetch the first
  // fragments of the chain after it (tail(j), j < AH), so no chain but the iteration's first
  // (whose K tile is only valid after the barrier) starts on an LDS read's latency.
  constexpr int AHK = AW_AHK, AHV = AW_AHV;
  i16x8 kp[AHK], vp[AHV];
  auto kread = [&](const char* kt, int i) __attribute__((always_inline)) {
    return A::read_row_a(kt, rbase, i % NJ, i / NJ);
  };
  auto vread = [&](const char* vt, int i) __attribute__((always_inline)) {
    const int jk = i / ND, dt = i % ND;
    return A::read_tr_a(vt, trb, (jk >> 1) * 32, jk & 1, dt * 32);
  };
  auto no_tail = [](int) __attribute__((always_inline)) {};
  // S^T = K·Q^T (key in registers, query on the lane; Q pre-scaled by c on the fp16 path).
  // PRE: kp already holds the chain's first AHK fragments.
  auto qk = [&](auto pre_c, const char* kt, const i16x8 (&qf)[DS], const aw::Row& st,
                f32x16 (&s)[NJ], auto&& hook, auto&& tail) __attribute__((always_inline)) {
    if constexpr (!decltype(pre_c)::value) {
#pragma unroll
      for (int i = 0; i < AHK; ++i) kp[i] = kread(kt, i);
    }
#pragma unroll
    for (int i = 0; i < NQK; ++i) {
      const int ds = i / NJ, j = i % NJ;
      if (ds == 0)
        s[j] = A::mma(kp[i % AHK], qf[0], zero16());
      else
        s[j] = A::mma(kp[i % AHK], qf[ds], s[j]);
      if (i + AHK < NQK) kp[i % AHK] = kread(kt, i + AHK);
      else tail(i + AHK - NQK);
      hook(i);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // O^T += V^T·P^T into the sub-block's AGPRs.  PRE: vp holds the first AHV fragments.
  auto pv = [&](auto ob_c, auto pre_c, const char* vt, const aw::Soft<BK>& sm, auto&& hook,
                auto&& tail) __attribute__((always_inline)) {
    constexpr int OB = decltype(ob_c)::value;
    if constexpr (!decltype(pre_c)::value) {
#pragma unroll
      for (int i = 0; i < AHV; ++i) vp[i] = vread(vt, i);
    }
    sfor<0, NPV>([&](auto ic) {
      constexpr int i = decltype(ic)::value, jk = i / ND, dt = i % ND;
      aw::pv_mfma<E, OB + 16 * dt, i == 0>(vp[i % AHV], sm.pb(jk));
      if constexpr (i + AHV < NPV) vp[i % AHV] = vread(vt, i + AHV);
      else tail(i + AHV - NPV);
      hook(i);
      __builtin_amdgcn_sched_barrier(0);
    });
  };

  // Value k of a sub-block's tile: P = exp2(S·c − m) against the row max the decision before
  // the pass settled, row-sum partial, packed in place by pairs (the order of Arith16::pack).
  // The empty volatile statements pin each value where it is computed, in the MFMA gap it was
  // placed in; without them the compiler moves the sums and packs into bursts between chains.
  auto smv = [&](f32x16 (&s)[NJ], aw::Soft<BK>& sm, const aw::Row& st, int k) __attribute__((always_inline)) {
    const int j = k >> 4, i = k & 15;
    const float v = s[j][i];
    float pv = __builtin_amdgcn_exp2f(PS ? v - st.m : __builtin_fmaf(v, c, -st.m));
    asm volatile("" : "+v"(pv));
    sm.rs[k & 3] += pv;
    asm volatile("" : "+v"(sm.rs[k & 3]));
    if ((k & 1) == 0) {
      sm.pe = pv;
    } else {
      unsigned pk = aw::pack2<E>(sm.pe, pv);
      asm volatile("" : "+v"(pk));
      sm.pw[k >> 3][(k & 7) >> 1] = pk;
    }
  };
  // The tile's row max (both lane halves), then the lazy-rescale decision (wave-uniform,
  // rarely taken): only the row state and the sub-block's O in AGPRs change in the branch.
  auto decide = [&](auto ob_c, const f32x16 (&s)[NJ], aw::Row& st) __attribute__((always_inline)) {
    constexpr int OB = decltype(ob_c)::value;
    float a4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k0 = 8 * q;
      float m0 = __builtin_fmaxf(__builtin_fmaxf(s[k0 >> 4][(k0 & 15)], s[k0 >> 4][(k0 & 15) + 1]),
                                 s[k0 >> 4][(k0 & 15) + 2]);
      m0 = __builtin_fmaxf(__builtin_fmaxf(m0, s[k0 >> 4][(k0 & 15) + 3]), s[k0 >> 4][(k0 & 15) + 4]);
      m0 = __builtin_fmaxf(__builtin_fmaxf(m0, s[k0 >> 4][(k0 & 15) + 5]), s[k0 >> 4][(k0 & 15) + 6]);
      a4[q] = __builtin_fmaxf(m0, s[k0 >> 4][(k0 & 15) + 7]);
    }
    const float mx = cross_half_max(__builtin_fmaxf(__builtin_fmaxf(a4[0], a4[1]), __builtin_fmaxf(a4[2], a4[3])));
    const float mt = PS ? mx : mx * c;
    if (__builtin_expect(__any(mt > st.m + THR), 0)) {
      MFA_KEEP_BRANCH();
      const float m_new = fmaxf(st.m, mt);
      const float corr = __builtin_amdgcn_exp2f(st.m - m_new);
      // Rows still at the initial max have O = 0 (every P so far was exp2(-inf)): no multiply.
      if (!__all(st.m == -kFltMax)) aw::scale_o<OB>(corr);
      st.m = m_new;
      st.lh *= corr;
    }
  };
  // After the tile's last value: l += Σ P.
  auto finish = [&](aw::Soft<BK>& sm, aw::Row& st) __attribute__((always_inline)) {
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
  // O of X0 (a[0:63]) straight to global memory, row per lane (the phase switch).
  auto store_x0 = [&](const aw::Row& st, int q0) __attribute__((always_inline)) {
    float l = cross_half_sum(st.lh) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    const float inv = p.o_mul / l;
    const int qi = q0 + l32;
    aw::drain_mfma();
    if (qi < p.R) {
      float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
      sfor<0, ND * 4>([&](auto ic) {
        constexpr int dt = decltype(ic)::value / 4, g = decltype(ic)::value % 4;
        constexpr int r = OB0 + dt * 16 + 4 * g;
        const int d = dt * 32 + 8 * g + 4 * hh;
        const float x0 = aread<r>(), x1 = aread<r + 1>(), x2 = aread<r + 2>(), x3 = aread<r + 3>();
        if (d < p.D) st_o4<false>(orow + d, x0 * inv, x1 * inv, x2 * inv, x3 * inv);
      });
      if (hh == 0) store_l(p, st.m + __log2f(l), b, h, qi);
    }
  };

  int vcur = 0;  // V slot of step u (u % 3)
  auto iteration = [&](int u, auto first_c, auto dma2_c) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr bool DMA2 = decltype(dma2_c)::value;  // step u + 1 stages two tiles
    const bool ph2 = u >= nA;
    if (MIRROR && u == nA && nA > 0) {
      // A is complete (its last PV ran in iteration u - 1): store it, then X0 becomes a second
      // state of B's rows.
      store_x0(st0, q00);
      st0.init();
      aw::zero_o<OB0, 64>();
      aw::settle_writes();
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) qf0[ds] = qf1[ds];
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
    constexpr int NCH = DMA2 ? 4 : AW_DMA_CHAINS;  // chains that carry the pieces
    constexpr int STRIDE = NCH * NQK / NP;         // gaps per piece
    auto dma = [&](int chain, int i) __attribute__((always_inline)) {
      const int g = chain * NQK + i;
      if (g < NCH * NQK && g % STRIDE == STRIDE / 2) {
        const int pc = g / STRIDE, which = pc / 4, k = pc % 4;
        if (which == 0) kd.issue_piece(khead, tn1, kn, k);
        else if (which == 1) vd.issue_piece(vhead, tn1, vn, k);
        else if (which == 2) kd.issue_piece(khead, tn0, kn + TILEB, k);
        else vd.issue_piece(vhead, tn0, vn + TILEB, k);
      }
    };
    const int t0 = key0(u), t1 = key1(u);
    using O0 = std::integral_constant<int, OB0>;
    using O1 = std::integral_constant<int, OB1>;

    auto pre_v = [&](const char* vt) __attribute__((always_inline)) {
      return [&, vt](int j) __attribute__((always_inline)) { if (j < AHV) vp[j] = vread(vt, j); };
    };
    auto pre_k = [&](const char* kt, bool from_pv) __attribute__((always_inline)) {
      // A PV chain's tail has AHV < AHK slots: its last one loads the rest.
      return [&, kt, from_pv](int j) __attribute__((always_inline)) {
        kp[j] = kread(kt, j);
        if (from_pv && j == AHV - 1) {
#pragma unroll
          for (int r = AHV; r < AHK; ++r) kp[r] = kread(kt, r);
        }
      };
    };
    using T_ = std::true_type;
    using F_ = std::false_type;

    // QK_0(u) | second half of softmax_1(u - 1); its tail prefetches PV_1's (or, in the first
    // iteration, QK_1's) first fragments.
    auto h_qk0 = [&](int i) __attribute__((always_inline)) {
      if constexpr (!FIRST) smv(s1, sm1, st1, HV + i);
      dma(0, i);
    };
    if constexpr (FIRST) qk(F_(), kt0, qf0, st0, s0, h_qk0, pre_k(kt1, false));
    else qk(F_(), kt0, qf0, st0, s0, h_qk0, pre_v(vt1));
    AW_ACC(0);
    if constexpr (!FIRST) finish(sm1, st1);
    mask(s0, t0, q00);
    decide(O0(), s0, st0);
    sm0.reset();
    AW_ACC(1);
    if constexpr (!FIRST) {
      // PV_1(u - 1) | first half of softmax_0(u).
      pv(O1(), T_(), vt1, sm1, [&](int i) __attribute__((always_inline)) {
        smv(s0, sm0, st0, i);
        dma(1, i);
      }, pre_k(kt1, true));
      AW_ACC(2);
    } else {
#pragma unroll
      for (int k = 0; k < HV; ++k) smv(s0, sm0, st0, k);
    }
    // QK_1(u) | second half of softmax_0(u).
    qk(T_(), kt1, qf1, st1, s1, [&](int i) __attribute__((always_inline)) {
      smv(s0, sm0, st0, HV + i);
      dma(2, i);
    }, pre_v(vt0));
    AW_ACC(3);
    finish(sm0, st0);
    mask(s1, t1, qB0);
    decide(O1(), s1, st1);
    sm1.reset();
    AW_ACC(4);
    // PV_0(u) | first half of softmax_1(u).
    pv(O0(), T_(), vt0, sm0, [&](int i) __attribute__((always_inline)) {
      smv(s1, sm1, st1, i);
      dma(3, i);
    }, no_tail);
    AW_ACC(5);
    if constexpr (FIRST) {
      // No PV_1(u - 1) chain carried its pieces.
#pragma unroll
      for (int i = 0; i < NQK; ++i) dma(1, i);
    }
    wait_vm();
    AW_ACC(6);
    __syncthreads();
    AW_ACC(7);
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
    finish(sm1, st1);
    const int vprev = vcur == 0 ? 2 : vcur - 1;
    pv(std::integral_constant<int, OB1>(), std::false_type(), vring + vprev * SLOT, sm1, no_tail,
       no_tail);
  }

  AW_ACC_END();
  // Epilogue.  Mirrored with a phase 2: X0 holds a second state of B's rows, merged into X1's
  // as the image is written.
  const bool store0 = !MIRROR || (nA > 0 && n2 == 0);
  const bool merge = MIRROR && n2 > 0;
  float ca = 1.f, cb = 0.f;
  if (merge) {
    const float mf = fmaxf(st1.m, st0.m);
    ca = __builtin_amdgcn_exp2f(st1.m - mf);
    cb = __builtin_amdgcn_exp2f(st0.m - mf);
    st1.lh = st1.lh * ca + st0.lh * cb;
    st1.m = mf;
  }
  // O leaves through LDS row images (the rings are free) as whole rows, non-temporal.
  constexpr int ORS = DP * 4 + 16;
  __syncthreads();  // every wave's last LDS reads are done before the images overwrite them
  aw::drain_mfma();
  auto lsum = [&](const aw::Row& st) __attribute__((always_inline)) {
    float l = cross_half_sum(st.lh) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    return l;
  };
  if (store0) {
    const float l = lsum(st0);
    const float inv = p.o_mul / l;
    char* orow = smem + (32 * w + l32) * ORS;
    sfor<0, ND * 4>([&](auto ic) {
      constexpr int dt = decltype(ic)::value / 4, g = decltype(ic)::value % 4;
      constexpr int r = OB0 + dt * 16 + 4 * g;
      *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * g + 4 * hh) * 4) =
          make_float4(aread<r>() * inv, aread<r + 1>() * inv, aread<r + 2>() * inv,
                      aread<r + 3>() * inv);
    });
    if (hh == 0 && q00 + l32 < p.R) store_l(p, st0.m + __log2f(l), b, h, q00 + l32);
  }
  {
    const float l = lsum(st1);
    const float inv = p.o_mul / l;
    const float ia = ca * inv, ib = cb * inv;
    char* orow = smem + (128 + 32 * w + l32) * ORS;
    sfor<0, ND * 4>([&](auto ic) {
      constexpr int dt = decltype(ic)::value / 4, g = decltype(ic)::value % 4;
      constexpr int r = OB1 + dt * 16 + 4 * g, r0 = OB0 + dt * 16 + 4 * g;
      float4 v;
      if (merge) {
        v = make_float4(aread<r>() * ia + aread<r0>() * ib, aread<r + 1>() * ia + aread<r0 + 1>() * ib,
                        aread<r + 2>() * ia + aread<r0 + 2>() * ib, aread<r + 3>() * ia + aread<r0 + 3>() * ib);
      } else {
        v = make_float4(aread<r>() * inv, aread<r + 1>() * inv, aread<r + 2>() * inv,
                        aread<r + 3>() * inv);
      }
      *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * g + 4 * hh) * 4) = v;
    });
    if (hh == 0 && qB0 + l32 < p.R) store_l(p, st1.m + __log2f(l), b, h, qB0 + l32);
  }
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
static hipError_t launch_fwd_aw(const FwdParams& p, hipStream_t stream) {
  constexpr int TILEB = BK * DP * 2;
  constexpr int RING = 5 * (MIRROR ? 2 : 1) * TILEB;
  constexpr int OIMG = 2 * 128 * (DP * 4 + 16);
  constexpr int LDS = RING > OIMG ? RING : OIMG;
  static_assert(LDS <= 160 * 1024, "LDS");
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  return launch(mfa_fwd_aw_kernel<E, DP, BK, MIRROR>, dim3(npairs * p.B * p.H), dim3(256), LDS,
                stream, q);
}

// hipErrorNotSupported when the configuration is not covered.  Causal problems run the
// mirrored schedule (no window, no ranges); unmasked ones 256-row blocks.
hipError_t fwd_aw_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream) {
  if (DP != 128 || p.mask.window || p.mask.ranges || p.mask.amask) return hipErrorNotSupported;
  if (p.mask.causal && !p.mask.skip_ok) return hipErrorNotSupported;
  const bool mir = p.mask.causal;
  if (elem == P_FP16)
    return mir ? launch_fwd_aw<F16, 128, 64, true>(p, stream) : launch_fwd_aw<F16, 128, 64, false>(p, stream);
  if (elem == P_BF16)
    return mir ? launch_fwd_aw<BF16, 128, 64, true>(p, stream) : launch_fwd_aw<BF16, 128, 64, false>(p, stream);
  return hipErrorNotSupported;
}

template __global__ void mfa_fwd_aw_kernel<F16, 128, 64, true>(FwdParams);
template __global__ void mfa_fwd_aw_kernel<F16, 128, 64, false>(FwdParams);
template __global__ void mfa_fwd_aw_kernel<BF16, 128, 64, true>(FwdParams);
template __global__ void mfa_fwd_aw_kernel<BF16, 128, 64, false>(FwdParams);

}  // namespace mfa
