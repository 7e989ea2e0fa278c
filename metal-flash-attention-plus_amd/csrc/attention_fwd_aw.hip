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
#ifdef AW_DEBUG_TRACE
__device__ float g_aw_trace[256];
#endif
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
// `keep`: the previous MFMA's P operand, held live until this MFMA issues.  The compiler sees
// an inline-assembly MFMA as done with its inputs when it issues, and may let the next VALU
// write their registers; the matrix core reads its B operand after issue, so a P register
// rewritten right behind its MFMA (the next tile's P packed in place) would be read late.
template <class E, int R, bool NOP>
__device__ __forceinline__ void pv_mfma(i16x8 a, i16x8 b, i16x8 keep, i16x8 keepa) {
  if constexpr (E::prec == P_FP16) {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a),
                   "v"(b), "n"(R), "v"(keep), "v"(keepa) : AW_O_CLOBBERS);
    else
      asm volatile("v_mfma_f32_32x32x16_f16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a), "v"(b),
                   "n"(R), "v"(keep), "v"(keepa) : AW_O_CLOBBERS);
  } else {
    if constexpr (NOP)
      asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a),
                   "v"(b), "n"(R), "v"(keep), "v"(keepa) : AW_O_CLOBBERS);
    else
      asm volatile("v_mfma_f32_32x32x16_bf16 a[%2:%2+15], %0, %1, a[%2:%2+15]" ::"v"(a), "v"(b),
                   "n"(R), "v"(keep), "v"(keepa) : AW_O_CLOBBERS);
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
  unsigned pt[2];      // words of the next tile's P held until the PV chain frees pw[0]
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
  using T_ = std::true_type;
  using F_ = std::false_type;
  constexpr bool PS = E::prec == P_FP16 && DP <= 128;
  constexpr int NJ = BK / 32, ND = DP / 32, DS = DP / 16;
  constexpr int NV = NJ * 16;                  // S values of a tile per lane (half its keys)
  constexpr int HV = NV / 2;                   // values of a sub-block per phase
  constexpr int TILEB = BK * DP * 2;
  constexpr int SLOT = (MIRROR ? 2 : 1) * TILEB;  // phase 2 stages two tiles per step
  constexpr float THR = 8.0f;
  constexpr int NKF = DS * NJ, NVF = NJ * 2 * ND;  // K / V fragments of a tile
  constexpr int NM = 2 * NKF;                  // MFMAs per phase (both sub-blocks)
  static_assert(DP == 128 && NKF == 16 && NVF == 16 && NM == 2 * HV, "one softmax value per MFMA gap");
  constexpr int OB0 = 0, OB1 = 64;             // AGPR bases of X0's and X1's O
  constexpr int AHK = AW_AHK, AHV = AW_AHV;
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

  // First key of X1's / X0's tile at step u (the same tile in phase 1).
  auto key1 = [&](int u) __attribute__((always_inline)) { return kb0 + (u < nA ? u : nA + 2 * (u - nA)) * BK; };
  auto key0 = [&](int u) __attribute__((always_inline)) { return kb0 + (u < nA ? u : nA + 2 * (u - nA) + 1) * BK; };
  auto kslot = [&](int u) __attribute__((always_inline)) { return kring + (u & 1) * SLOT; };
  auto vslot = [&](int u) __attribute__((always_inline)) { return vring + (u % 3) * SLOT; };
  auto dma_k = [&](int u) __attribute__((always_inline)) {
    kd.issue(khead, key1(u), kslot(u));
    if (MIRROR && u >= nA) kd.issue(khead, key0(u), kslot(u) + TILEB);
  };
  auto dma_v = [&](int u) __attribute__((always_inline)) {
    vd.issue(vhead, key1(u), vslot(u));
    if (MIRROR && u >= nA) vd.issue(vhead, key0(u), vslot(u) + TILEB);
  };

  // Prologue: K of steps 0 and 1 and V of step 0, then both sub-blocks' Q rows.
  dma_k(0);
  dma_v(0);
  if (U > 1) dma_k(1);
  i16x8 qf0[DS], qf1[DS];
  load_q2_raw<DP>(qf0, p, b, h, q00 + l32, q00 + l32 < p.R, hh);
  load_q2_raw<DP>(qf1, p, b, h, qB0 + l32, qB0 + l32 < p.R, hh);
  aw::Row st0, st1;
  st0.init();
  st1.init();
  aw::zero_o<0, 128>();
  aw::Soft<BK> sm0, sm1;
  sm0.reset();
  sm1.reset();
  // S of the current step (written by phase A) and the half of the previous step's S whose
  // values phase A's gaps still carry (key block 1).
  f32x16 sc0[NJ], sc1[NJ], sp0[NJ], sp1[NJ];
  wait_vm();
  prescale_q2<E, DP>(qf0, c);
  prescale_q2<E, DP>(qf1, c);
  aw::settle_writes();
  __syncthreads();
  AW_ACC_DECL();

  // Fragment streams.  Phase A (S = K·Q^T for both sub-blocks) reads each K fragment once for
  // both when they share a tile (SH), in key-block-major order (all of S[0] first); phase B
  // (O^T += V^T·P^T for both) reads each V fragment once likewise.  A phase's last read-ahead
  // slots prefetch the first fragments of the next phase (tail).
  i16x8 kp[2 * AHK], vp[2 * AHV];
  auto kread = [&](const char* kt, int f) __attribute__((always_inline)) {
    return A::read_row_a(kt, rbase, f / DS, f % DS);
  };
  auto vread = [&](const char* vt, int f) __attribute__((always_inline)) {
    const int jk = f / ND, dt = f % ND;
    return A::read_tr_a(vt, trb, (jk >> 1) * 32, jk & 1, dt * 32);
  };
  // Load n of a phase's stream: fragment n / 2 of sub-block n % 2's tile (not shared), or
  // fragment n (shared).
  auto kload = [&](auto sh_c, const char* k0t, const char* k1t, int n) __attribute__((always_inline)) {
    if constexpr (decltype(sh_c)::value) kp[n % AHK] = kread(k1t, n);
    else kp[n % (2 * AHK)] = kread((n & 1) ? k1t : k0t, n >> 1);
  };
  auto vload = [&](auto sh_c, const char* v0t, const char* v1t, int n) __attribute__((always_inline)) {
    if constexpr (decltype(sh_c)::value) vp[n % AHV] = vread(v1t, n);
    else vp[n % (2 * AHV)] = vread((n & 1) ? v1t : v0t, n >> 1);
  };
  auto no_tail = [](int) __attribute__((always_inline)) {};

  // Phase A: MFMA i updates S[j] of sub-block x = i % 2 with fragment f = i / 2 (j = f / DS).
  auto phase_a = [&](auto sh_c, const char* k0t, const char* k1t, auto&& hook, auto&& tail)
                     __attribute__((always_inline)) {
    constexpr bool SH = decltype(sh_c)::value;
    constexpr int NL = SH ? NKF : 2 * NKF, AH = SH ? AHK : 2 * AHK;
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int f = i / 2, x = i % 2, j = f / DS, ds = f % DS;
      const i16x8 kf = SH ? kp[f % AHK] : kp[i % (2 * AHK)];
      f32x16 (&s)[NJ] = x ? sc1 : sc0;
      s[j] = A::mma(kf, x ? qf1[ds] : qf0[ds], ds == 0 ? zero16() : s[j]);
      const int n = SH ? f : i;  // the load this MFMA consumed last
      if (!SH || x == 1) {
        if (n + AH < NL) kload(sh_c, k0t, k1t, n + AH);
        else tail(n + AH - NL);
      }
      hook(i);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // Phase B: MFMA i adds V fragment f = i / 2 times P of sub-block x = i % 2 to its O.
  auto phase_b = [&](auto sh_c, const char* v0t, const char* v1t, auto&& hook, auto&& tail)
                     __attribute__((always_inline)) {
    constexpr bool SH = decltype(sh_c)::value;
    constexpr int NL = SH ? NVF : 2 * NVF, AH = SH ? AHV : 2 * AHV;
    i16x8 vprev = SH ? vp[0] : vp[0];
    sfor<0, NM>([&](auto ic) {
      constexpr int i = decltype(ic)::value, f = i / 2, x = i % 2, jk = f / ND, dt = f % ND;
      const i16x8 vf = SH ? vp[f % AHV] : vp[i % (2 * AHV)];
      constexpr int ip = i > 0 ? i - 1 : 0, jkp = (ip / 2) / ND;
      aw::pv_mfma<E, (x ? OB1 : OB0) + 16 * dt, i == 0>(vf, x ? sm1.pb(jk) : sm0.pb(jk),
                                                      (ip & 1) ? sm1.pb(jkp) : sm0.pb(jkp), vprev);
      vprev = vf;
      if constexpr (i == NM - 1) asm volatile("s_nop 3" ::"v"(vf), "v"(x ? sm1.pb(jk) : sm0.pb(jk)));
      constexpr int n = SH ? f : i;
      if constexpr (!SH || x == 1) {
        if constexpr (n + AH < NL) vload(sh_c, v0t, v1t, n + AH);
        else tail(n + AH - NL);
      }
      hook(i);
      __builtin_amdgcn_sched_barrier(0);
    });
  };
  auto kpre = [&](auto sh_c, const char* k0t, const char* k1t) __attribute__((always_inline)) {
    constexpr int AH = decltype(sh_c)::value ? AHK : 2 * AHK;
    return [&, sh_c, k0t, k1t](int j) __attribute__((always_inline)) {
      if (j < AH) kload(sh_c, k0t, k1t, j);
    };
  };
  auto vpre = [&](auto sh_c, const char* v0t, const char* v1t) __attribute__((always_inline)) {
    constexpr int AH = decltype(sh_c)::value ? AHV : 2 * AHV;
    return [&, sh_c, v0t, v1t](int j) __attribute__((always_inline)) {
      if (j < AH) vload(sh_c, v0t, v1t, j);
    };
  };

  // Value k of a sub-block's tile: P = exp2(S·c − m) against the row max the decision before
  // the pass settled, row-sum partial, packed in place by pairs (the order of Arith16::pack).
  // The empty volatile statements pin each value where it is computed, in the MFMA gap it was
  // placed in; without them the compiler moves the sums and packs into bursts between phases.
  auto smv = [&](f32x16 (&s)[NJ], aw::Soft<BK>& sm, const aw::Row& st, int k, bool hold = false)
                 __attribute__((always_inline)) {
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
      if (hold) sm.pt[(k & 7) >> 1] = pk;
      else sm.pw[k >> 3][(k & 7) >> 1] = pk;
    }
  };
  // Gap i of phase B carries value i / 2 of the current S of sub-block i % 2; gap i of phase A
  // value HV + i / 2 of the previous S.
  // Phase B's MFMAs 0..7 still read the previous tile's P word block 0: the words its gaps
  // 0..7 complete are held and written at gap 8.
  auto gap_cur = [&](int i) __attribute__((always_inline)) {
    if (i & 1) smv(sc1, sm1, st1, i / 2, i < 8);
    else smv(sc0, sm0, st0, i / 2, i < 8);
    if (i == 8) {
      sm0.pw[0][0] = sm0.pt[0];
      sm0.pw[0][1] = sm0.pt[1];
      sm1.pw[0][0] = sm1.pt[0];
      sm1.pw[0][1] = sm1.pt[1];
    }
  };
  auto gap_prev = [&](int i) __attribute__((always_inline)) {
    if (i & 1) smv(sp1, sm1, st1, HV + i / 2);
    else smv(sp0, sm0, st0, HV + i / 2);
  };
  // The tile's row max (both lane halves), then the lazy-rescale decision (wave-uniform,
  // rarely taken).  Only the row state changes here; O is scaled after the phase that adds the
  // previous tile's P (corr, returned; 1 = nothing to do).
  auto decide = [&](const f32x16 (&s)[NJ], aw::Row& st) __attribute__((always_inline)) {
    float a4[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int jj = q >> 1, i0 = (q & 1) * 8;
      float m0 = __builtin_fmaxf(__builtin_fmaxf(s[jj][i0], s[jj][i0 + 1]), s[jj][i0 + 2]);
      m0 = __builtin_fmaxf(__builtin_fmaxf(m0, s[jj][i0 + 3]), s[jj][i0 + 4]);
      m0 = __builtin_fmaxf(__builtin_fmaxf(m0, s[jj][i0 + 5]), s[jj][i0 + 6]);
      a4[q] = __builtin_fmaxf(m0, s[jj][i0 + 7]);
    }
    const float mx = cross_half_max(__builtin_fmaxf(__builtin_fmaxf(a4[0], a4[1]), __builtin_fmaxf(a4[2], a4[3])));
    const float mt = PS ? mx : mx * c;
    bool scale = false;
    float corr = 1.f;
    if (__builtin_expect(__any(mt > st.m + THR), 0)) {
      MFA_KEEP_BRANCH();
      const float m_new = fmaxf(st.m, mt);
      corr = __builtin_amdgcn_exp2f(st.m - m_new);
      // Rows still at the initial max have O = 0 (every P so far was exp2(-inf)): no multiply.
      scale = !__all(st.m == -kFltMax);
      st.m = m_new;
      st.lh *= corr;
    }
    return scale ? corr : 1.f;
  };
  // After the tile's last value: l += Σ P.
  auto finish = [&](aw::Soft<BK>& sm, aw::Row& st) __attribute__((always_inline)) {
    st.lh += (sm.rs[0] + sm.rs[1]) + (sm.rs[2] + sm.rs[3]);
    sm.reset();
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
  auto store_x0 = [&](float m, float lh, int q0) __attribute__((always_inline)) {
    float l = cross_half_sum(lh) + kFltMin;
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
      if (hh == 0) store_l(p, m + __log2f(l), b, h, qi);
    }
  };
  // DMA pieces of a phase B: K of step u + 2 and V of step u + 1, one piece every other gap.
  auto dma_gap = [&](int u, int i) __attribute__((always_inline)) {
    if ((i & 1) == 0) {
      const int pc = i >> 1, which = pc & 3, k = pc >> 2;  // 16 slots: K1 V1 K0 V0 x 4
      const int uk = u + 2, uv = u + 1;
      if (which == 0 && uk < U) kd.issue_piece(khead, key1(uk), kslot(uk), k);
      if (which == 1 && uv < U) vd.issue_piece(vhead, key1(uv), vslot(uv), k);
      if (which == 2 && MIRROR && uk < U && uk >= nA) kd.issue_piece(khead, key0(uk), kslot(uk) + TILEB, k);
      if (which == 3 && MIRROR && uv < U && uv >= nA) vd.issue_piece(vhead, key0(uv), vslot(uv) + TILEB, k);
    }
  };

  float mA = 0.f, lA = 0.f;  // A's row state at the phase switch
  // Step u: phase A(u) [values HV.. of S(u-1)]; decisions on S(u); barrier; phase B(u): PV(u-1)
  // [values 0..HV-1 of S(u); DMA]; O scaled for decisions of u.
  auto step = [&](int u, auto first_c, auto sh_c, auto shp_c) __attribute__((always_inline)) {
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr bool SH = decltype(sh_c)::value;    // X0 and X1 read one K tile at step u
    constexpr bool SHP = decltype(shp_c)::value;  // ... and one V tile at step u - 1
    const bool sw = MIRROR && u == nA && nA > 0;
    if (sw) {
#pragma unroll
      for (int ds = 0; ds < DS; ++ds) qf0[ds] = qf1[ds];
    }
    const char* kt1 = kslot(u);
    const char* kt0 = kt1 + (SH ? 0 : TILEB);
    const char* vt1 = vslot(u - 1);
    const char* vt0 = vt1 + (SHP ? 0 : TILEB);
    if constexpr (FIRST) {
#pragma unroll
      for (int j = 0; j < (SH ? AHK : 2 * AHK); ++j) kload(sh_c, kt0, kt1, j);
      phase_a(sh_c, kt0, kt1, no_tail, no_tail);
    } else {
#ifdef AW_DBG_NOPRE
      if constexpr (!SH) {
#pragma unroll
        for (int j = 0; j < 2 * AHK; ++j) kload(sh_c, kt0, kt1, j);
      }
#endif
      phase_a(sh_c, kt0, kt1, gap_prev, vpre(shp_c, vt0, vt1));
    }
    AW_ACC(0);
    if constexpr (!FIRST) {
      finish(sm0, st0);
      finish(sm1, st1);
    }
    if (sw) {  // A's last values are summed: keep its state, X0 starts B's second state
      mA = st0.m;
      lA = st0.lh;
      st0.init();
      q00 = qB0;
    }
    mask(sc0, key0(u), q00);
    mask(sc1, key1(u), qB0);
    const float corr0 = decide(sc0, st0);
    const float corr1 = decide(sc1, st1);
#ifdef AW_DEBUG_TRACE
    if (blockIdx.x == 0 && tid == 0 && u < 16) {
      g_aw_trace[u * 8 + 0] = st0.m; g_aw_trace[u * 8 + 1] = st0.lh; g_aw_trace[u * 8 + 2] = corr0;
      g_aw_trace[u * 8 + 3] = st1.m; g_aw_trace[u * 8 + 4] = st1.lh; g_aw_trace[u * 8 + 5] = corr1;
    }
#endif
    AW_ACC(1);
    wait_vm();
    AW_ACC(2);
    __syncthreads();
    AW_ACC(3);
    // K of step u + 1 is now valid for every wave: phase B's tail may prefetch it.
    const bool shn = !MIRROR || u + 1 < nA;
    const char* kn1 = kslot(u + 1);
    const char* kn0 = kn1 + (shn ? 0 : TILEB);
    auto tail = [&](int j) __attribute__((always_inline)) {
#ifdef AW_DBG_NOPRE
      if (!shn) return;
#endif
      if (u + 1 < U) {
        if (shn) kpre(T_(), kn0, kn1)(j);
        else kpre(F_(), kn0, kn1)(j);
      }
    };
    if constexpr (FIRST) {
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        gap_cur(i);
        dma_gap(u, i);
      }
#pragma unroll
      for (int j = 0; j < 2 * AHK; ++j) tail(j);
    } else {
      phase_b(shp_c, vt0, vt1, [&](int i) __attribute__((always_inline)) {
        gap_cur(i);
        dma_gap(u, i);
      }, [&](int j) __attribute__((always_inline)) {
        // Phase B's tail has fewer slots than phase A needs: its last one loads the rest.
        constexpr int AHB = SHP ? AHV : 2 * AHV;
        if (j < AHB - 1) tail(j);
        else if (j == AHB - 1) {
#pragma unroll
          for (int r = AHB - 1; r < 2 * AHK; ++r) tail(r);
        }
      });
    }
    AW_ACC(4);
    if (sw) {  // A's last P has been added (PV(u - 1) above): A leaves, X0's O restarts
      store_x0(mA, lA, rbA * 128 + 32 * w);
      aw::zero_o<OB0, 64>();
      aw::settle_writes();
    }
    if (__builtin_expect(corr0 != 1.f, 0)) aw::scale_o<OB0>(corr0);
    if (__builtin_expect(corr1 != 1.f, 0)) aw::scale_o<OB1>(corr1);
#ifdef AW_DEBUG_TRACE
    {
      aw::drain_mfma();
      const float a0v = aread<0>(), a64v = aread<64>();
      if (blockIdx.x == 0 && tid == 0 && u < 16) { g_aw_trace[u * 8 + 6] = a0v; g_aw_trace[u * 8 + 7] = a64v; }
    }
#endif
    // The half of S whose values the next phase A carries.
    sp0[NJ - 1] = sc0[NJ - 1];
    sp1[NJ - 1] = sc1[NJ - 1];
    AW_ACC(5);
  };

  if (U > 0) {
    if (nA == 0 && MIRROR) step(0, T_(), F_(), F_());
    else step(0, T_(), T_(), T_());
    int u = 1;
    if constexpr (MIRROR) {
      for (; u < nA && u < U; ++u) step(u, F_(), T_(), T_());
      if (u < U && u == nA && nA > 0) {
        step(u, F_(), F_(), T_());  // the switch step: K tiles split, V still shared
        ++u;
      }
      for (; u < U; ++u) step(u, F_(), F_(), F_());
    } else {
      for (; u < U; ++u) step(u, F_(), T_(), T_());
    }
    // Drain: values HV.. of S(U - 1), then PV(U - 1).
#pragma unroll
    for (int i = 0; i < NM; ++i) gap_prev(i);
    finish(sm0, st0);
    finish(sm1, st1);
    const bool shl = !MIRROR || U - 1 < nA;
    const char* vt1 = vslot(U - 1);
    const char* vt0 = vt1 + (shl ? 0 : TILEB);
    if (shl) {
#pragma unroll
      for (int j = 0; j < AHV; ++j) vload(T_(), vt0, vt1, j);
      phase_b(T_(), vt0, vt1, no_tail, no_tail);
    } else {
#pragma unroll
      for (int j = 0; j < 2 * AHV; ++j) vload(F_(), vt0, vt1, j);
      phase_b(F_(), vt0, vt1, no_tail, no_tail);
    }
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
