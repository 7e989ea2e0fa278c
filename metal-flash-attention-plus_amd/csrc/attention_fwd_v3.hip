// attention_fwd_v3.hip — third-generation forward for 16-bit Q/K/V at D = 128 on gfx950.
//
// Same algorithm and numerics contract as attention_fwd_v2.hip (the reference forward,
// AttentionKernel+Source.swift:372-416: S = QK^T, base-2 online softmax with lazy rescale,
// O = PV / l, L = m + log2 l), for no mask or the causal mask.
//
// What changes is the organisation of the work, aimed at the two limits measured on v2
// (DESIGN.md §3): a wave's own softmax could not overlap its own MFMAs (QK^T -> max -> exp ->
// PV is one dependency chain), and the 8-wave pair kernel's barrier put both waves of a SIMD
// in the same phase at the same time.  Here:
//   * one 256-thread workgroup per CU, one wave per SIMD with the whole 512-entry register
//     file; every wave carries TWO 32-row accumulator streams A and B;
//   * the streams are software-pipelined half a tile apart, so every MFMA phase of one stream
//     has the other stream's softmax beside it:
//         M1: S_A = K·Q_A^T               | exp, row sum, pack of B's previous tile
//         M2: O_B += V·P_B^T (previous)   | row max of A
//         -- barrier (K/V tiles issued one iteration earlier are complete); rare rescale of A
//         M3: S_B = K·Q_B^T               | exp, row sum, pack of A
//         M4: O_A += V·P_A^T              | row max of B      [LDS-DMA: V of j+1, K of j+2]
//         -- rare rescale of B
//   * every phase issues the first fragment reads of the NEXT phase in its own MFMA gaps, so
//     no phase starts by waiting for LDS (with one wave per SIMD nothing else hides that
//     latency; v3's first build, which read each phase's fragments just in time, spent 31 %
//     of its wave cycles in s_waitcnt);
//   * masks are applied through the initial accumulator of the QK^T chain (-inf at masked
//     keys), so the steady-state phases carry no mask code at all;
//   * non-causal: a workgroup owns 256 query rows (stream A rows 0-127, stream B rows
//     128-255), both streams read the same K/V tile, so the K/V bytes staged per MFMA are half
//     of v2's;
//   * causal: a workgroup owns the mirrored pair of 128-row blocks X (light) and Y (heavy) of
//     one head (equal work for every workgroup).  Phase 1: A = X rows, B = Y rows on the same
//     tile, until X's keys end; X is then stored and phase 2 runs A and B over Y's remaining
//     key tiles alternately (A even, B odd), two partial softmax states of the same rows that
//     merge in registers at the end.
// LDS: a 5-slot K ring and a 4-slot V ring (16 KiB tiles, 144 KiB).  K tiles are staged two
// iterations ahead (the next iteration's first QK^T fragments are read during M4, before the
// iteration boundary), V tiles one ahead; every DMA of iteration j is issued in M4 and waited
// for at iteration j+1's barrier, which is also what makes its slot reuse safe.
#include <mutex>
#include <type_traits>

#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {
namespace fwd3 {

constexpr int DP = 128, BK = 64, ND = DP / 32, DS = DP / 16, NJ = BK / 32;
constexpr int TILEB = BK * DP * 2;  // one K or V tile: 16 KiB
constexpr int KSLOTS = 5, VSLOTS = 4;
constexpr int LDS_BYTES = (KSLOTS + VSLOTS) * TILEB;  // 144 KiB
constexpr int NM = 16;                                // MFMAs per phase (either product)
constexpr float THR = 8.0f;
using DMA = DmaA<DP, BK, 256>;

// Scheduling fence for MFMAs and LDS reads only: VALU, SALU and transcendental instructions
// (the other stream's softmax) may still move across it into the MFMA chain, but fragment
// reads stay where the source puts them (hoisted, they would hold dozens of extra registers).
__device__ __forceinline__ void pin_mem_order() { __builtin_amdgcn_sched_barrier(0x0406); }

// One 32-row accumulator stream of a wave: the lane's query row, halves split D.
struct Stream {
  f32x16 o[ND];
  f32x16 s[NJ];
  i16x8 pb[2 * NJ];
  f32x16 negm;  // −moff in every register (fp16): the QK^T chain's initial accumulator
  float m;      // running max (log2 units)
  float moff;   // max folded into S' by the MFMA (fp16)
  float lh;     // partial row sum of this half-wave's keys
  __device__ __forceinline__ void init() {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
      o[dt] = zero16();
      asm volatile("" : "+a"(o[dt]));  // O lives in AGPRs (see mfma_acc_a)
    }
    negm = zero16();
    m = -kFltMax;
    moff = 0.f;
    lh = 0.f;
  }
};

// First MFMA of a QK^T chain in the untied form (dst != srcC).  As a builtin, hipcc picks the
// tied form for one of the two chains and copies the 16-register initial tile into it first
// (8 v_mov_b64 per chain and tile).  The leading s_nop covers a VALU write of the initial tile
// just before (2 wait states); the builtin MFMAs that continue the chain accumulate into the
// same registers, which the hardware interlocks.
template <class E>
__device__ __forceinline__ f32x16 mfma_first(const i16x8& a, const i16x8& b, const f32x16& c) {
  f32x16 d;
  if constexpr (E::prec == P_FP16)
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
  else
    asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %3" : "=&v"(d) : "v"(a), "a"(b), "v"(c));
  return d;
}

// O^T += V^T·P^T on an AGPR accumulator.  The builtin MFMA would pin every accumulator of the
// kernel to one register file (-mfma-vgpr-form puts all in VGPRs, which then spill Q and the
// DMA offsets into AGPRs and reload them before every use); as inline asm, O lives in AGPRs
// (only the PV chain and the rare rescale touch it) while S stays in VGPRs for the softmax.
// hipcc does not pad hazards inside asm: the leading s_nop covers a VALU write of P (or an
// AGPR write of O) right before the MFMA (2 wait states needed, 3 given); O is read back by
// VALU only after mfma_drain() or a barrier plus an MFMA phase.
template <class E>
__device__ __forceinline__ void mfma_acc_a(f32x16& acc, const i16x8& a, const i16x8& b) {
  if constexpr (E::prec == P_FP16)
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_f16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else
    asm volatile("s_nop 2\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}
// Covers the MFMA -> VALU read latency of an asm MFMA's accumulator (16 passes).
__device__ __forceinline__ void mfma_drain() {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
}

// Fragment k (0..15) of a phase's operand: QK^T reads K rows (k -> key half k % 2, k-step
// k / 2), PV reads V transposed (k -> key step k / ND, head-dim tile k % ND).
template <class E>
struct KFrag {
  const char* t;
  const int* rb;
  __device__ __forceinline__ i16x8 operator()(int k) const {
    const int rbase[2] = {rb[0], rb[1]};
    return Arith16<E, DP>::read_row_a(t, rbase, k % NJ, k / NJ);
  }
};
template <class E>
struct VFrag {
  const char* t;
  const int* tb;
  __device__ __forceinline__ i16x8 operator()(int k) const {
    const int trb[2] = {tb[0], tb[1]};
    const int jk = k / ND, dt = k % ND;
    return Arith16<E, DP>::read_tr_a(t, trb, (jk >> 1) * 32, jk & 1, dt * 32);
  }
};

// S^T = K·Q^T (16 MFMAs): key on the MFMA row (registers), query on the lane.  i0 / i1 are
// the initial accumulators of keys 0-31 / 32-63 (−m, or 0 for bf16; −inf where masked).
// cur: this phase's first NP fragments (read by the previous phase); nxt <- the next
// phase's first NP fragments, read in this phase's last MFMA gaps.  slot(i) issues the VALU
// work placed in MFMA gap i (a slice of the other stream's softmax); every gap is closed by a
// full scheduling barrier, so the interleave is exactly the source order (hipcc, left to
// itself, clusters the softmax VALU and leaves the matrix pipe idle between MFMA runs).
template <class E, int NP, class Next, class Slot>
__device__ __forceinline__ void qk(Stream& st, const KFrag<E>& rd, const i16x8 (&qf)[DS],
                                   const f32x16& i0, const f32x16& i1, i16x8 (&cur)[NP],
                                   i16x8 (&nxt)[NP], const Next& rdn, Slot&& slot) {
  using A = Arith16<E, DP>;
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int ds = i / NJ, j = i % NJ;
    if (ds == 0)
      st.s[j] = mfma_first<E>(cur[i % NP], qf[0], j == 0 ? i0 : i1);
    else
      st.s[j] = A::mma(cur[i % NP], qf[ds], st.s[j]);
    if (i + NP < NM)
      cur[i % NP] = rd(i + NP);
    else
      nxt[i + NP - NM] = rdn(i + NP - NM);
    slot(i);
    __builtin_amdgcn_sched_barrier(0);
  }
  slot(NM);  // the pipelined slices' last stage, right behind the chain
  __builtin_amdgcn_sched_barrier(0);
}

// O^T += V^T·P^T (16 MFMAs), same fragment pipeline and gap slots (slot(i), i < 16).
template <class E, int NP, class Next, class Slot>
__device__ __forceinline__ void pv(Stream& st, const VFrag<E>& rd, i16x8 (&cur)[NP],
                                   i16x8 (&nxt)[NP], const Next& rdn, Slot&& slot) {
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int jk = i / ND, dt = i % ND;
    mfma_acc_a<E>(st.o[dt], cur[i % NP], st.pb[jk]);
    if (i + NP < NM)
      cur[i % NP] = rd(i + NP);
    else
      nxt[i + NP - NM] = rdn(i + NP - NM);
    slot(i);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Two fp32 values rounded to one packed 16-bit pair (v_cvt_pk_f16_f32 / v_cvt_pk_bf16_f32).
template <class E>
__device__ __forceinline__ uint32_t pack2(float a, float b) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  if constexpr (E::prec == P_FP16) {
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, h2));
  } else {
    typedef __bf16 b2 __attribute__((ext_vector_type(2)));
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(f2{a, b}, b2));
  }
}

// Slice i (0..16) of a stream's softmax for one MFMA gap, software-pipelined by one gap so
// nothing waits on the transcendental latency: P = exp2(S') of elements 2i, 2i+1 (i < 16),
// then the 16-bit pack (one operand word) and the row-sum share (two partial sums) of the
// pair exponentiated in the previous gap (i > 0).
template <class E, bool PS>
__device__ __forceinline__ void expo_slice(Stream& st, float c, int i, float (&rs)[2]) {
  if (i < 16) {
    const int j = i / 8, e = 2 * (i % 8);
    float x0 = st.s[j][e], x1 = st.s[j][e + 1];
    if constexpr (!PS) {
      x0 = __builtin_fmaf(x0, c, -st.m);
      x1 = __builtin_fmaf(x1, c, -st.m);
    }
    st.s[j][e] = __builtin_amdgcn_exp2f(x0);
    st.s[j][e + 1] = __builtin_amdgcn_exp2f(x1);
  }
  if (i > 0) {
    const int h = i - 1, j = h / 8, e = 2 * (h % 8);
    const float p0 = st.s[j][e], p1 = st.s[j][e + 1];
    rs[0] += p0;
    rs[1] += p1;
    const int jk = j * 2 + (h % 8) / 4, w = h % 4;
    const uint32_t word = pack2<E>(p0, p1);
    uint4 v = __builtin_bit_cast(uint4, st.pb[jk]);
    if (w == 0) v.x = word;
    if (w == 1) v.y = word;
    if (w == 2) v.z = word;
    if (w == 3) v.w = word;
    st.pb[jk] = __builtin_bit_cast(i16x8, v);
  }
}

// Slice i (0..15) of a stream's row max: elements 2i, 2i+1 into one of four maximum chains.
__device__ __forceinline__ void max_slice(const Stream& st, int i, float (&r)[4]) {
  const int j = i / 8, e = 2 * (i % 8), k = i % 4;
  const float a = st.s[j][e], b = st.s[j][e + 1];
  r[k] = i < 4 ? __builtin_elementwise_maximum(a, b)
               : __builtin_elementwise_maximum(r[k], __builtin_elementwise_maximum(a, b));
}
template <bool PS>
__device__ __forceinline__ float max_final(const Stream& st, const float (&r)[4], float c) {
  const float mx = cross_half_maximum(__builtin_elementwise_maximum(
      __builtin_elementwise_maximum(r[0], r[1]), __builtin_elementwise_maximum(r[2], r[3])));
  return PS ? mx + st.moff : mx * c;
}

// Tile max of the lane's row in absolute log2 units (both halves).
template <bool PS>
__device__ __forceinline__ float rowmax(const Stream& st, float c) {
  // Four independent chains (v_maximum3_f32: no operand canonicalisation, unlike fmaxf).
  float r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int j = k >> 1, i0 = 8 * (k & 1);
    float x = __builtin_elementwise_maximum(st.s[j][i0], st.s[j][i0 + 1]);
#pragma unroll
    for (int i = 2; i < 8; ++i) x = __builtin_elementwise_maximum(x, st.s[j][i0 + i]);
    r[k] = x;
  }
  const float mx = cross_half_maximum(__builtin_elementwise_maximum(
      __builtin_elementwise_maximum(r[0], r[1]), __builtin_elementwise_maximum(r[2], r[3])));
  return PS ? mx + st.moff : mx * c;
}

// Lazy rescale (threshold THR in log2 units, cdna_hip_programming.md T13): a rare, wave-uniform
// branch placed between phases, where the stream's O is not in use by an MFMA.
template <bool PS>
__device__ __forceinline__ void rescale(Stream& st, float mt) {
  if (__any(mt > st.m + THR)) {
    MFA_KEEP_BRANCH();
    const float m_new = fmaxf(st.m, mt);
    const float corr = __builtin_amdgcn_exp2f(st.m - m_new);
    st.m = m_new;
    st.lh *= corr;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) st.o[dt][i] *= corr;
      asm volatile("" : "+a"(st.o[dt]));  // back to AGPRs inside the rare branch
    }
    if constexpr (PS) {
      // Rows still at the initial max saw only masked keys (S' = −inf): keep their offset.
      const float moff_new = m_new > kMaskLevel ? m_new : st.moff;
      const float shift = moff_new - st.moff;
      st.moff = moff_new;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) st.s[j][i] -= shift;
#pragma unroll
      for (int i = 0; i < 16; ++i) st.negm[i] = -moff_new;
    }
  }
}

// P = exp2(S'), its row sum, then P packed to the 16-bit B operands of the PV product (the
// fp32 P dies at the pack, so the packed operand can take its registers).
template <class E, bool PS>
__device__ __forceinline__ void expo(Stream& st, float c) {
  using A = Arith16<E, DP>;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float x = PS ? st.s[j][i] : __builtin_fmaf(st.s[j][i], c, -st.m);
      st.s[j][i] = __builtin_amdgcn_exp2f(x);
    }
  float r0 = 0.f, r1 = 0.f, r2 = 0.f, r3 = 0.f;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      r0 += st.s[j][i];
      r1 += st.s[j][i + 1];
      r2 += st.s[j][i + 2];
      r3 += st.s[j][i + 3];
    }
  st.lh += (r0 + r1) + (r2 + r3);
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) st.pb[j * 2 + ks] = A::pack(st.s[j], ks);
}

// Initial accumulators of a masked tile: keys t + 32j + acc_row(i, hh) past `hi` (the row's
// last visible key, relative to t + 4hh) are −inf.
template <bool PS>
__device__ __forceinline__ void masked_init(const Stream& st, int hi, f32x16& i0, f32x16& i1) {
  asm volatile("" : "+v"(hi));  // keeps the compares below inside the (rare) branch
  const float base = PS ? -st.moff : 0.f;
  const float ninf = -__builtin_inff();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int kk = (i & 3) + 8 * (i >> 2);
    i0[i] = kk > hi ? ninf : base;
    i1[i] = kk + 32 > hi ? ninf : base;
  }
}

template <class E, bool PS>
__device__ __forceinline__ void load_q(i16x8 (&qf)[DS], const FwdParams& p, int b, int h, int qi,
                                       bool qvalid, int hh, float c) {
  const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh +
                         (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
  for (int s = 0; s < DS; ++s) {
    const int d0 = 16 * s + 8 * hh;
    i16x8 v = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (qvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
    if constexpr (PS) {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (short)E::from_f32(E::to_f32((uint16_t)v[j]) * c);
    }
    // Q is read only by the QK^T MFMAs, which take it straight from AGPRs.
    asm volatile("" : "=a"(qf[s]) : "0"(v));
  }
}

// Final O = O / l and L = m + log2 l of one stream's rows.
__device__ __forceinline__ void store_stream(const FwdParams& p, const f32x16 (&o)[ND], float m,
                                             float lh, int b, int h, int qi, bool qvalid, int hh) {
  float l = cross_half_sum(lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if (!qvalid) return;
  const float inv = p.o_mul / l;
  float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = dt * 32 + 8 * g + 4 * hh;
      if (d < p.D)
        *reinterpret_cast<float4*>(orow + d) =
            make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
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

template <int V> using IC = std::integral_constant<int, V>;

// Diagnostic build only (tools/diag/v3_stamps.hip defines V3_STAMPS): per-wave shader-cycle
// totals of the iteration's segments, into a buffer no kernel output is computed from.
#ifdef V3_STAMPS
__device__ unsigned long long g_v3_stamps[1 << 16][8];
#define V3_SEG_DECL() unsigned long long seg_[8] = {0, 0, 0, 0, 0, 0, 0, 0}, segt_ = v3_clock()
#define V3_SEG(k)                          \
  do {                                     \
    const unsigned long long t_ = v3_clock(); \
    seg_[k] += t_ - segt_;                 \
    segt_ = t_;                            \
  } while (0)
#define V3_SEG_END()                                                                 \
  do {                                                                               \
    if ((threadIdx.x & 63) == 0)                                                     \
      for (int k_ = 0; k_ < 8; ++k_)                                                 \
        g_v3_stamps[blockIdx.x * 4 + (threadIdx.x >> 6)][k_] = seg_[k_];             \
  } while (0)
__device__ __forceinline__ unsigned long long v3_clock() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#else
#define V3_SEG_DECL() do {} while (0)
#define V3_SEG(k) do {} while (0)
#define V3_SEG_END() do {} while (0)
#endif

// TUNE (development A/B): 0 = shipped; 1 = steady-state DMA spread over M3 and M4;
// 2 = no DMA in the steady loop (timing ablation, wrong results); 3 = 8 fragments read ahead.
template <class E, bool CAUSAL, int TUNE = 0>
__global__ void __launch_bounds__(256, 1) mfa_fwd3_kernel(FwdParams p) {
  constexpr bool PS = E::prec == P_FP16;
  constexpr int NP = TUNE == 3 ? 8 : 6;  // fragments read ahead
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kring = smem;
  char* const vring = smem + KSLOTS * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};

  // Work unit: (b, h) and the two 128-row blocks X (stream A in phase 1) and Y (stream B).
  const int BH = p.B * p.H;
  int bh, u;
  xcd_unit_block(blockIdx.x, BH, p.nblk, &bh, &u);
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int nb128 = (p.R + 127) / 128;
  int X, Y;
  if (CAUSAL) {
    X = u;
    Y = nb128 - 1 - u;
  } else {
    X = 2 * u;
    Y = 2 * u + 1;
  }
  const int q0X = 128 * X, q0Y = 128 * Y;
  const int qiX = q0X + 32 * wave + l32, qiY = q0Y + 32 * wave + l32;
  const float c = p.c_log2;

  // Tile schedule.  Phase 1 (j < n1): A and B read tile j.  Phase 2: A reads n1 + 2(j − n1),
  // B the tile after it.
  const int ntile = (p.C + BK - 1) / BK;
  int n1, n2;
  if (CAUSAL) {
    const int nY = (min(p.C, q0Y + 128) + BK - 1) / BK;
    n1 = X == Y ? 0 : (min(p.C, q0X + 128) + BK - 1) / BK;
    n2 = (nY - n1 + 1) / 2;
  } else {
    n1 = ntile;
    n2 = 0;
  }
  const int J = n1 + n2;
  auto ta_of = [&](int j) { return j < n1 ? j : n1 + 2 * (j - n1); };
  auto tb_of = [&](int j) { return j < n1 ? j : n1 + 2 * (j - n1) + 1; };
  auto tiles_of = [&](int j) { return j >= J ? 0 : j < n1 ? 1 : 2; };
  // Last key visible to the lane's row in tile t, relative to t + 4·hh (masked_init).
  auto hi_of = [&](int t, int qi) {
    const int base = t * BK + 4 * hh;
    int hi = p.C - 1 - base;
    if (CAUSAL) hi = min(hi, qi - base);
    return hi;
  };
  auto needs_mask = [&](int t, int q0) {
    return t * BK + BK > p.C || (CAUSAL && t * BK + BK - 1 > q0);
  };

  DMA kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;
  auto kslot = [&](int t) { return kring + (int)((unsigned)t % KSLOTS) * TILEB; };
  auto vslot = [&](int t) { return vring + (t & (VSLOTS - 1)) * TILEB; };
  auto issue_k = [&](int j) {  // K tiles of iteration j
    const int n = tiles_of(j);
    if (n >= 1) kd.issue(khead, ta_of(j) * BK, kslot(ta_of(j)));
    if (n >= 2) kd.issue(khead, tb_of(j) * BK, kslot(tb_of(j)));
  };
  auto issue_v = [&](int j) {  // V tiles of iteration j
    const int n = tiles_of(j);
    if (n >= 1) vd.issue(vhead, ta_of(j) * BK, vslot(ta_of(j)));
    if (n >= 2) vd.issue(vhead, tb_of(j) * BK, vslot(tb_of(j)));
  };

  issue_k(0);
  issue_v(0);
  issue_k(1);
  i16x8 qX[DS], qY[DS];
  load_q<E, PS>(qX, p, b, h, qiX, qiX < p.R, hh, c);
  load_q<E, PS>(qY, p, b, h, qiY, qiY < p.R, hh, c);
  Stream sa, sb;
  sa.init();
  sb.init();
  // Stream B enters the first iteration with a "previous tile" whose scores are all -inf:
  // its exp, PV (against the loaded first V tile: finite values times P = 0) and row sum add
  // exactly nothing, so no iteration needs a separate first-tile body.
#pragma unroll
  for (int j = 0; j < NJ; ++j) sb.s[j] = zero16() - __builtin_inff();
  wait_vm();
  __syncthreads();

  // Fragment pipeline registers: kf feeds the QK^T phases, vf the PV phases.
  i16x8 kf[NP], vf[NP];
  if (J > 0) {
    const KFrag<E> r0{kslot(ta_of(0)), rbase};
#pragma unroll
    for (int k = 0; k < NP; ++k) kf[k] = r0(k);
  }

  // One pipelined iteration.  TIL: tiles per iteration in this loop (1 phase 1, 2 phase 2;
  // fixes the DMA issue count of the steady state), -1 = decided at run time.  MASKS: 0 = no
  // tile of the iteration is masked (no mask code at all), 1 = masks decided at run time.
  V3_SEG_DECL();
  auto iter = [&](auto til_c, auto masks_c, const i16x8(&qa)[DS], int j, int q0a, int qia) {
    constexpr int TIL = decltype(til_c)::value;
    constexpr bool MASKS = decltype(masks_c)::value != 0;
    const int ta = ta_of(j), tb = tb_of(j);
    const int tbp = j > 0 ? tb_of(j - 1) : ta;
    // The next iteration's first K tile (the last iteration reads its own again, harmlessly:
    // a branch here would put a control-flow join right behind the PV chain, where hipcc may
    // copy O between AGPRs before the last asm MFMA has written it).
    const int tn = (TIL > 0 || j + 1 < J) ? ta_of(j + 1) : ta;
    const KFrag<E> kA{kslot(ta), rbase}, kB{kslot(tb), rbase}, kN{kslot(tn), rbase};
    const VFrag<E> vBp{vslot(tbp), trb}, vA{vslot(ta), trb};

    // ---- M1: S_A = K·Q_A^T | exp, row sum, pack of B's previous tile; reads for M2
    float rsb[2] = {0.f, 0.f};
    auto m1 = [&](int i) { expo_slice<E, PS>(sb, c, i, rsb); };
    if (MASKS && needs_mask(ta, q0a)) {
      f32x16 i0, i1;
      masked_init<PS>(sa, hi_of(ta, qia), i0, i1);
      qk<E, NP>(sa, kA, qa, i0, i1, kf, vf, vBp, m1);
    } else {
      qk<E, NP>(sa, kA, qa, PS ? sa.negm : zero16(), PS ? sa.negm : zero16(), kf, vf, vBp, m1);
    }
    sb.lh += rsb[0] + rsb[1];
    V3_SEG(6);
    // ---- M2: O_B += V·P_B^T (B's previous tile) | row max of A; reads for M3
    float ra[4];
    pv<E, NP>(sb, vBp, vf, kf, kB, [&](int i) { max_slice(sa, i, ra); });
    if constexpr (MASKS) mfma_drain();
    const float mta = max_final<PS>(sa, ra, c);
    V3_SEG(0);
    // Tiles issued in the previous iteration's M4 have landed (every wave's own pieces), and
    // after the barrier every wave has passed M2: their slots may be refilled in M4 below.
    wait_vm();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    V3_SEG(1);
    rescale<PS>(sa, mta);
    V3_SEG(2);

    // ---- M3: S_B = K·Q_B^T | exp, row sum, pack of A; reads for M4
    float rsa[2] = {0.f, 0.f};
    auto m3 = [&](int i) {
      expo_slice<E, PS>(sa, c, i, rsa);
      if constexpr (TUNE == 1 && TIL == 1) {
        if (i % 4 == 2) kd.issue_piece(khead, (j + 2) * BK, kslot(j + 2), i / 4);
      }
    };
    if (MASKS && needs_mask(tb, q0Y)) {
      f32x16 i0, i1;
      masked_init<PS>(sb, hi_of(tb, qiY), i0, i1);
      qk<E, NP>(sb, kB, qY, i0, i1, kf, vf, vA, m3);
    } else {
      qk<E, NP>(sb, kB, qY, PS ? sb.negm : zero16(), PS ? sb.negm : zero16(), kf, vf, vA, m3);
    }
    sa.lh += rsa[0] + rsa[1];
    V3_SEG(7);
    // ---- M4: O_A += V·P_A^T | row max of B; reads for the next M1; DMA (V of j+1, K of j+2)
    float rb[4];
    if constexpr (TIL == 1 && (TUNE == 1 || TUNE == 2)) {
      // TUNE 1: the K half of the DMA went into M3's gaps (below the QK^T call).
      pv<E, NP>(sa, vA, vf, kf, kN, [&](int i) {
        max_slice(sb, i, rb);
        if (TUNE == 1 && i % 4 == 2) vd.issue_piece(vhead, (j + 1) * BK, vslot(j + 1), i / 4);
      });
    } else if constexpr (TIL == 1) {
      // One DMA piece in every other gap.
      pv<E, NP>(sa, vA, vf, kf, kN, [&](int i) {
        max_slice(sb, i, rb);
        if (i % 2 == 0) {
          if (i < 2 * DMA::PPW)
            vd.issue_piece(vhead, (j + 1) * BK, vslot(j + 1), i / 2);
          else
            kd.issue_piece(khead, (j + 2) * BK, kslot(j + 2), i / 2 - DMA::PPW);
        }
      });
    } else if constexpr (TIL == 2) {
      const int a1 = ta_of(j + 1), a2 = ta_of(j + 2);
      pv<E, NP>(sa, vA, vf, kf, kN, [&](int i) {
        max_slice(sb, i, rb);
        const int q = i % DMA::PPW, t = i / DMA::PPW;
        if (t == 0) vd.issue_piece(vhead, a1 * BK, vslot(a1), q);
        if (t == 1) vd.issue_piece(vhead, (a1 + 1) * BK, vslot(a1 + 1), q);
        if (t == 2) kd.issue_piece(khead, a2 * BK, kslot(a2), q);
        if (t == 3) kd.issue_piece(khead, (a2 + 1) * BK, kslot(a2 + 1), q);
      });
    } else {
      issue_v(j + 1);
      issue_k(j + 2);
      pv<E, NP>(sa, vA, vf, kf, kN, [&](int i) { max_slice(sb, i, rb); });
    }
    if constexpr (MASKS) mfma_drain();  // generic bodies end in branches and joins
    const float mtb = max_final<PS>(sb, rb, c);
    V3_SEG(3);
    rescale<PS>(sb, mtb);
    V3_SEG(4);
  };

  // Masked tiles (causal diagonal, the key edge, phase 2's filler tile) only ever fall in the
  // last two iterations of a phase, and the steady body also needs the next two iterations
  // to be of its own phase: so each phase is a steady loop plus two straight-line generic
  // iterations.  (A generic body inside a loop gets merged with the steady loop by the
  // compiler, and the two register assignments then cost AGPR copies every iteration.)
  int j = 0;
  for (const int e1 = n1 - 2; j < e1; ++j) iter(IC<1>(), IC<0>(), qX, j, q0X, qiX);
  mfma_drain();
  if (j < n1) iter(IC<-1>(), IC<1>(), qX, j++, q0X, qiX);
  if (j < n1) iter(IC<-1>(), IC<1>(), qX, j++, q0X, qiX);
  if (CAUSAL) {
    if (n1 > 0) {
      // X is complete: store it and restart stream A on Y's second key range.
      mfma_drain();
      store_stream(p, sa.o, sa.m, sa.lh, b, h, qiX, qiX < p.R, hh);
      sa.init();
    }
    for (const int e2 = J - 2; j < e2; ++j) iter(IC<2>(), IC<0>(), qY, j, q0Y, qiY);
    mfma_drain();
    if (j < J) iter(IC<-1>(), IC<1>(), qY, j++, q0Y, qiY);
    if (j < J) iter(IC<-1>(), IC<1>(), qY, j++, q0Y, qiY);
  }
  V3_SEG(5);
  V3_SEG_END();
  // B's last tile.
  if (J > 0) {
    expo<E, PS>(sb, c);
    const VFrag<E> vB{vslot(tb_of(J - 1)), trb};
#pragma unroll
    for (int k = 0; k < NP; ++k) vf[k] = vB(k);
    pv<E, NP>(sb, vB, vf, kf, vB, [](int) {});
  }
  mfma_drain();
  if (CAUSAL) {
    // Merge the two partial states of Y's rows (A: second key range, B: first).
    const float mf = fmaxf(sa.m, sb.m);
    const float ca = __builtin_amdgcn_exp2f(sa.m - mf);
    const float cb = __builtin_amdgcn_exp2f(sb.m - mf);
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) sb.o[dt][i] = sa.o[dt][i] * ca + sb.o[dt][i] * cb;
    store_stream(p, sb.o, mf, sa.lh * ca + sb.lh * cb, b, h, qiY, qiY < p.R, hh);
  } else {
    store_stream(p, sa.o, sa.m, sa.lh, b, h, qiX, qiX < p.R, hh);
    store_stream(p, sb.o, sb.m, sb.lh, b, h, qiY, qiY < p.R, hh);
  }
}

}  // namespace fwd3

// hipErrorNotSupported when the configuration is not covered (the caller falls back).
hipError_t fwd3_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream) {
  if (DP != 128 || p.mask.window) return hipErrorNotSupported;
  // Opt-in until it beats the v2 kernels (MFA_FWD3=1).
  const char* e3 = getenv("MFA_FWD3");
  if (!e3 || e3[0] != '1') return hipErrorNotSupported;
  FwdParams q = p;
  const int nb128 = (p.R + 127) / 128;
  q.nblk = p.mask.causal ? (nb128 + 1) / 2 : (p.R + 255) / 256;
  const dim3 grid(q.nblk * p.B * p.H), block(256);
  static const int tune = getenv("MFA_V3_TUNE") ? atoi(getenv("MFA_V3_TUNE")) : 0;
#define MFA_F3T(EE, CA, T)                                                     \
  {                                                                            \
    return launch(fwd3::mfa_fwd3_kernel<EE, CA, T>, grid, block, fwd3::LDS_BYTES, \
                  stream, q);                                    \
  }
#define MFA_F3(EE, CA)                                                         \
  {                                                                            \
    if (tune == 1) MFA_F3T(EE, CA, 1)                                          \
    if (tune == 2) MFA_F3T(EE, CA, 2)                                          \
    if (tune == 3) MFA_F3T(EE, CA, 3)                                          \
    MFA_F3T(EE, CA, 0)                                                         \
  }
  if (elem == P_FP16) {
    if (p.mask.causal) MFA_F3(F16, true) else MFA_F3(F16, false)
  }
  if (elem == P_BF16) {
    if (p.mask.causal) MFA_F3(BF16, true) else MFA_F3(BF16, false)
  }
#undef MFA_F3
#undef MFA_F3T
  return hipErrorNotSupported;
}

}  // namespace mfa
