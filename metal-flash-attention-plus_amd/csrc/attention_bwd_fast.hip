// attention_bwd_fast.hip — the two phases of the reference's 7-GEMM backward, tuned for the
// common case on gfx950: fp16/bf16 Q/K/V/dO with 16-byte aligned contiguous rows, D % 8 == 0,
// D <= DP ∈ {64, 128, 256}, no mask or causal / sliding-window masks whose fully masked tiles
// may be skipped.  Same algorithm and numerics contract as attention_bwd.h
// (AttentionKernel+Source.swift:418-511, Softmax.swift:31-236 / :795-804); everything else goes
// to that generic kernel.  Additive masks and sparse ranges run a separate instantiation
// (MSK = true) that applies every mask element by element on every tile, skips nothing unless
// skip_ok, and takes the exact-product path for rows at the mask level (fully masked rows),
// as the generic kernel does; the unmasked instantiations are untouched by it.
//
// Structure (both phases): 4 waves, one per SIMD (up to 512 registers per lane), 32 rows per
// wave held in registers for the whole kernel; the traversed operand pair streams through a
// double-buffered LDS ring filled by LDS-DMA (buffer_load ... lds, no staging registers), one
// barrier per tile.  Fragment reads are issued a few MFMAs ahead of their use and the order is
// pinned with sched_barrier (left alone, hipcc issues each read right before its MFMA).  With
// one wave per SIMD nothing else hides the softmax, so its VALU work is threaded between the
// MFMAs of the next product that does not depend on it (exp under dP, dS under dV or dQ).
//
//   bwd_q  (3 GEMMs): S^T = K·Q^T, dP^T = V·dO^T (query on the lane), P^T = exp2(S^T·c − L),
//                     dS^T = P^T∘(dP^T·scale − D), dQ^T += K^T·dS^T.  Writes D.
//   bwd_kv (4 GEMMs): S = Q·K^T, dP = dO·V^T (key on the lane), dV^T += dO^T·P,
//                     dK^T += Q^T·dS; sums over every query head of the kv group (GQA).
//
// Rows past the end need no masks: the DMA zero-fills K/V/Q/dO rows past C or R, so their
// products vanish (bwd_q: K^T·dS^T with zero K rows; bwd_kv: L = +inf gives P = dS = 0 for
// query rows past R, and key lanes past C are never stored).  Only the causal / window
// diagonal tiles run the mask code; with skip_ok no row is masked everywhere, so
// exp2(S·c − L) needs no mask-level special case.
#include "mfa_stage.h"
#include "mfa_dispatch.h"
#include "kv_bytes.h"

namespace mfa {

// D = 256 backwardKeyValue schedule: softmax work threaded between the MFMAs (true) or the
// dual-chain schedule with the softmax as one block (false).
constexpr bool kBwdKv256Interleave = true;
// backwardKeyValue: stage the next Q/dO tiles all at once at the top of the step (default)
// or piece by piece between the first chain's MFMAs (development A/B: with the loop's waits
// fixed the upfront issue is faster at every D, e.g. D=256 B4 H32 S4096 4.26 vs 4.53 ms and
// D=128 2.40 vs 2.51 ms; tools/diag/bwd_stamps*).
#ifndef MFA_SPREAD_EVERY
#define MFA_SPREAD_EVERY 2  // one piece per this many MFMAs of the first chain
#endif
#ifndef MFA_SPREAD_MIN_DP
#define MFA_SPREAD_MIN_DP 1024
#endif
template <int DP>
constexpr bool spread_dma() { return DP >= MFA_SPREAD_MIN_DP; }

// Diagnostic builds only: MFA_BWDQ_DMA_AT = 1 / 2 issues backwardQuery's next tile after the
// S / dP chain instead of at the step's top.  Stamped, the later issue looked 20 % faster at
// D = 256, but the stamps themselves had slowed that kernel by 46 %; the library A/B puts all
// three placements within 0.5-1.4 % of each other.
#ifndef MFA_BWDQ_DMA_AT
#define MFA_BWDQ_DMA_AT 0
#endif
#define MFA_BWDQ_ISSUE_AT(at)                                                        \
  do {                                                                               \
    if (MFA_BWDQ_DMA_AT == (at) && !QKV && t + BT < kend) {                          \
      kd.issue(khead, t + BT, kb0 + (cur ^ 1) * TILEB);                              \
      vd.issue(vhead, t + BT, vb0 + (cur ^ 1) * TILEB);                              \
    }                                                                                \
  } while (0)

// Diagnostic build only (tools/diag/bwd_stamps.hip defines MFA_BSTAMPS): per-wave shader-clock
// totals of the backwardKeyValue phases, into a buffer no output is computed from.
#ifdef MFA_BSTAMPS
__device__ unsigned long long g_mfa_bstamps[1 << 18];
#define BST_DECL()                               \
  unsigned long long bst_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}; \
  unsigned long long bst_t = __builtin_amdgcn_s_memtime()
#define BST(slot)                                               \
  do {                                                          \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    bst_acc[slot] += t_ - bst_t;                                \
    bst_t = t_;                                                 \
  } while (0)
#define BST_END()                                                                  \
  do {                                                                             \
    if ((threadIdx.x & 63) == 0)                                                   \
      for (int s_ = 0; s_ < 8; ++s_)                                               \
        g_mfa_bstamps[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + s_] = \
            bst_acc[s_];                                                           \
  } while (0)
// Prologue points (cycles since the kernel's first stamp), in the second half of the buffer.
#define BSTP(slot)                                                                        \
  do {                                                                                    \
    const unsigned long long tp_ = __builtin_amdgcn_s_memtime();                          \
    if ((threadIdx.x & 63) == 0)                                                          \
      g_mfa_bstamps[(1 << 17) + ((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * 8 + \
                    (slot)] = tp_ - bst_t;                                                \
  } while (0)
#else
#define BSTP(slot) do {} while (0)
#define BST_DECL() do {} while (0)
#define BST(slot) do {} while (0)
#define BST_END() do {} while (0)
#endif


// Row fragments of one row (16-bit, contiguous): elements d = 16*s + 8*hh + j.
template <int DP>
__device__ __forceinline__ void load_frags16(i16x8 (&f)[DP / 16], const uint16_t* row, bool valid,
                                             int D, int hh) {
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) {
    const int d0 = 16 * s + 8 * hh;
    f[s] = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (valid && d0 < D) f[s] = *reinterpret_cast<const i16x8*>(row + d0);
  }
}

// Two MFMA chains over the head dimension sharing the register operand index:
//   acc1[j] += A1(rows j*32..) · b1[ds],  acc2[j] += A2(rows j*32..) · b2[ds]
// with A fragments read from LDS row tiles AH instructions ahead of their MFMA.
template <class A, int NJ, class Hook>
__device__ __forceinline__ void dual_rows_chain(const char* t1, const char* t2,
                                                const i16x8* b1, const i16x8* b2,
                                                f32x16 (&acc1)[NJ], f32x16 (&acc2)[NJ],
                                                const int (&rbase)[2], Hook&& hook) {
  constexpr int NM = A::DSTEPS * NJ * 2;
  constexpr int AH = 4;
  i16x8 fr[AH];
  auto rd = [&](int i) {
    const int pair = i >> 1, which = i & 1;
    const int ds = pair / NJ, j = pair % NJ;
    return A::read_row_a(which ? t2 : t1, rbase, j, ds);
  };
#pragma unroll
  for (int i = 0; i < AH; ++i) fr[i] = rd(i);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int pair = i >> 1, which = i & 1;
    const int ds = pair / NJ, j = pair % NJ;
    if (which)
      acc2[j] = A::mma(fr[i % AH], b2[ds], acc2[j]);
    else
      acc1[j] = A::mma(fr[i % AH], b1[ds], acc1[j]);
    if (i + AH < NM) fr[i % AH] = rd(i + AH);
    hook(i);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// acc[j] += A(rows j*32.. of an LDS row tile, k-step ds) · b[ds] over all (ds, j), fragment
// reads AH MFMAs ahead, order pinned; after MFMA i the hook runs VALU slice i, so work that
// does not feed this chain (the previous product's softmax) issues between its MFMAs.
template <class A, int NJ, bool ZERO = false, class Hook>
__device__ __forceinline__ void rows_chain(const char* tile, const i16x8* b, f32x16 (&acc)[NJ],
                                           const int (&rbase)[2], Hook&& hook) {
  constexpr int NM = A::DSTEPS * NJ;
  constexpr int AH = A::DSTEPS >= 16 ? 3 : 4;  // D=256 runs at the 512-register limit
  i16x8 fr[AH];
#pragma unroll
  for (int i = 0; i < AH; ++i) fr[i] = A::read_row_a(tile, rbase, i % NJ, i / NJ);
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int ds = i / NJ, j = i % NJ;
    acc[j] = A::mma(fr[i % AH], b[ds], (ZERO && ds == 0) ? zero16() : acc[j]);
    if (i + AH < NM) fr[i % AH] = A::read_row_a(tile, rbase, (i + AH) % NJ, (i + AH) / NJ);
    hook(i);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// acc[dt] += A^T(transposed reads of an LDS row tile) · b[jk] over (jk, dt), jk = 32-row
// sub-tile x k-step; hook(i) after MFMA i as above.
template <class A, int NJ, int ND, class Hook>
__device__ __forceinline__ void tr_chain(const char* tile, const int (&trb)[2], const i16x8* b,
                                         f32x16 (&acc)[ND], Hook&& hook) {
  constexpr int NM = NJ * 2 * ND;
  constexpr int AH = 3;
  i16x8 fr[AH];
#pragma unroll
  for (int i = 0; i < AH; ++i) {
    const int jk = i / ND, dt = i % ND;
    fr[i] = A::read_tr_a(tile, trb, (jk >> 1) * 32, jk & 1, dt * 32);
  }
#pragma unroll
  for (int i = 0; i < NM; ++i) {
    const int jk = i / ND, dt = i % ND;
    acc[dt] = A::mma(fr[i % AH], b[jk], acc[dt]);
    if (i + AH < NM) {
      const int jn = (i + AH) / ND, dn = (i + AH) % ND;
      fr[i % AH] = A::read_tr_a(tile, trb, (jn >> 1) * 32, jn & 1, dn * 32);
    }
    hook(i);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------------------------------
// backwardQuery.  Grid: nblk x B x H, heaviest causal blocks first.  BT keys per tile.
// KVQ: K/V storage — SRC_SAME (16-bit, LDS-DMA into the ring), or SRC_I8 / SRC_I4 per-tensor
// quantised: the stored bytes of tile t + 2 move by LDS-DMA into a byte ring (kv_bytes.h) at
// the top of step t, and tile t + 1's bytes are widened into its 16-bit slot between the S
// chain's MFMAs (which carry no other VALU work), so the MFMA operands are those of the
// dequantisation pass + 16-bit kernel path, without the pass or its scratch copy.
template <class E, int DP, int BT, bool MSK = false, int KVQ = SRC_SAME>
__global__ void __launch_bounds__(256, 1) mfa_bwd_q_fast_kernel(BwdParams p) {
  using A = Arith16<E, DP>;
  constexpr int NT = 256, BQ = 128, NJ = BT / 32, DS = DP / 16, ND = DP / 32;
  constexpr int TILEB = BT * DP * 2;
  constexpr bool QKV = KVQ != SRC_SAME;
  static_assert(!(QKV && MSK), "quantised K/V: no element-wise mask instantiation");
  using KB = KvBytes<E, DP, BT, QKV ? KVQ : SRC_I8, NT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;
  char* const rawk = smem + 4 * TILEB;       // QKV: byte ring, K slots 0, 1 then V slots 0, 1
  char* const rawv = rawk + 2 * KB::SLOT;

  const int tid = threadIdx.x;
  BST_DECL();  // (diagnostic builds: the backwardQuery phases, tools/diag/bwd_stamps q)
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  int bh, blk;
  xcd_unit_block(blockIdx.x, p.B * p.H, p.nblk, &bh, &blk);
  const int rb = p.nblk - 1 - blk;  // heaviest causal blocks first
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;
  const int64_t row = (int64_t)(b * p.H + h) * p.R + qi;

  i16x8 qf[DS], dof[DS];
  {
    const int qq = qvalid ? qi : 0;
    load_frags16<DP>(qf, (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh +
                             (int64_t)qq * p.q.ss, qvalid, p.D, hh);
    load_frags16<DP>(dof, (const uint16_t*)p.dO_op.ptr + (int64_t)b * p.dO_op.sb +
                              (int64_t)h * p.dO_op.sh + (int64_t)qq * p.dO_op.ss,
                     qvalid, p.D, hh);
  }
  BSTP(0);

  // K/V ring: issue the first tile before the D prologue so its latency hides behind it.
  int kend = p.C;
  if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
  int kbeg = 0;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
    kbeg = lo > 0 ? (int)(lo / BT) * BT : 0;
  }
  // MSK: ranges, causal and window each leave an interval of keys, so a row's unmasked keys are
  // one interval [elo, ehi); a row with none (elo >= ehi, stored as [C, 0)) is masked
  // everywhere and sits at the mask level, where every key counts (uniform P).  Unless the block
  // holds such a row, its key tiles run over the union of its rows' intervals only (the others
  // give P = 0 exactly); tiles inside every row's interval need no per-element mask.
  int elo = 0, ehi = p.C, tin_lo = 0, tin_hi = p.C;
  if constexpr (MSK) {
    int64_t lo = 0, hi = p.C;
    if (p.mask.ranges && qvalid) {
      const uint32_t* rp = p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + qi);
      lo = rp[0];
      hi = min((int64_t)rp[1], (int64_t)p.C);
    }
    if (p.mask.causal) hi = min(hi, (int64_t)qi + 1);
    if (p.mask.window) lo = max(lo, (int64_t)qi - (int64_t)p.mask.window_size);
    const bool empty = qvalid && lo >= hi;
    elo = empty ? p.C : (int)lo;
    ehi = empty ? 0 : (int)hi;
    // Block reductions over valid rows: union [umn, umx) of the non-empty rows, intersection
    // [tin_lo, tin_hi) of all rows, and whether any row is empty.
    int umn = qvalid && !empty ? elo : p.C, umx = qvalid && !empty ? ehi : 0;
    int imx = qvalid ? elo : 0, imn = qvalid ? ehi : p.C;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      umn = min(umn, __shfl_xor(umn, o));
      umx = max(umx, __shfl_xor(umx, o));
      imx = max(imx, __shfl_xor(imx, o));
      imn = min(imn, __shfl_xor(imn, o));
    }
    const bool wempty = __ballot(empty) != 0;
    int* red = reinterpret_cast<int*>(smem + 4 * TILEB);
    if (lane == 0) {
      red[wave * 5] = umn; red[wave * 5 + 1] = umx; red[wave * 5 + 2] = imx;
      red[wave * 5 + 3] = imn; red[wave * 5 + 4] = wempty;
    }
    __syncthreads();
    bool any_empty = false;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      umn = min(umn, red[w * 5]); umx = max(umx, red[w * 5 + 1]);
      imx = max(imx, red[w * 5 + 2]); imn = min(imn, red[w * 5 + 3]);
      any_empty = any_empty || red[w * 5 + 4];
    }
    if (!any_empty) {
      kbeg = max(kbeg, (umn / BT) * BT);
      kend = min(kend, umx);
    }
    tin_lo = imx;
    tin_hi = imn;
  }
  DmaA<DP, BT, NT> kd, vd;
  KB kq, vq;
  // Element offsets -> byte offsets: 16-bit x 2, INT8 x 1, INT4 / 2.
  auto head_bytes = [&](const Operand& op) {
    const int64_t e = (int64_t)b * op.sb + (int64_t)kvh * op.sh;
    return (const char*)op.ptr + (QKV ? e >> KB::SH : e * 2);
  };
  const char* khead = head_bytes(p.k);
  const char* vhead = head_bytes(p.v);
  const int kss = QKV ? (int)(p.k.ss >> KB::SH) : 0, vss = QKV ? (int)(p.v.ss >> KB::SH) : 0;
  const int kbytes = QKV ? (int)((int64_t)(p.C - 1) * kss + (p.D >> KB::SH)) : 0;
  const int vbytes = QKV ? (int)((int64_t)(p.C - 1) * vss + (p.D >> KB::SH)) : 0;
  const float zk = (float)p.k.zp, zv = (float)p.v.zp;
  if constexpr (QKV) {
    kq.init(tid, p.D, kss);
    vq.init(tid, p.D, vss);
    if (kbeg < kend) {
      kq.dma(khead, kss, kbytes, kbeg, rawk);
      vq.dma(vhead, vss, vbytes, kbeg, rawv);
      if (kbeg + BT < kend) {
        kq.dma(khead, kss, kbytes, kbeg + BT, rawk + KB::SLOT);
        vq.dma(vhead, vss, vbytes, kbeg + BT, rawv + KB::SLOT);
      }
    }
  } else {
    kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
    vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
    if (kbeg < kend) {
      kd.issue(khead, kbeg, kb0);
      vd.issue(vhead, kbeg, vb0);
    }
  }

  BSTP(1);
  // D = scale · Σ_d dO∘O (computeD, Softmax.swift:31-236): dO as stored (16-bit), O fp32.
  float dsum = 0.f;
  if (qvalid) {
    const float* orow = p.o + row * p.D;
#pragma unroll
    for (int s = 0; s < DS; ++s) {
      const int d0 = 16 * s + 8 * hh;
      if (d0 < p.D) {
        const float4 oa = *reinterpret_cast<const float4*>(orow + d0);
        const float4 ob = *reinterpret_cast<const float4*>(orow + d0 + 4);
        const float ov[8] = {oa.x, oa.y, oa.z, oa.w, ob.x, ob.y, ob.z, ob.w};
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum += E::to_f32((uint16_t)dof[s][j]) * ov[j];
      }
    }
  }
  dsum = cross_half_sum(dsum);
  BSTP(2);
  const float Drow = p.dscale * dsum;
  float Lrow = __builtin_inff();
  if (qvalid) {
    Lrow = p.l_f16 ? f16_to_f32(reinterpret_cast<const uint16_t*>(p.l)[row])
                   : reinterpret_cast<const float*>(p.l)[row];
    if (hh == 0) {
      if (p.d_bf16)  // BF16 memory form = upper half of the FP32 bits (Caching.swift:413-421)
        reinterpret_cast<uint16_t*>(p.dD)[row] = (uint16_t)(__builtin_bit_cast(uint32_t, Drow) >> 16);
      else
        reinterpret_cast<float*>(p.dD)[row] = Drow;
    }
  }
  const float c = p.c_log2, sc = p.scale;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;
  // MSK: a row at the mask level (every key masked) takes the rounded product S·c before
  // subtracting L, as the generic kernel does (attention_bwd.h).
  // MSK takes the rounded product for every row (two VALU, no per-lane select): exact for
  // rows at the mask level, within rounding of the fused form elsewhere.
  auto pexp = [&](float x) {
    if constexpr (MSK)
      return __builtin_amdgcn_exp2f(mul_rn(x, c) - Lrow);
    else
      return __builtin_amdgcn_exp2f(__builtin_fmaf(x, c, -Lrow));
  };

  f32x16 dq[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dq[dt] = zero16();

  BSTP(3);
  wait_vm();
  BSTP(4);
  if constexpr (QKV) {
    // The first tile's bytes are in (the second's may be too): widen the first.
    __asm__ __volatile__("" ::: "memory");
    if (kbeg < kend) {
#pragma unroll
      for (int m = 0; m < KB::NPIECE; ++m) {
        kq.widen(kb0, kq.read(rawk, m), zk, m, p.C - kbeg);
        vq.widen(vb0, vq.read(rawv, m), zv, m, p.C - kbeg);
      }
    }
  }
  __syncthreads();
  BSTP(5);
  BST(7);
  int cur = 0;
  for (int t = kbeg; t < kend; t += BT) {
    if constexpr (QKV) {
      // Tile t + 2's bytes into the byte slot tile t's left (widened during the last step).
      if (t + 2 * BT < kend) {
        kq.dma(khead, kss, kbytes, t + 2 * BT, rawk + cur * KB::SLOT);
        vq.dma(vhead, vss, vbytes, t + 2 * BT, rawv + cur * KB::SLOT);
      }
    } else if (MFA_BWDQ_DMA_AT == 0 && t + BT < kend) {
      kd.issue(khead, t + BT, kb0 + (cur ^ 1) * TILEB);
      vd.issue(vhead, t + BT, vb0 + (cur ^ 1) * TILEB);
    }
    const char* kt = kb0 + cur * TILEB;
    const char* vt = vb0 + cur * TILEB;
    BST(0);
    // S^T = K·Q^T; masks; dP^T = V·dO^T with P^T = exp2(S^T·c − L) computed between its
    // MFMAs; dQ^T += K^T·dS^T with each k-step's dS^T = P^T∘(dP^T·scale − D) computed under
    // the previous k-step's MFMAs.
    f32x16 s[NJ], dp[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { s[j] = zero16(); dp[j] = zero16(); }
    // MSK: this tile's additive-mask values, issued before the S chain so it hides them;
    // element (j, i) is key t + 32j + 8(i>>2) + 4hh + (i&3) of this lane's row.
    float am[MSK ? NJ : 1][16];
    if constexpr (MSK) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) am[j][i] = 0.f;
      if (p.mask.amask) {  // wave-uniform: no per-element branch without an additive mask
        const float* arow = p.mask.amask + row * p.C;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = t + 32 * j + 8 * (i >> 2) + 4 * hh + (i & 3);
            if (qvalid && key < p.C) am[j][i] = arow[key];
          }
      }
    }
    if constexpr (QKV) {
      // Tile t + 1 widened piece by piece under the S chain, which carries no other VALU work:
      // 2·NPIECE pieces (K and V), one after every EVERY-th MFMA, each piece's bytes read into
      // registers before the chain so no widening waits on its LDS read.
      constexpr int NM = DS * NJ, NPW = 2 * KB::NPIECE, EVERY = NM / NPW;
      static_assert(NM % NPW == 0 && EVERY >= 1, "widening slots");
      const bool wnext = t + BT < kend;
      const int nrows = p.C - (t + BT);
      const char* rk = rawk + (cur ^ 1) * KB::SLOT;
      const char* rv = rawv + (cur ^ 1) * KB::SLOT;
      char* const kn = kb0 + (cur ^ 1) * TILEB;
      char* const vn = vb0 + (cur ^ 1) * TILEB;
      // Piece w: K piece w / 2 (w even) or V piece w / 2 (w odd).
      uint4 raws[NPW];
#pragma unroll
      for (int w = 0; w < NPW; ++w)
        raws[w] = wnext ? ((w & 1) ? vq.read(rv, w >> 1) : kq.read(rk, w >> 1))
                        : make_uint4(0u, 0u, 0u, 0u);
      rows_chain<A, NJ>(kt, qf, s, rbase, [&](int i) {
        if (i % EVERY == EVERY - 1 && wnext) {
          const int w = i / EVERY;
          if (w & 1)
            vq.widen(vn, raws[w], zv, w >> 1, nrows);
          else
            kq.widen(kn, raws[w], zk, w >> 1, nrows);
        }
      });
    } else {
      rows_chain<A, NJ>(kt, qf, s, rbase, [](int) {});
    }
    MFA_BWDQ_ISSUE_AT(1);
    if constexpr (MSK) {
      if (t >= tin_lo && min(t + BT, p.C) <= tin_hi) {
        if (p.mask.amask) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) s[j][i] += am[j][i];
        }
      } else {
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int key = t + 32 * j + 8 * (i >> 2) + 4 * hh + (i & 3);
            s[j][i] = (key < elo || key >= ehi) ? kMaskValue : s[j][i] + am[j][i];
          }
      }
    }
    const bool diag = !MSK && ((p.mask.causal && t + BT - 1 > q0) || p.mask.window);
    if (diag) {
      MFA_KEEP_BRANCH();
      {
        const int base = t + 4 * hh;
        const int hi = p.mask.causal ? qi - base : 0x3fffffff;
        const int lo = p.mask.window ? qi - wsz - base : -0x40000000;
        mask_outside<NJ>(s, lo, hi, kMaskValue);
      }
    }
    BST(1);
    {
      constexpr int EPM = 16 / DS;  // P elements per dP MFMA (NJ*16 over DS*NJ MFMAs)
      rows_chain<A, NJ>(vt, dof, dp, rbase, [&](int i) {
#pragma unroll
        for (int e = 0; e < EPM; ++e) {
          const int idx = i * EPM + e, jj = idx >> 4, ii = idx & 15;
          s[jj][ii] = pexp(s[jj][ii]);
        }
      });
    }
    MFA_BWDQ_ISSUE_AT(2);
    BST(2);
    {
      // dS^T of k-step jk = registers 8*(jk&1)..+7 of sub-tile jk>>1, packed as the B operand.
      i16x8 sb[NJ * 2];
      auto ds_step = [&](int jk) {
        const int j = jk >> 1, base = 8 * (jk & 1);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          dp[j][base + e] = s[j][base + e] * __builtin_fmaf(dp[j][base + e], sc, -Drow);
        sb[jk] = A::pack(dp[j], jk & 1);
      };
      ds_step(0);
      constexpr int EPM = 8 / ND;  // dS elements per dQ MFMA: next k-step's 8 over ND MFMAs
      tr_chain<A, NJ, ND>(kt, trb, sb, dq, [&](int i) {
        const int jk = i / ND, r = i % ND;
        if (jk + 1 < NJ * 2) {
          const int jn = jk + 1, j = jn >> 1, base = 8 * (jn & 1);
#pragma unroll
          for (int e = 0; e < EPM; ++e) {
            const int el = base + r * EPM + e;
            dp[j][el] = s[j][el] * __builtin_fmaf(dp[j][el], sc, -Drow);
          }
          if (r == ND - 1) sb[jn] = A::pack(dp[j], jn & 1);
        }
      });
    }
    BST(3);
    wait_vm();
    BST(4);
    __syncthreads();
    BST(5);
    cur ^= 1;
  }

  if (qvalid) {
    float* out = p.dq + row * p.D;
    const float mul = p.dq_mul;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (d < p.D)
          *reinterpret_cast<float4*>(out + d) =
              make_float4(dq[dt][4 * g] * mul, dq[dt][4 * g + 1] * mul, dq[dt][4 * g + 2] * mul,
                          dq[dt][4 * g + 3] * mul);
      }
  }
  BST(6);
  BST_END();
}

// ---------------------------------------------------------------------------------------
// backwardKeyValue.  Grid: nblk x B x H_kv (first key blocks carry the most causal query
// tiles).  128 keys per workgroup; BQ query rows per step.
// KVQ: K/V storage — SRC_SAME (16-bit), or SRC_I8 / SRC_I4 per-tensor quantised (a separate
// instantiation, so the 16-bit kernel's register allocation is untouched).
template <class E, int DP, int BQ, int KVQ = SRC_SAME, bool MSK = false>
__global__ void __launch_bounds__(256, 1) mfa_bwd_kv_fast_kernel(BwdParams p) {
  using A = Arith16<E, DP>;
  constexpr int NT = 256, BK = 128, NJ = BQ / 32, DS = DP / 16, ND = DP / 32;
  constexpr int TILEB = BQ * DP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const qb0 = smem;
  char* const ob0 = smem + 2 * TILEB;
  float* const lb0 = reinterpret_cast<float*>(smem + 4 * TILEB);  // [2][BQ] L, then [2][BQ] D
  float* const db0 = lb0 + 2 * BQ;
  // MSK: [2][BQ] unmasked key interval per row, [2][BQ][BK] additive mask, [2] step flags.
  int2* const rg0 = reinterpret_cast<int2*>(db0 + 2 * BQ);
  float* const am0 = reinterpret_cast<float*>(rg0 + 2 * BQ);
  int* const fl0 = reinterpret_cast<int*>(am0 + 2 * BQ * 128);
  // MSK without an additive mask: the mask tile region holds every row's interval (rgall, up
  // to RCAP rows) and every query tile's step flags (flall), computed once in the pre-pass, so
  // the steps neither load ranges nor wait on wave 0 to convert them.
  constexpr int AMB = 2 * BQ * 128 * 4, RCAP = (AMB - 512) / 8;
  int2* const rgall = reinterpret_cast<int2*>(am0);
  uint8_t* const flall = reinterpret_cast<uint8_t*>(rgall + RCAP);

  const int tid = threadIdx.x;
  BST_DECL();  // (diagnostic builds: slot 7 = everything before the step loop)
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  int bh, kb;
  xcd_unit_block(blockIdx.x, p.B * p.Hkv, p.nblk, &bh, &kb);
  const int b = bh / p.Hkv, kvh = bh % p.Hkv;
  const int k0 = kb * BK;
  const int ki = k0 + wave * 32 + l32;
  const bool kvalid = ki < p.C;

  // The key block's K and V rows (MFMA A operands for the whole kernel).  Under MSK they are
  // issued right after the pre-pass's range loads, so those do not wait behind them (vmcnt
  // counts in issue order) while their latencies still overlap.
  i16x8 kf[DS], vf[DS];
  auto load_kv = [&]() __attribute__((always_inline)) {
    const int kk = kvalid ? ki : 0;
    if constexpr (KVQ != SRC_SAME) {
      // Quantised per-tensor K/V (QuantizedAttention.backwardKeyValue): the key block's rows
      // are read once per workgroup, so they are widened here, in registers, to exactly the
      // operands the dequantisation pass would have written (the integers q - zp; the scales
      // stay folded) — no pass, no dense copy, bit-identical results.
      auto qload = [&](i16x8 (&f)[DS], const Operand& op) {
        const int64_t rowoff = (int64_t)b * op.sb + (int64_t)kvh * op.sh + (int64_t)kk * op.ss;
        const float zp = (float)op.zp;
#pragma unroll
        for (int sidx = 0; sidx < DS; ++sidx) {
          const int d0 = 16 * sidx + 8 * hh;
          uint4 v = make_uint4(0u, 0u, 0u, 0u);
          if (kvalid && d0 < p.D) v = dequant_fast<E, KVQ>(load_qchunk<KVQ>(op, rowoff, d0, p.D), zp);
          f[sidx] = __builtin_bit_cast(i16x8, v);
        }
      };
      qload(kf, p.k);
      qload(vf, p.v);
    } else {
      load_frags16<DP>(kf, (const uint16_t*)p.k.ptr + (int64_t)b * p.k.sb +
                               (int64_t)kvh * p.k.sh + (int64_t)kk * p.k.ss, kvalid, p.D, hh);
      load_frags16<DP>(vf, (const uint16_t*)p.v.ptr + (int64_t)b * p.v.sb +
                               (int64_t)kvh * p.v.sh + (int64_t)kk * p.v.ss, kvalid, p.D, hh);
    }
  };
  if constexpr (!MSK) load_kv();
  int qbeg = 0, qend = p.R;
  if (p.mask.causal && p.mask.skip_ok) qbeg = (k0 / BQ) * BQ;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t hi = (int64_t)k0 + BK + (int64_t)p.mask.window_size;
    if (hi < qend) qend = (int)hi;
  }
  const bool pre = MSK && !p.mask.amask && p.R <= RCAP;
  if constexpr (MSK) {
    // The rows that see this key block (their unmasked interval meets [k0, k0 + BK)) or sit at
    // the mask level (no unmasked key: they see every key): the query tiles run from the first
    // to the last of them only (the intervals are the same for every head of the kv group).
    // A pre-pass over the rows' intervals, one row per thread per 256.
    // (32-bit: C and R are below 2^31 and range ends are clamped to C; 16 rows per thread in
    // flight at once — at R = 4096 every thread's rows take one load latency.)
    int rmin = p.R, rmax = -1;
    const uint2* rrow = reinterpret_cast<const uint2*>(p.mask.ranges) + (int64_t)(b * p.Hkv + kvh) * p.R;
    const int ws = (int)min(p.mask.window_size, 0x7fffffffu);
    constexpr int PRE_N = 16;  // rows per thread whose loads are in flight together
    // One chunk of PRE_N rows per thread.  D <= 128: the key block's K/V rows are loaded after
    // the pre-pass, under the reduction, the step flags and the first tiles.  Issued between the
    // range loads and their use (the previous form), they were waited for there: every load sits
    // in an exec-masked branch, so hipcc cannot count them and the first use of a range waited
    // with vmcnt(0) for the whole key block from HBM (13.3k of the prologue's 19.7k cycles per
    // wave at band 8, tools/diag/bwd_stamps prologue points).  D = 256, at the register limit,
    // keeps the previous form (moved, it spills).
    auto pre_chunk = [&](const uint2 (&rr)[PRE_N], int q0) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < PRE_N; ++j) {
        const int q = q0 + j * NT;
        if (q < p.R) {
          int lo = (int)min(rr[j].x, 0x7fffffffu);
          int hi = (int)min(rr[j].y, (uint32_t)p.C);
          if (p.mask.causal) hi = min(hi, q + 1);
          if (p.mask.window) lo = max(lo, q - ws);
          if (lo >= hi || (lo < k0 + BK && hi > k0)) {
            rmin = min(rmin, q);
            rmax = max(rmax, q);
          }
          if (pre) rgall[q] = lo >= hi ? make_int2(p.C, 0) : make_int2(lo, hi);
        }
      }
    };
    auto pre_load = [&](uint2 (&rr)[PRE_N], int q0) __attribute__((always_inline)) {
#pragma unroll
      for (int j = 0; j < PRE_N; ++j) {
        const int q = q0 + j * NT;
        rr[j] = make_uint2(0u, 0x7fffffffu);
        if (p.mask.ranges && q < p.R) rr[j] = rrow[q];
      }
    };
    if constexpr (DP <= 128) {
      uint2 rr[PRE_N];
      for (int q0 = tid; q0 < p.R; q0 += PRE_N * NT) {
        pre_load(rr, q0);
        if (q0 == tid) BSTP(5);
        pre_chunk(rr, q0);
        if (q0 == tid) BSTP(6);
      }
      load_kv();
    } else {
      int q0 = tid;
      do {
        uint2 rr[PRE_N];
#pragma unroll
        for (int j = 0; j < PRE_N; ++j) {
          const int q = q0 + j * NT;
          rr[j] = make_uint2(0u, 0x7fffffffu);
          if (p.mask.ranges && q < p.R) rr[j] = rrow[q];
        }
        if (q0 == tid) load_kv();
#pragma unroll
        for (int j = 0; j < PRE_N; ++j) {
          const int q = q0 + j * NT;
          if (q < p.R) {
            int lo = (int)min(rr[j].x, 0x7fffffffu);
            int hi = (int)min(rr[j].y, (uint32_t)p.C);
            if (p.mask.causal) hi = min(hi, q + 1);
            if (p.mask.window) lo = max(lo, q - ws);
            if (lo >= hi || (lo < k0 + BK && hi > k0)) {
              rmin = min(rmin, q);
              rmax = max(rmax, q);
            }
            if (pre) rgall[q] = lo >= hi ? make_int2(p.C, 0) : make_int2(lo, hi);
          }
        }
        q0 += PRE_N * NT;
      } while (q0 < p.R);
    }
    BSTP(0);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      rmin = min(rmin, __shfl_xor(rmin, o));
      rmax = max(rmax, __shfl_xor(rmax, o));
    }
    int* red = reinterpret_cast<int*>(smem);  // before any tile lands in LDS
    if (lane == 0) { red[wave * 2] = rmin; red[wave * 2 + 1] = rmax; }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NT / 64; ++w) {
      rmin = min(rmin, red[w * 2]);
      rmax = max(rmax, red[w * 2 + 1]);
    }
    __syncthreads();
    BSTP(1);
    qbeg = max(qbeg, (rmin / BQ) * BQ);
    qend = min(qend, rmax + 1);
    if (pre) {
      // Step flags of the query tiles [qbeg, qend), one wave per tile (lane = row); the barrier
      // before the loop orders them for every wave.
      for (int i = qbeg / BQ + wave; i * BQ < qend; i += NT / 64) {
        const int q = i * BQ + lane;
        const bool v = lane < BQ && q < p.R;
        const int2 e = v ? rgall[q] : make_int2(0, 0);
        const bool empty = e.x >= e.y;
        const bool skip = !v || (!empty && (e.y <= k0 || e.x >= k0 + BK));
        const bool full = !v || (!empty && e.x <= k0 && e.y >= min(k0 + BK, p.C));
        const int f = (__ballot(skip) == ~0ull ? 1 : 0) | (__ballot(full) == ~0ull ? 2 : 0);
        if (lane == 0) flall[i] = (uint8_t)f;
      }
    }
  }
  BSTP(2);
  const int ntile = qbeg < qend ? (qend - qbeg + BQ - 1) / BQ : 0;
  const int ngroup = (p.H - kvh + p.Hkv - 1) / p.Hkv;  // query heads h = kvh + g*Hkv
  const int nsteps = ntile * ngroup;

  DmaA<DP, BQ, NT> qd, od;
  qd.init((int)p.q.ss * 2, p.R, p.D * 2, tid);
  od.init((int)p.dO_op.ss * 2, p.R, p.D * 2, tid);
  auto qhead = [&](int h) {
    return (const char*)p.q.ptr + ((int64_t)b * p.q.sb + (int64_t)h * p.q.sh) * 2;
  };
  auto ohead = [&](int h) {
    return (const char*)p.dO_op.ptr + ((int64_t)b * p.dO_op.sb + (int64_t)h * p.dO_op.sh) * 2;
  };
  // L and D of the step's BQ query rows: one value per thread of the first BQ threads, staged
  // through registers into LDS (converted to fp32); L = +inf past R makes P = dS = 0 there.
  // The loads leave raw bits in registers and are converted only at the step's end, so their
  // latency hides under the step (a conversion right after the load waits for it).
  uint32_t lraw = 0u, draw = 0u;
  uint2 rraw = make_uint2(0u, 0xffffffffu);
  bool ldv = false;
  auto ld_load = [&](int h, int t) {
    if (tid < BQ) {
      const int q = t + tid;
      ldv = q < p.R;
      const int64_t r = (int64_t)(b * p.H + h) * p.R + (ldv ? q : 0);
      lraw = p.l_f16 ? (uint32_t)reinterpret_cast<const uint16_t*>(p.l)[r]
                     : reinterpret_cast<const uint32_t*>(p.l)[r];
      draw = p.d_bf16 ? (uint32_t)reinterpret_cast<const uint16_t*>(p.dD)[r]
                      : reinterpret_cast<const uint32_t*>(p.dD)[r];
      if (MSK && p.mask.ranges && !pre)  // ranges are per kv head: [B, H_kv, R, 2]
        rraw = *reinterpret_cast<const uint2*>(
            p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + (ldv ? q : 0)));
    }
  };
  // MSK: ranges, causal and window each leave an interval of keys, so row q's unmasked keys
  // are one interval [elo, ehi), stored per row; a row with none ([C, 0)) is masked everywhere
  // and sits at the mask level, where every key counts (uniform P).  Step flags (wave 0 holds
  // the BQ rows): 1 = no row sees this key block and none is empty (P = dS = 0 exactly: the
  // step is skipped), 2 = every row sees the whole block (no per-element mask).
  auto ld_store = [&](int buf, int tq) {
    if (tid < BQ) {
      const float lv = p.l_f16 ? f16_to_f32((uint16_t)lraw) : __builtin_bit_cast(float, lraw);
      const float dv = p.d_bf16 ? bf16_to_f32((uint16_t)draw) : __builtin_bit_cast(float, draw);
      lb0[buf * BQ + tid] = ldv ? lv : __builtin_inff();
      db0[buf * BQ + tid] = ldv ? dv : 0.f;
      if (MSK && !pre) {
        // 32-bit: C and R are below 2^31, and range ends are clamped to C.
        const int q = tq + tid;
        int lo = 0, hi = p.C;
        if (p.mask.ranges) {
          lo = (int)min(rraw.x, 0x7fffffffu);
          hi = (int)min(rraw.y, (uint32_t)p.C);
        }
        if (p.mask.causal) hi = min(hi, q + 1);
        if (p.mask.window)
          lo = max(lo, q - (int)min(p.mask.window_size, 0x7fffffffu));
        const bool empty = lo >= hi;
        const int elo = empty ? p.C : (int)lo, ehi = empty ? 0 : (int)hi;
        rg0[buf * BQ + tid] = make_int2(elo, ehi);
        const bool skip = !ldv || (!empty && (ehi <= k0 || elo >= k0 + BK));
        const bool full = !ldv || (!empty && elo <= k0 && ehi >= min(k0 + BK, p.C));
        const uint64_t act = __ballot(true);
        const int f = (__ballot(skip) == act ? 1 : 0) | (__ballot(full) == act ? 2 : 0);
        if (tid == 0) fl0[buf] = f;
      }
    }
  };

  // MSK: LDS-DMA of a step's additive-mask tile — query rows t..t+BQ of head h, this block's
  // BK keys — row-major into dst (2 rows per 1-KiB piece, lane l at byte 16l: row 2n + l/32,
  // keys k0 + 4(l%32)..+3); rows past R read as zeros.  No staging registers (at D = 256 the
  // kernel is at the register limit).  Needs C % 4 == 0 (16-byte rows; see bwd_fast_eligible).
  auto am_issue = [&](int h, int t, float* dst) {
    if (!p.mask.amask) return;
    constexpr int PPW = BQ / 2 / (NT / 64);
    const char* head = (const char*)(p.mask.amask + (int64_t)(b * p.H + h) * p.R * p.C);
    const int ln = __lane_id();  // recomputed here rather than held across the step
    const int voff = (ln >> 5) * p.C * 4 + k0 * 4 + 16 * (ln & 31);
    const int wv = __builtin_amdgcn_readfirstlane(wave);  // piece indices in scalar registers
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int n = wv + (NT / 64) * i, row = t + 2 * n;
      const int64_t left = (int64_t)(p.R - row) * p.C * 4;
      lds_dma16(head + (int64_t)row * p.C * 4, left <= 0 ? 0 : (int)min(left, (int64_t)0x7fffffff),
                voff, (char*)dst + n * 1024);
    }
  };

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }
  const float c = p.c_log2, sc = p.scale;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;
  // P = exp2(S·c − L).  MSK takes the rounded product first for every row (two VALU, no
  // per-lane select, as the query phase does): exact for rows at the mask level, within
  // rounding of the fused form elsewhere.
  auto pexp = [&](float x, float l) {
    if constexpr (MSK)
      return __builtin_amdgcn_exp2f(mul_rn(x, c) - l);
    else
      return __builtin_amdgcn_exp2f(__builtin_fmaf(x, c, -l));
  };

  if (nsteps > 0) {
    qd.issue(qhead(kvh), qbeg, qb0);
    od.issue(ohead(kvh), qbeg, ob0);
    if (MSK) am_issue(kvh, qbeg, am0);
    ld_load(kvh, qbeg);
    BSTP(3);
    wait_vm();
    BSTP(4);
    ld_store(0, qbeg);
  }
  // Unconditionally drained before the loop: otherwise the K/V fragment loads count as
  // possibly pending at the loop header and hipcc puts a vmcnt(0) before their first use in
  // every step (which then also waits for the step's own prefetch).
  wait_vm();
  __syncthreads();
  BST(7);

  int cur = 0;
  // Step s covers query tile t of query head h = kvh + g·Hkv (g = s / ntile), walked
  // incrementally: a per-step integer division costs a few hundred cycles of the step.
  const int qlast = qbeg + (ntile - 1) * BQ;
  int t = qbeg, h = kvh;
  for (int step = 0; step < nsteps; ++step) {
    const bool has_next = step + 1 < nsteps;
    const int tn = t < qlast ? t + BQ : qbeg;
    const int hn = t < qlast ? h : h + p.Hkv;
    if (has_next) ld_load(hn, tn);
    // MSK at D = 256 spills a few registers; their reloads wait for every outstanding load
    // (vmcnt(0)), so the next step's tiles are issued after the S/dP chains, where none is left.
#ifndef MFA_BWD_LATE_ALL
#define MFA_BWD_LATE_ALL 0  // diagnostic builds: the unmasked D = 256 key phase issues late too
#endif
    constexpr bool late_dma = (MSK || MFA_BWD_LATE_ALL) && DP >= 256;
    auto issue_next = [&]() {
      if (MSK && has_next) am_issue(hn, tn, am0 + (cur ^ 1) * BQ * BK);
      if (!(spread_dma<DP>() && !MSK) && has_next) {
        qd.issue(qhead(hn), tn, qb0 + (cur ^ 1) * TILEB);
        od.issue(ohead(hn), tn, ob0 + (cur ^ 1) * TILEB);
      }
    };
    if (!late_dma) issue_next();
    BST(0);
    // The next step's Q and dO tiles: one LDS-DMA piece after every other MFMA of the first
    // chain, so each piece's issue cost sits in an MFMA gap.
    auto dma_hook = [&](int i) {
      constexpr int PPW = DmaA<DP, BQ, NT>::PPW;
      constexpr int EVERY = MFA_SPREAD_EVERY;
      if (spread_dma<DP>() && !MSK && (i % EVERY) == 0 && i / EVERY < 2 * PPW && has_next) {
        const int k = i / EVERY;
        if (k < PPW)
          qd.issue_piece(qhead(hn), tn, qb0 + (cur ^ 1) * TILEB, k);
        else
          od.issue_piece(ohead(hn), tn, ob0 + (cur ^ 1) * TILEB, k - PPW);
      }
    };
    const char* qt = qb0 + cur * TILEB;
    const char* ot = ob0 + cur * TILEB;
    const float* lt = lb0 + cur * BQ;
    const float* dtl = db0 + cur * BQ;
    const int2* rgt = pre ? rgall + t : rg0 + cur * BQ;
    const float* amt = am0 + cur * BQ * BK;  // + this lane's key column (at the reads)
    const int flags = MSK ? __builtin_amdgcn_readfirstlane(pre ? (int)flall[t / BQ] : fl0[cur]) : 0;

    f32x16 s[NJ], dp[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { s[j] = zero16(); dp[j] = zero16(); }
    // L and D of accumulator row (j, i) = query j*32 + 8*(i>>2) + 4*hh + (i&3).
    auto lds4 = [&](const float* base, float (&v)[NJ][16]) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const float4 x = *reinterpret_cast<const float4*>(base + j * 32 + 8 * g4 + 4 * hh);
          v[j][4 * g4] = x.x; v[j][4 * g4 + 1] = x.y; v[j][4 * g4 + 2] = x.z; v[j][4 * g4 + 3] = x.w;
        }
    };
    // MSK: bit 16j + i of mbits = accumulator element (j, i) outside its row's interval
    // (query t + 32j + 8(i>>2) + 4hh + (i&3), this lane's key), computed before the S chain
    // from two 16-byte LDS reads per four rows — one wait per step, not one per element.
    uint32_t mbits = 0u;
    auto mask_bits = [&]() {
      const int hl = (DP >= 256 ? __lane_id() : lane) >> 5;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
          const int ql0 = 32 * j + 8 * g4 + 4 * hl;
          const int4 ra = *reinterpret_cast<const int4*>(rgt + ql0);
          const int4 rb = *reinterpret_cast<const int4*>(rgt + ql0 + 2);
          const int lo[4] = {ra.x, ra.z, rb.x, rb.z}, hi[4] = {ra.y, ra.w, rb.y, rb.w};
#pragma unroll
          for (int e = 0; e < 4; ++e)
            mbits |= (ki < lo[e] || ki >= hi[e] ? 1u : 0u) << (16 * j + 4 * g4 + e);
        }
    };
    // At D <= 128 before the S chain (its latency hides there); at D = 256 (register limit)
    // after it, where the chain's fragment registers are free.
    if (DP <= 128 && MSK && !(flags & 2)) mask_bits();
    auto apply_mask = [&]() {
      if constexpr (MSK) {
        if (DP > 128 && !(flags & 2)) mask_bits();
        if (!p.mask.amask && (flags & 2)) return;
        // Additive-mask values of the tile (LDS, lanes read consecutive keys), all issued
        // before the first use; at D = 256 (register limit) eight at a time.
        constexpr int G = DP >= 256 ? 4 : 16;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int i0 = 0; i0 < 16; i0 += G) {
            float a[G];
#pragma unroll
            for (int i = 0; i < G; ++i) {
              const int ii = i0 + i;
              // At D = 256 the lane's offsets are recomputed rather than held across the step.
              const int ln = DP >= 256 ? __lane_id() : lane;
              const int col = (DP >= 256 ? __builtin_amdgcn_readfirstlane(wave) : wave) * 32 + (ln & 31);
              a[i] = p.mask.amask ? amt[(32 * j + 8 * (ii >> 2) + 4 * (ln >> 5) + (ii & 3)) * BK + col] : 0.f;
            }
#pragma unroll
            for (int i = 0; i < G; ++i)
              s[j][i0 + i] = ((mbits >> (16 * j + i0 + i)) & 1u) ? kMaskValue : s[j][i0 + i] + a[i];
            if (G < 16) __builtin_amdgcn_sched_barrier(0);
          }
        return;
      }
      if ((p.mask.causal && k0 + BK - 1 > t) || p.mask.window) {
        MFA_KEEP_BRANCH();
        {
          // Queries q = t + 4hh + kk stay for q >= ki (causal) and q <= ki + wsz (window).
          const int base = t + 4 * hh;
          const int lo = p.mask.causal ? ki - base : -0x40000000;
          const int hi = p.mask.window ? ki + wsz - base : 0x3fffffff;
          mask_outside<NJ>(s, lo, hi, kMaskValue);
        }
      }
    };
    if (MSK && (flags & 1)) {
      // No row of this step sees the key block: nothing to add (the next tiles' DMA still
      // lands before the barrier).
      if (late_dma) issue_next();
      // (Mask steps issue the next tiles up front: no spread pieces under MSK.)
    } else if constexpr (DP <= 128) {
      // S = Q·K^T; masks; dP = dO·V^T with P = exp2(S·c − L) computed between its MFMAs;
      // dV^T += dO^T·P with dS = P∘(dP·scale − D) computed between its MFMAs; dK^T += Q^T·dS.
      // The S and dP accumulators are read once each into VGPR values (P, and dS eight at a
      // time), never updated in place: in-place updates of MFMA accumulators cost a
      // register-file copy per element each way.
      auto pack8 = [](const float* x) {
        i16x8 f;
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] = (short)E::from_f32(x[e]);
        return f;
      };
      rows_chain<A, NJ, true>(qt, kf, s, rbase, dma_hook);
      apply_mask();
      BST(1);
      float pf[NJ][16];
      {
        float lv[NJ][16];
        lds4(lt, lv);
        constexpr int EPM = 16 / DS;
        rows_chain<A, NJ, true>(ot, vf, dp, rbase, [&](int i) {
#pragma unroll
          for (int e = 0; e < EPM; ++e) {
            const int idx = i * EPM + e, jj = idx >> 4, ii = idx & 15;
            pf[jj][ii] = pexp(s[jj][ii], lv[jj][ii]);
          }
        });
      }
      BST(2);
      i16x8 pb[NJ * 2], sb[NJ * 2];
#pragma unroll
      for (int jk = 0; jk < NJ * 2; ++jk) pb[jk] = pack8(&pf[jk >> 1][8 * (jk & 1)]);
      float dv_[NJ][16];
      lds4(dtl, dv_);
      constexpr int NMV = NJ * 2 * ND;
      constexpr int EPM = (NJ * 16 + NMV - 1) / NMV;
      float d8[8];
      tr_chain<A, NJ, ND>(ot, trb, pb, dv, [&](int i) {
#pragma unroll
        for (int e = 0; e < EPM; ++e) {
          const int idx = i * EPM + e;
          if (idx < NJ * 16) {
            const int jj = idx >> 4, ii = idx & 15;
            d8[ii & 7] = pf[jj][ii] * __builtin_fmaf(dp[jj][ii], sc, -dv_[jj][ii]);
            if ((ii & 7) == 7) sb[jj * 2 + (ii >> 3)] = pack8(d8);
          }
        }
      });
      BST(3);
      tr_chain<A, NJ, ND>(qt, trb, sb, dk, [](int) {});
      BST(4);
    } else if constexpr (kBwdKv256Interleave) {
      // D = 256 at the 512-register limit: the interleave above, with L and D read from LDS
      // four rows at a time inside the hooks (one group ahead) instead of held for the tile.
      auto ldg = [&](const float* base, int grp, float (&v)[4]) {
        const float4 x =
            *reinterpret_cast<const float4*>(base + (grp >> 2) * 32 + 8 * (grp & 3) + 4 * hh);
        v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      };
      constexpr int NG = NJ * 4;  // 4-row groups of the tile
      // S and dP chains together (the registers do not hold a hook's working set beside
      // both chains), then P, then dS threaded through the dV chain.
      dual_rows_chain<A, NJ>(qt, ot, kf, vf, s, dp, rbase, dma_hook);
      if (late_dma) issue_next();
      apply_mask();
      BST(1);
      static_assert(NJ == 1, "D = 256 runs 32-query steps");
      // P of k-step 0 (registers 0..7) before the dV chain, which needs it first; P of k-step 1
      // between the chain's first eight MFMAs (they use k-step 0), dS under all sixteen.
      i16x8 pb[2], sb[2];
      float lq[4][4];
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) ldg(lt, g4, lq[g4]);
#pragma unroll
      for (int ii = 0; ii < 8; ++ii)
        s[0][ii] = pexp(s[0][ii], lq[ii >> 2][ii & 3]);
      pb[0] = A::pack(s[0], 0);
      BST(2);
      {
        constexpr int NMV = 2 * ND;
        static_assert(NMV == 16, "one dS element per dV MFMA");
        float dq[2][4];
        ldg(dtl, 0, dq[0]);
        tr_chain<A, NJ, ND>(ot, trb, pb, dv, [&](int i) {
          if (i < 8) {
            const int ii = 8 + i;
            s[0][ii] = pexp(s[0][ii], lq[ii >> 2][ii & 3]);
            if (i == 7) pb[1] = A::pack(s[0], 1);
          }
          const int ii = i, grp = ii >> 2, k = ii & 3;
          if (k == 0 && grp + 1 < NG) ldg(dtl, grp + 1, dq[(grp + 1) & 1]);
          dp[0][ii] = s[0][ii] * __builtin_fmaf(dp[0][ii], sc, -dq[grp & 1][k]);
          if ((ii & 7) == 7) sb[ii >> 3] = A::pack(dp[0], ii >> 3);
        });
      }
      BST(3);
      tr_chain<A, NJ, ND>(qt, trb, sb, dk, [](int) {});
      BST(4);
    } else {
      // D = 256 (previous schedule) runs at the register limit: S and dP chains together, then the softmax, then
      // dV and dK together.
      dual_rows_chain<A, NJ>(qt, ot, kf, vf, s, dp, rbase, dma_hook);
      if (late_dma) issue_next();
      apply_mask();
      float lv[NJ][16], dv_[NJ][16];
      lds4(lt, lv);
      lds4(dtl, dv_);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = pexp(s[j][i], lv[j][i]);
          s[j][i] = pv;
          dp[j][i] = pv * __builtin_fmaf(dp[j][i], sc, -dv_[j][i]);
        }
      constexpr int NM = NJ * 2 * ND * 2;
      constexpr int AH = 4;
      i16x8 pb[NJ * 2], sb[NJ * 2];
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          pb[j * 2 + ks] = A::pack(s[j], ks);
          sb[j * 2 + ks] = A::pack(dp[j], ks);
        }
      auto rd = [&](int i) {
        const int pair = i >> 1, which = i & 1;
        const int jk = pair / ND, dt = pair % ND;
        return A::read_tr_a(which ? qt : ot, trb, (jk >> 1) * 32, jk & 1, dt * 32);
      };
      i16x8 fr[AH];
#pragma unroll
      for (int i = 0; i < AH; ++i) fr[i] = rd(i);
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        const int pair = i >> 1, which = i & 1;
        const int jk = pair / ND, dt = pair % ND;
        if (which)
          dk[dt] = A::mma(fr[i % AH], sb[jk], dk[dt]);
        else
          dv[dt] = A::mma(fr[i % AH], pb[jk], dv[dt]);
        if (i + AH < NM) fr[i % AH] = rd(i + AH);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    wait_vm();
    BST(5);
    if (has_next) ld_store(cur ^ 1, tn);
    __syncthreads();
    BST(6);
    cur ^= 1;
    t = tn;
    h = hn;
  }
  BST_END();

  if (kvalid) {
    const int64_t krow = (int64_t)(b * p.Hkv + kvh) * p.C + ki;
    float* ok = p.dk + krow * p.D;
    float* ov = p.dv + krow * p.D;
    const float mul = p.dk_mul;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (d < p.D) {
          *reinterpret_cast<float4*>(ok + d) =
              make_float4(dk[dt][4 * g] * mul, dk[dt][4 * g + 1] * mul, dk[dt][4 * g + 2] * mul,
                          dk[dt][4 * g + 3] * mul);
          *reinterpret_cast<float4*>(ov + d) =
              make_float4(dv[dt][4 * g], dv[dt][4 * g + 1], dv[dt][4 * g + 2], dv[dt][4 * g + 3]);
        }
      }
  }
}

template <int DP> struct BwdFastCfg {
  static constexpr int BT = DP >= 256 ? 32 : 64;  // bwd_q key tile
  static constexpr int BQ = DP >= 256 ? 32 : 64;  // bwd_kv query tile
};

template <class E, int DP>
static hipError_t launch_bwd_q_fast(const BwdParams& p, hipStream_t stream) {
  constexpr int BT = BwdFastCfg<DP>::BT;
  constexpr int LDS = 4 * BT * DP * 2;
  BwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const dim3 grid(q.nblk * p.B * p.H);
  if (p.k.prec == P_INT8 || p.k.prec == P_INT4) {
    // Quantised K/V widened on load: the 16-bit ring plus the byte ring (4 tiles of bytes).
    if (p.mask.amask || p.mask.ranges || p.v.prec != p.k.prec) return hipErrorNotSupported;
    if (p.k.prec == P_INT8) {
      using KB = KvBytes<E, DP, BT, SRC_I8, 256>;
      return launch(mfa_bwd_q_fast_kernel<E, DP, BT, false, SRC_I8>, grid, dim3(256),
                    LDS + 4 * KB::SLOT, stream, q);
    }
    using KB = KvBytes<E, DP, BT, SRC_I4, 256>;
    return launch(mfa_bwd_q_fast_kernel<E, DP, BT, false, SRC_I4>, grid, dim3(256),
                  LDS + 4 * KB::SLOT, stream, q);
  }
  if (p.mask.amask || p.mask.ranges)
    return launch(mfa_bwd_q_fast_kernel<E, DP, BT, true>, grid, dim3(256), LDS + 128, stream, q);
  return launch(mfa_bwd_q_fast_kernel<E, DP, BT>, grid, dim3(256), LDS, stream, q);
}

template <class E, int DP>
static hipError_t launch_bwd_kv_fast(const BwdParams& p, hipStream_t stream) {
  constexpr int BQ = BwdFastCfg<DP>::BQ;
  constexpr int LDS = 4 * BQ * DP * 2 + 4 * BQ * 4;
  BwdParams q = p;
  q.nblk = (p.C + 127) / 128;
  const dim3 grid(q.nblk * p.B * p.Hkv);
  if (p.mask.amask || p.mask.ranges) {
    if (p.k.prec != P_FP16 && p.k.prec != P_BF16) return hipErrorNotSupported;
    return launch(mfa_bwd_kv_fast_kernel<E, DP, BQ, SRC_SAME, true>, grid, dim3(256),
                  LDS + 2 * BQ * 8 + 2 * BQ * 128 * 4 + 16, stream, q);
  }
  if (p.k.prec == P_INT8) return launch(mfa_bwd_kv_fast_kernel<E, DP, BQ, SRC_I8>, grid, dim3(256), LDS, stream, q);
  if (p.k.prec == P_INT4) return launch(mfa_bwd_kv_fast_kernel<E, DP, BQ, SRC_I4>, grid, dim3(256), LDS, stream, q);
  return launch(mfa_bwd_kv_fast_kernel<E, DP, BQ>, grid, dim3(256), LDS, stream, q);
}

// kind: 0 = backwardQuery, 1 = backwardKeyValue.  hipErrorNotSupported when not covered.
hipError_t bwd_fast_dispatch(const BwdParams& p, int kind, int elem, int DP, hipStream_t stream) {
#define MFA_BF(ELEM, EE, DPV)                                                       \
  if (elem == ELEM && DP == DPV)                                                    \
    return kind == 0 ? launch_bwd_q_fast<EE, DPV>(p, stream)                        \
                     : launch_bwd_kv_fast<EE, DPV>(p, stream);
  MFA_BF(P_FP16, F16, 64)
  MFA_BF(P_FP16, F16, 128)
  MFA_BF(P_FP16, F16, 256)
  MFA_BF(P_BF16, BF16, 64)
  MFA_BF(P_BF16, BF16, 128)
  MFA_BF(P_BF16, BF16, 256)
#undef MFA_BF
  return hipErrorNotSupported;
}

}  // namespace mfa

// Explicit instantiations: hipcc does not emit every host-side kernel stub that the dispatch
// table above references when the kernels are only named through the launch templates.
namespace mfa {
#define MFA_BF_INST(EE, DPV)                                                                   \
  template __global__ void mfa_bwd_q_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BT>(BwdParams);   \
  template __global__ void mfa_bwd_kv_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BQ>(BwdParams);    \
  template __global__ void mfa_bwd_kv_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BQ, SRC_I8>(BwdParams); \
  template __global__ void mfa_bwd_kv_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BQ, SRC_I4>(BwdParams); \
  template __global__ void mfa_bwd_q_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BT, true>(BwdParams);   \
  template __global__ void mfa_bwd_q_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BT, false, SRC_I8>(BwdParams); \
  template __global__ void mfa_bwd_q_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BT, false, SRC_I4>(BwdParams); \
  template __global__ void mfa_bwd_kv_fast_kernel<EE, DPV, BwdFastCfg<DPV>::BQ, SRC_SAME, true>(BwdParams);
MFA_BF_INST(F16, 64)
MFA_BF_INST(F16, 128)
MFA_BF_INST(F16, 256)
MFA_BF_INST(BF16, 64)
MFA_BF_INST(BF16, 128)
MFA_BF_INST(BF16, 256)
#undef MFA_BF_INST
}  // namespace mfa
