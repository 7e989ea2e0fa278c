// attention_bwd.h — the two backward phases of the reference's 7-GEMM backward, on gfx950.
//
// backwardQuery (AttentionKernel+Source.swift:418-459, setup computeD Softmax.swift:31-236):
//   D = scale·rowsum(dO∘O) ; per key tile: S = Q·K^T, P = exp2(S·log2e·scale - L),
//   dP = dO·V^T, dS = P∘(dP·scale - D), dQ += dS·K                         (3 GEMMs)
// backwardKeyValue (AttentionKernel+Source.swift:461-511):
//   per query tile: S^T = K·Q^T, P^T, dV += P^T·dO, dP^T = V·dO^T, dS^T, dK += dS^T·Q (4 GEMMs)
//
// No atomics: each phase owns its outputs (dQ per query block, dK/dV per key block), which is
// the reference's design for hardware without float atomics (README.md:89-94) and gives
// bit-reproducible gradients.  GQA/MQA: the key/value phase sums over every query head of the
// group inside one workgroup (the reference stores per query head without a reduction,
// SURVEY.md §8a quirk 2).
//
// Both phases keep "their" operand on the MFMA lane so every accumulator feeds the next
// product directly (see mfa_device.h):
//   bwd_q : S^T / dP^T / dS^T with the query on the lane; dQ^T += K^T·dS^T (K^T via tr-read).
//   bwd_kv: S / dP / dS with the key on the lane; dV^T += dO^T·P, dK^T += Q^T·dS
//           (dO^T and Q^T via tr-read of the row-major LDS tiles).
#pragma once
#include "mfa_stage.h"

namespace mfa {

__device__ __forceinline__ float load_l(const BwdParams& p, int64_t i) {
  return p.l_f16 ? f16_to_f32(reinterpret_cast<const uint16_t*>(p.l)[i])
                 : reinterpret_cast<const float*>(p.l)[i];
}
__device__ __forceinline__ float load_d(const BwdParams& p, int64_t i) {
  return p.d_bf16 ? bf16_to_f32(reinterpret_cast<const uint16_t*>(p.dD)[i])
                  : reinterpret_cast<const float*>(p.dD)[i];
}
__device__ __forceinline__ float load_elem(const Operand& op, int64_t e) {
  switch (op.prec) {
    case P_FP32: return reinterpret_cast<const float*>(op.ptr)[e];
    case P_FP16: return f16_to_f32(reinterpret_cast<const uint16_t*>(op.ptr)[e]);
    case P_BF16: return bf16_to_f32(reinterpret_cast<const uint16_t*>(op.ptr)[e]);
    default: return 0.f;
  }
}

// Mask predicate shared by both phases (query row q, key col k).  Returns the value S takes.
__device__ __forceinline__ float mask_value(const BwdParams& p, float s, int q, int k, int b, int h,
                                            int kvh) {
  if (k >= p.C || q >= p.R) return -__builtin_inff();
  if (p.mask.amask) s += p.mask.amask[((int64_t)(b * p.H + h) * p.R + q) * p.C + k];
  bool m = false;
  if (p.mask.causal && k > q) m = true;
  if (p.mask.window && (int64_t)q > (int64_t)k + (int64_t)p.mask.window_size) m = true;
  if (p.mask.ranges) {
    const uint32_t* rp = p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + q);
    if ((uint32_t)k < rp[0] || (uint32_t)k >= rp[1]) m = true;
  }
  return m ? kMaskValue : s;
}

// This lane's half of Σ_d dO[qi, d]·O[qi, d] (computeD, AttentionKernel+Softmax.swift:31-236),
// from the values in memory (dO registers are FP32 in the reference, Precisions.swift:183-185);
// lane half hh takes d in [KSTEP/2·hh, KSTEP/2·(hh+1)) of every KSTEP-wide step.
template <class A>
__device__ __forceinline__ float rowsum_do_o(const BwdParams& p, int b, int h, int qi, int hh) {
  const float* orow = p.o + (int64_t)(b * p.H + h) * p.R * p.D + (int64_t)qi * p.o_ss;
  const int64_t dorow = (int64_t)b * p.dO_op.sb + (int64_t)h * p.dO_op.sh + (int64_t)qi * p.dO_op.ss;
  float dsum = 0.f;
  for (int d0 = (A::KSTEP / 2) * hh; d0 < p.D; d0 += A::KSTEP) {
#pragma unroll
    for (int j = 0; j < A::KSTEP / 2; ++j) {
      const int d = d0 + j;
      if (d < p.D)
        dsum += load_elem(p.dO_op, dorow + (int64_t)d * p.dO_op.sd) * orow[(int64_t)d * p.o_sd];
    }
  }
  return dsum;
}

// ---------------------------------------------------------------------------------------
// backwardQuery: grid = nblk x B x H (1-D, heaviest causal blocks first); NW waves x 32 queries.
template <class A, int DP, int BT, int NW, int KSRC>
__global__ void __launch_bounds__(NW * 64) mfa_bwd_q_kernel(BwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NW * 64;
  constexpr int BQ = NW * 32;
  constexpr int NJ = BT / 32;
  constexpr int TILEB = A::is_f32 ? BT * (DP + 1) * 4 : BT * DP * 2;
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int rb = p.nblk - 1 - bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;
  const int64_t row = (int64_t)(b * p.H + h) * p.R + qi;

  typename A::frag qf[A::DSTEPS];
  typename A::frag dof[A::DSTEPS];
  load_row_frags<A, DP>(qf, p.q, b, h, qi, qvalid, hh, p.D);
  load_row_frags<A, DP>(dof, p.dO_op, b, h, qi, qvalid, hh, p.D);

  // D = scale · Σ_d dO∘O over the lane's half of the head dimension (computeD), from the
  // values in memory (dO registers are FP32 in the reference, Precisions.swift:183-185).
  float dsum = qvalid ? rowsum_do_o<A>(p, b, h, qi, hh) : 0.f;
  dsum = xhalf_sum(dsum);
  const float Drow = p.dscale * dsum;  // D_sram *= dotProductScale(derivative: true)
  const float Lrow = qvalid ? load_l(p, row) : 0.f;
  if (qvalid && hh == 0) {
    if (p.d_bf16)  // BF16 memory form = upper half of the FP32 bits (Caching.swift:413-421)
      reinterpret_cast<uint16_t*>(p.dD)[row] = (uint16_t)(__builtin_bit_cast(uint32_t, Drow) >> 16);
    else
      reinterpret_cast<float*>(p.dD)[row] = Drow;
  }

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
    kbeg = lo > 0 ? (int)(lo / BT) * BT : 0;
  }

  f32x16 dq[DP / 32];
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt) dq[dt] = zero16();
  const float c = p.c_log2;

  Stager<A, BT, DP, NT, KSRC> sk;
  Stager<A, BT, DP, NT, KSRC> sv;
  if (kbeg < kend) {
    sk.load(p.k, b, kvh, kbeg, p.C, p.D);
    sv.load(p.v, b, kvh, kbeg, p.C, p.D);
    sk.store(kb0, p.k, b, kvh, kbeg, p.C, p.D);
    sv.store(vb0, p.v, b, kvh, kbeg, p.C, p.D);
  }
  __syncthreads();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BT) {
    const bool has_next = t + BT < kend;
    if (has_next) {
      sk.load(p.k, b, kvh, t + BT, p.C, p.D);
      sv.load(p.v, b, kvh, t + BT, p.C, p.D);
    }
    const char* kt = kb0 + cur * TILEB;
    const char* vt = vb0 + cur * TILEB;

    f32x16 s[NJ], dp[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { s[j] = zero16(); dp[j] = zero16(); }
#pragma unroll
    for (int ds = 0; ds < A::DSTEPS; ++ds) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        s[j] = A::mma(A::read_row(kt, j * 32 + l32, ds, hh), qf[ds], s[j]);
        dp[j] = A::mma(A::read_row(vt, j * 32 + l32, ds, hh), dof[ds], dp[j]);
      }
    }
    const bool need_mask = (t + BT > p.C) || (p.mask.causal && t + BT - 1 > q0) ||
                           p.mask.window || p.mask.ranges || p.mask.amask || !qvalid;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        float x = s[j][i];
        if (need_mask) {
          const int key = t + j * 32 + acc_row(i, hh);
          if (key >= p.C || !qvalid) {
            x = -__builtin_inff();
          } else {
            if (p.mask.amask) x += p.mask.amask[row * p.C + key];
            bool m = false;
            if (p.mask.causal && key > qi) m = true;
            if (p.mask.window && (int64_t)qi > (int64_t)key + (int64_t)p.mask.window_size) m = true;
            if (p.mask.ranges && ((uint32_t)key < range.x || (uint32_t)key >= range.y)) m = true;
            if (m) x = kMaskValue;
          }
        }
        const float xc = Lrow < kMaskLevel ? mul_rn(x, c) : x * c;
        const float pv = __builtin_amdgcn_exp2f(xc - Lrow);
        s[j][i] = pv;
        dp[j][i] = pv * (dp[j][i] * p.scale - Drow);  // dS (derivative softmax, :795-804)
      }
    }
    // dQ^T += K^T · dS^T
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag db = A::pack(dp[j], ks);
#pragma unroll
        for (int dt = 0; dt < DP / 32; ++dt)
          dq[dt] = A::mma(A::read_tr(kt, j * 32, ks, dt * 32, lane), db, dq[dt]);
      }
    }

    if (has_next) {
      sk.store(kb0 + (cur ^ 1) * TILEB, p.k, b, kvh, t + BT, p.C, p.D);
      sv.store(vb0 + (cur ^ 1) * TILEB, p.v, b, kvh, t + BT, p.C, p.D);
    }
    __syncthreads();
    cur ^= 1;
  }

  if (qvalid) {
    float* out = p.dq + (int64_t)(b * p.H + h) * p.R * p.D + (int64_t)qi * p.dq_ss;
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (d + e < p.D) out[(int64_t)(d + e) * p.dq_sd] = dq[dt][4 * g + e] * p.dq_mul;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// backwardKeyValue: grid = (nblk x B x H_kv, DP / DC); NW waves x 32 keys; traverses every
// query head of the group and every query tile.  Workgroup y accumulates dK/dV columns
// [DC·y, DC·y + DC) only: at DP = 256 (DC = 128) the 256-column accumulators beside the
// fragments and staging registers spilled ~470 registers; the two column halves each recompute
// S and dP instead (1.5x the MFMA work of the unsplit kernel, no scratch).
template <class A, int DP, int BT, int NW, int QSRC, int DC = DP>
__global__ void __launch_bounds__(NW * 64) mfa_bwd_kv_kernel(BwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int NT = NW * 64;
  constexpr int BK = NW * 32;
  constexpr int NJ = BT / 32;
  constexpr int NDC = DC / 32;
  constexpr int TILEB = A::is_f32 ? BT * (DP + 1) * 4 : BT * DP * 2;
  char* const qb0 = smem;
  char* const ob0 = smem + 2 * TILEB;
  float* const lb0 = reinterpret_cast<float*>(smem + 4 * TILEB);  // [2][BT] L, [2][BT] D
  float* const db0 = lb0 + 2 * BT;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.Hkv;
  const int bid = blockIdx.x;
  const int kb = bid / BH;  // causal: the first key blocks carry the most query tiles
  const int bh = bid % BH;
  const int b = bh / p.Hkv, kvh = bh % p.Hkv;
  const int k0 = kb * BK;
  const int ki = k0 + wave * 32 + l32;
  const bool kvalid = ki < p.C;

  typename A::frag kf[A::DSTEPS];
  typename A::frag vf[A::DSTEPS];
  load_row_frags<A, DP>(kf, p.k, b, kvh, ki, kvalid, hh, p.D);
  load_row_frags<A, DP>(vf, p.v, b, kvh, ki, kvalid, hh, p.D);

  int qbeg = 0, qend = p.R;
  if (p.mask.causal && p.mask.skip_ok) qbeg = (k0 / BT) * BT;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t hi = (int64_t)k0 + BK + (int64_t)p.mask.window_size;
    if (hi < qend) qend = (int)hi;
  }
  const int ntile = qbeg < qend ? (qend - qbeg + BT - 1) / BT : 0;
  // Query heads of this kv head: h = kvh + g*Hkv (kv_head = head % num_kv_heads).
  const int ngroup = (p.H - kvh + p.Hkv - 1) / p.Hkv;
  const int nsteps = ntile * ngroup;

  const int oc0 = (int)blockIdx.y * DC;
  f32x16 dk[NDC], dv[NDC];
#pragma unroll
  for (int dt = 0; dt < NDC; ++dt) { dk[dt] = zero16(); dv[dt] = zero16(); }
  const float c = p.c_log2;

  Stager<A, BT, DP, NT, QSRC> sq;
  Stager<A, BT, DP, NT, A::is_f32 ? SRC_SAME : SRC_F32ANY> so;
  float lreg = 0.f, dreg = 0.f;
  auto stage_load = [&](int step) {
    const int g = step / ntile, t = qbeg + (step % ntile) * BT;
    const int h = kvh + g * p.Hkv;
    sq.load(p.q, b, h, t, p.R, p.D);
    so.load(p.dO_op, b, h, t, p.R, p.D);
    if (tid < BT) {
      const int q = t + tid;
      const int64_t r = (int64_t)(b * p.H + h) * p.R + q;
      lreg = q < p.R ? load_l(p, r) : 0.f;
      dreg = q < p.R ? load_d(p, r) : 0.f;
    }
  };
  auto stage_store = [&](int step, int buf) {
    const int g = step / ntile, t = qbeg + (step % ntile) * BT;
    const int h = kvh + g * p.Hkv;
    sq.store(qb0 + buf * TILEB, p.q, b, h, t, p.R, p.D);
    so.store(ob0 + buf * TILEB, p.dO_op, b, h, t, p.R, p.D);
    if (tid < BT) {
      lb0[buf * BT + tid] = lreg;
      db0[buf * BT + tid] = dreg;
    }
  };

  if (nsteps > 0) {
    stage_load(0);
    stage_store(0, 0);
  }
  __syncthreads();

  int cur = 0;
  for (int step = 0; step < nsteps; ++step) {
    const bool has_next = step + 1 < nsteps;
    if (has_next) stage_load(step + 1);
    const int g = step / ntile, t = qbeg + (step % ntile) * BT;
    const int h = kvh + g * p.Hkv;
    const char* qt = qb0 + cur * TILEB;
    const char* ot = ob0 + cur * TILEB;
    const float* lt = lb0 + cur * BT;
    const float* dt_ = db0 + cur * BT;

    // S = Q·K^T and dP = dO·V^T with the key on the lane, queries in registers.
    f32x16 s[NJ], dp[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) { s[j] = zero16(); dp[j] = zero16(); }
#pragma unroll
    for (int ds = 0; ds < A::DSTEPS; ++ds) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        s[j] = A::mma(A::read_row(qt, j * 32 + l32, ds, hh), kf[ds], s[j]);
        dp[j] = A::mma(A::read_row(ot, j * 32 + l32, ds, hh), vf[ds], dp[j]);
      }
    }
    const bool need_mask = !kvalid || (t + BT > p.R) || (p.mask.causal && k0 + BK - 1 > t) ||
                           p.mask.window || p.mask.ranges || p.mask.amask;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qloc = j * 32 + acc_row(i, hh);
        float x = s[j][i];
        if (need_mask) x = mask_value(p, x, t + qloc, ki, b, h, kvh);
        const float lq = lt[qloc];
        const float xc = lq < kMaskLevel ? mul_rn(x, c) : x * c;
        const float pv = __builtin_amdgcn_exp2f(xc - lq);
        s[j][i] = pv;
        dp[j][i] = pv * (dp[j][i] * p.scale - dt_[qloc]);
      }
    }
    // dV^T += dO^T · P ; dK^T += Q^T · dS
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag pb = A::pack(s[j], ks);
        const typename A::frag sb = A::pack(dp[j], ks);
#pragma unroll
        for (int d = 0; d < NDC; ++d) {
          dv[d] = A::mma(A::read_tr(ot, j * 32, ks, oc0 + d * 32, lane), pb, dv[d]);
          dk[d] = A::mma(A::read_tr(qt, j * 32, ks, oc0 + d * 32, lane), sb, dk[d]);
        }
      }
    }
    if (has_next) stage_store(step + 1, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  if (kvalid) {
    const int64_t slice = (int64_t)(b * p.Hkv + kvh) * p.C * p.D;
    float* ok = p.dk + slice + (int64_t)ki * p.dk_ss;
    float* ov = p.dv + slice + (int64_t)ki * p.dv_ss;
#pragma unroll
    for (int d = 0; d < NDC; ++d) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int dd = oc0 + d * 32 + 8 * g + 4 * hh;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (dd + e < p.D) {
            ok[(int64_t)(dd + e) * p.dk_sd] = dk[d][4 * g + e] * p.dk_mul;
            ov[(int64_t)(dd + e) * p.dv_sd] = dv[d][4 * g + e];
          }
      }
    }
  }
}

template <class A, int DP, int BT, int NW, int KSRC>
hipError_t launch_bwd_q(const BwdParams& p, hipStream_t stream) {
  constexpr int TILEB = A::is_f32 ? BT * (DP + 1) * 4 : BT * DP * 2;
  constexpr int LDS = 4 * TILEB;
  auto kern = mfa_bwd_q_kernel<A, DP, BT, NW, KSRC>;
  return launch(kern, dim3(p.nblk * p.B * p.H), dim3(NW * 64), LDS, stream, p);
}

template <class A, int DP, int BT, int NW, int QSRC>
hipError_t launch_bwd_kv(const BwdParams& p, hipStream_t stream) {
  constexpr int TILEB = A::is_f32 ? BT * (DP + 1) * 4 : BT * DP * 2;
  constexpr int LDS = 4 * TILEB + 4 * BT * 4;
  constexpr int DC = DP >= 256 ? (A::is_f32 ? 64 : 128) : DP;  // dK/dV columns per workgroup
  auto kern = mfa_bwd_kv_kernel<A, DP, BT, NW, QSRC, DC>;
  return launch(kern, dim3(p.nblk * p.B * p.Hkv, DP / DC), dim3(NW * 64), LDS, stream, p);
}

}  // namespace mfa
