// attention_bigd.hip — the D-blocked forward and backward for head dimensions above 256.
//
// The reference's parameter tables end at maximumHeadDimension 384 and fall back to their
// last row for any larger D (AttentionDescriptor+Parameters.swift:44-69, :116, :142); with no
// operand register-cached it spills O to the FP32 O buffer every traversal block and streams
// every other operand in head-dimension blocks of Bd (README.md:96-104, "infinite head
// dimension").  Same idea on gfx950, with no D limit and no O spill:
//
//   * every contraction over the head dimension (S = Q·K^T, and dP = dO·V^T in the backward)
//     runs in column chunks of DC (128 16-bit / 64 FP32 elements): both operands' [rows][DC]
//     chunks are staged through LDS (register prefetch of the next chunk during the MFMAs of
//     the current one), so no full-D operand is ever held in registers;
//   * the output columns are split into DC-wide slices, one per workgroup (grid.y): its
//     accumulator slice (O^T, dQ^T or dK^T/dV^T) stays in registers for the whole kernel.
//     Each slice's workgroup recomputes S (and dP) over the full D — the price of the split,
//     2·D + 2·DC FLOP per pair and slice in the forward instead of 4·D.
//
// Numerics are those of attention_fwd.hip / attention_bwd.h (same softmax code, exact FP32
// MFMA for FP32 inputs, 16-bit MFMA operands with FP32 accumulation otherwise).  Quantised
// operands reach these kernels through the dequantisation pass (kv_dequant.hip).
#include "attention_bwd.h"
#include "mfa_dispatch.h"

namespace mfa {

template <class A, int ROWS, int DC>
struct BigTile {
  static constexpr int bytes = A::is_f32 ? ROWS * (DC + 1) * 4 : ROWS * DC * 2;
};

// ---------------------------------------------------------------------------------------
// Forward: grid (nblk·B·H, ceil(D / DC)); 4 waves x 32 queries, output columns
// [DC·blockIdx.y, +DC).  Per 32-key tile: nc chunk stages of S^T += K_c·Q_c^T; the last one
// also stages the V slice and ends with the online softmax and O^T += V_slice^T·P^T.
template <class A, int DC>
__global__ void __launch_bounds__(256) mfa_fwd_bigd_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128, BK = 32, ND = DC / 32;
  constexpr int QTB = BigTile<A, BQ, DC>::bytes, KTB = BigTile<A, BK, DC>::bytes;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const qt = smem;
  char* const kt = smem + QTB;
  char* const vt = kt + KTB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.H;
  const int rb = p.nblk - 1 - (int)blockIdx.x / BH;  // heaviest (causal) blocks first
  const int bh = (int)blockIdx.x % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int oc0 = (int)blockIdx.y * DC;
  const int nc = (p.D + DC - 1) / DC;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;

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
  const int ntile = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const int nstage = ntile * nc;

  Stager<A, BQ, DC, NT, SRC_SAME> sq;
  Stager<A, BK, DC, NT, SRC_SAME> sk, sv;
  // Stage i: tile i / nc, chunk c = i % nc (Q_c and K_c); the last chunk's stage also brings
  // the tile's V slice, so that its PV runs right after the softmax.
  auto issue = [&](int i) {
    const int t = kbeg + (i / nc) * BK, c0 = (i % nc) * DC;
    sq.load(p.q, b, h, q0, p.R, p.D - c0, (int64_t)c0 * p.q.sd);
    sk.load(p.k, b, kvh, t, p.C, p.D - c0, (int64_t)c0 * p.k.sd);
    if (i % nc == nc - 1) sv.load(p.v, b, kvh, t, p.C, p.D - oc0, (int64_t)oc0 * p.v.sd);
  };
  auto commit = [&](int i) {
    const int t = kbeg + (i / nc) * BK, c0 = (i % nc) * DC;
    sq.store(qt, p.q, b, h, q0, p.R, p.D - c0);
    sk.store(kt, p.k, b, kvh, t, p.C, p.D - c0);
    if (i % nc == nc - 1) sv.store(vt, p.v, b, kvh, t, p.C, p.D - oc0);
  };

  f32x16 o[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) o[dt] = zero16();
  float m = -kFltMax, l = kFltMin;
  const float c = p.c_log2;
  f32x16 s[1];
  s[0] = zero16();

  if (nstage > 0) {
    issue(0);
    commit(0);
  }
  __syncthreads();
  for (int i = 0; i < nstage; ++i) {
    const int t = kbeg + (i / nc) * BK, ck = i % nc;
    if (i + 1 < nstage) issue(i + 1);
    if (ck == 0) s[0] = zero16();
#pragma unroll 4
    for (int ds = 0; ds < DC / A::KSTEP; ++ds)
      s[0] = A::mma(A::read_row(kt, l32, ds, hh), A::read_row(qt, wave * 32 + l32, ds, hh), s[0]);
    if (ck == nc - 1) {
      const bool need_mask = (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) ||
                             p.mask.window || p.mask.ranges || p.mask.amask;
      if (need_mask) apply_masks<1>(s, t, qi, hh, p, b, h, range);
      float mx = s[0][0];
#pragma unroll
      for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[0][r]);
      mx = xhalf_max(mx);
      const float m_new = mx * c;
      float corr = 1.f;
      if (m_new > m) {
        corr = __builtin_amdgcn_exp2f(m - m_new);
        m = m_new;
      }
      float rs = 0.f;
      const bool exact = __any(m < kMaskLevel);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float x = exact ? mul_rn(s[0][r], c) - m : s[0][r] * c - m;
        const float pv = __builtin_amdgcn_exp2f(x);
        s[0][r] = pv;
        rs += pv;
      }
      rs = xhalf_sum(rs);
      l = l * corr + rs;
      if (!(l > 0.f)) l = kFltMin;
      if (__any(corr != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= corr;
      }
      // O^T += V_slice^T · P^T
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag pb = A::pack(s[0], ks);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          o[dt] = A::mma(A::read_tr(vt, 0, ks, dt * 32, lane), pb, o[dt]);
      }
    }
    __syncthreads();
    if (i + 1 < nstage) commit(i + 1);
    __syncthreads();
  }

  if (qvalid) {
    const float inv = p.o_mul / l;
    float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int d = oc0 + dt * 32 + 8 * g + 4 * hh + e;
          if (d < p.D) orow[(int64_t)d * p.o_sd] = o[dt][4 * g + e] * inv;
        }
    if (hh == 0 && blockIdx.y == 0) {
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
// backwardQuery: grid (nblk·B·H, ceil(D / DC)); 4 waves x 32 queries, dQ columns
// [DC·blockIdx.y, +DC).  Per 32-key tile: nc chunk stages of S^T += K_c·Q_c^T and
// dP^T += V_c·dO_c^T, chunk blockIdx.y last so that the K tile in LDS after the last stage is
// the slice dQ^T += K_slice^T·dS^T reads.  DOS: dO staged as stored (SRC_SAME) or FP32
// rounded to the compute type (SRC_F32ANY, the quantised API's FP32 dO).
template <class A, int DC, int DOS>
__global__ void __launch_bounds__(256) mfa_bwd_q_bigd_kernel(BwdParams p) {
  constexpr int NT = 256, BQ = 128, BT = 32, ND = DC / 32;
  constexpr int QTB = BigTile<A, BQ, DC>::bytes, KTB = BigTile<A, BT, DC>::bytes;
  constexpr int DOSRC = DOS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const qt = smem;
  char* const dot = smem + QTB;
  char* const kt = dot + QTB;
  char* const vt = kt + KTB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.H;
  const int rb = p.nblk - 1 - (int)blockIdx.x / BH;
  const int bh = (int)blockIdx.x % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int ob = blockIdx.y, oc0 = ob * DC;
  const int nc = (p.D + DC - 1) / DC;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;
  const int64_t row = (int64_t)(b * p.H + h) * p.R + qi;

  const float dsum = xhalf_sum(qvalid ? rowsum_do_o<A>(p, b, h, qi, hh) : 0.f);
  const float Drow = p.dscale * dsum;
  const float Lrow = qvalid ? load_l(p, row) : 0.f;
  if (qvalid && hh == 0 && ob == 0) {
    if (p.d_bf16)
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
  const int ntile = kend > kbeg ? (kend - kbeg + BT - 1) / BT : 0;
  const int nstage = ntile * nc;

  Stager<A, BQ, DC, NT, SRC_SAME> sq;
  Stager<A, BQ, DC, NT, DOSRC> sdo;
  Stager<A, BT, DC, NT, SRC_SAME> sk, sv;
  // Stage i: tile i / nc, chunk (ob + 1 + i % nc) % nc — chunk ob last.
  auto chunk = [&](int i) { return (ob + 1 + i % nc) % nc; };
  auto issue = [&](int i) {
    const int t = kbeg + (i / nc) * BT, c0 = chunk(i) * DC;
    sq.load(p.q, b, h, q0, p.R, p.D - c0, (int64_t)(c0) * p.q.sd);
    sdo.load(p.dO_op, b, h, q0, p.R, p.D - c0, (int64_t)(c0) * p.dO_op.sd);
    sk.load(p.k, b, kvh, t, p.C, p.D - c0, (int64_t)(c0) * p.k.sd);
    sv.load(p.v, b, kvh, t, p.C, p.D - c0, (int64_t)(c0) * p.v.sd);
  };
  auto commit = [&](int i) {
    const int t = kbeg + (i / nc) * BT, c0 = chunk(i) * DC;
    sq.store(qt, p.q, b, h, q0, p.R, p.D - c0);
    sdo.store(dot, p.dO_op, b, h, q0, p.R, p.D - c0);
    sk.store(kt, p.k, b, kvh, t, p.C, p.D - c0);
    sv.store(vt, p.v, b, kvh, t, p.C, p.D - c0);
  };

  f32x16 dq[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dq[dt] = zero16();
  const float c = p.c_log2;
  f32x16 s = zero16(), dp = zero16();

  if (nstage > 0) {
    issue(0);
    commit(0);
  }
  __syncthreads();
  for (int i = 0; i < nstage; ++i) {
    const int t = kbeg + (i / nc) * BT, ck = i % nc;
    if (i + 1 < nstage) issue(i + 1);
    if (ck == 0) {
      s = zero16();
      dp = zero16();
    }
#pragma unroll 4
    for (int ds = 0; ds < DC / A::KSTEP; ++ds) {
      s = A::mma(A::read_row(kt, l32, ds, hh), A::read_row(qt, wave * 32 + l32, ds, hh), s);
      dp = A::mma(A::read_row(vt, l32, ds, hh), A::read_row(dot, wave * 32 + l32, ds, hh), dp);
    }
    if (ck == nc - 1) {
      const bool need_mask = (t + BT > p.C) || (p.mask.causal && t + BT - 1 > q0) ||
                             p.mask.window || p.mask.ranges || p.mask.amask || !qvalid;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = s[r];
        if (need_mask) {
          const int key = t + acc_row(r, hh);
          if (key >= p.C || !qvalid) {
            x = -__builtin_inff();
          } else {
            if (p.mask.amask) x += p.mask.amask[row * p.C + key];
            bool mk = false;
            if (p.mask.causal && key > qi) mk = true;
            if (p.mask.window && (int64_t)qi > (int64_t)key + (int64_t)p.mask.window_size) mk = true;
            if (p.mask.ranges && ((uint32_t)key < range.x || (uint32_t)key >= range.y)) mk = true;
            if (mk) x = kMaskValue;
          }
        }
        const float xc = Lrow < kMaskLevel ? mul_rn(x, c) : x * c;
        const float pv = __builtin_amdgcn_exp2f(xc - Lrow);
        s[r] = pv;
        dp[r] = pv * (dp[r] * p.scale - Drow);
      }
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag db = A::pack(dp, ks);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
          dq[dt] = A::mma(A::read_tr(kt, 0, ks, dt * 32, lane), db, dq[dt]);
      }
    }
    __syncthreads();
    if (i + 1 < nstage) commit(i + 1);
    __syncthreads();
  }

  if (qvalid) {
    float* out = p.dq + (int64_t)(b * p.H + h) * p.R * p.D + (int64_t)qi * p.dq_ss;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int d = oc0 + dt * 32 + 8 * g + 4 * hh + e;
          if (d < p.D) out[(int64_t)d * p.dq_sd] = dq[dt][4 * g + e] * p.dq_mul;
        }
  }
}

// ---------------------------------------------------------------------------------------
// backwardKeyValue: grid (nblk·B·H_kv, ceil(D / DC)); 4 waves x 32 keys, dK/dV columns
// [DC·blockIdx.y, +DC).  Steps run over every query head of the kv group and every 32-query
// tile (GQA summed in the workgroup, no atomics); per step nc chunk stages of
// S += Q_c·K_c^T and dP += dO_c·V_c^T (key on the lane), chunk blockIdx.y last so that the
// Q / dO tiles in LDS after the last stage are the slices dK^T += Q_slice^T·dS and
// dV^T += dO_slice^T·P read.
template <class A, int DC, int DOS>
__global__ void __launch_bounds__(256) mfa_bwd_kv_bigd_kernel(BwdParams p) {
  constexpr int NT = 256, BK = 128, BT = 32, ND = DC / 32;
  constexpr int KTB = BigTile<A, BK, DC>::bytes, QTB = BigTile<A, BT, DC>::bytes;
  constexpr int DOSRC = DOS;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kt = smem;
  char* const vt = smem + KTB;
  char* const qt = vt + KTB;
  char* const dot = qt + QTB;
  float* const lt = reinterpret_cast<float*>(dot + QTB);  // [BT] L, then [BT] D
  float* const dtl = lt + BT;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.Hkv;
  const int kb = (int)blockIdx.x / BH;
  const int bh = (int)blockIdx.x % BH;
  const int b = bh / p.Hkv, kvh = bh % p.Hkv;
  const int ob = blockIdx.y, oc0 = ob * DC;
  const int nc = (p.D + DC - 1) / DC;
  const int k0 = kb * BK;
  const int ki = k0 + wave * 32 + l32;
  const bool kvalid = ki < p.C;

  int qbeg = 0, qend = p.R;
  if (p.mask.causal && p.mask.skip_ok) qbeg = (k0 / BT) * BT;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t hi = (int64_t)k0 + BK + (int64_t)p.mask.window_size;
    if (hi < qend) qend = (int)hi;
  }
  const int ntile = qbeg < qend ? (qend - qbeg + BT - 1) / BT : 0;
  const int ngroup = (p.H - kvh + p.Hkv - 1) / p.Hkv;
  const int nstep = ntile * ngroup;
  // Stage i: step i / (2·nc); chunk position k = (i / 2) % nc (chunk (ob + 1 + k) % nc, so
  // chunk ob comes last); half i % 2: 0 stages K_c (own rows) and Q_c (tile) for
  // S += Q_c·K_c^T, 1 stages V_c and dO_c for dP += dO_c·V_c^T.  Halving the stages halves the
  // staging registers in flight across the MFMAs.
  const int nstage = nstep * nc * 2;

  Stager<A, BK, DC, NT, SRC_SAME> sown;
  Stager<A, BT, DC, NT, SRC_SAME> sq;
  Stager<A, BT, DC, NT, DOSRC> sdo;
  float lreg = 0.f, dreg = 0.f;
  auto where = [&](int i, int& h, int& t, int& c0) {
    const int st = i / (2 * nc);
    h = kvh + (st / ntile) * p.Hkv;
    t = qbeg + (st % ntile) * BT;
    c0 = ((ob + 1 + (i / 2) % nc) % nc) * DC;
  };
  auto issue = [&](int i) {
    int h, t, c0;
    where(i, h, t, c0);
    if ((i & 1) == 0) {
      sown.load(p.k, b, kvh, k0, p.C, p.D - c0, (int64_t)c0 * p.k.sd);
      sq.load(p.q, b, h, t, p.R, p.D - c0, (int64_t)c0 * p.q.sd);
    } else {
      sown.load(p.v, b, kvh, k0, p.C, p.D - c0, (int64_t)c0 * p.v.sd);
      sdo.load(p.dO_op, b, h, t, p.R, p.D - c0, (int64_t)c0 * p.dO_op.sd);
    }
    if (i % (2 * nc) == 0 && tid < BT) {
      const int q = t + tid;
      const int64_t r = (int64_t)(b * p.H + h) * p.R + q;
      lreg = q < p.R ? load_l(p, r) : 0.f;
      dreg = q < p.R ? load_d(p, r) : 0.f;
    }
  };
  auto commit = [&](int i) {
    int h, t, c0;
    where(i, h, t, c0);
    if ((i & 1) == 0) {
      sown.store(kt, p.k, b, kvh, k0, p.C, p.D - c0);
      sq.store(qt, p.q, b, h, t, p.R, p.D - c0);
    } else {
      sown.store(vt, p.v, b, kvh, k0, p.C, p.D - c0);
      sdo.store(dot, p.dO_op, b, h, t, p.R, p.D - c0);
    }
    if (i % (2 * nc) == 0 && tid < BT) {
      lt[tid] = lreg;
      dtl[tid] = dreg;
    }
  };

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    dk[dt] = zero16();
    dv[dt] = zero16();
  }
  const float c = p.c_log2;
  f32x16 s = zero16(), dp = zero16();

  if (nstage > 0) {
    issue(0);
    commit(0);
  }
  __syncthreads();
  for (int i = 0; i < nstage; ++i) {
    int h, t, c0;
    where(i, h, t, c0);
    const int ck = i % (2 * nc);
    if (i + 1 < nstage) issue(i + 1);
    if (ck == 0) {
      s = zero16();
      dp = zero16();
    }
    if ((i & 1) == 0) {
#pragma unroll 4
      for (int ds = 0; ds < DC / A::KSTEP; ++ds)
        s = A::mma(A::read_row(qt, l32, ds, hh), A::read_row(kt, wave * 32 + l32, ds, hh), s);
    } else {
#pragma unroll 4
      for (int ds = 0; ds < DC / A::KSTEP; ++ds)
        dp = A::mma(A::read_row(dot, l32, ds, hh), A::read_row(vt, wave * 32 + l32, ds, hh), dp);
    }
    if (ck == 2 * nc - 1) {
      const bool need_mask = !kvalid || (t + BT > p.R) || (p.mask.causal && k0 + BK - 1 > t) ||
                             p.mask.window || p.mask.ranges || p.mask.amask;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qloc = acc_row(r, hh);
        float x = s[r];
        if (need_mask) x = mask_value(p, x, t + qloc, ki, b, h, kvh);
        const float lq = lt[qloc];
        const float xc = lq < kMaskLevel ? mul_rn(x, c) : x * c;
        const float pv = __builtin_amdgcn_exp2f(xc - lq);
        s[r] = pv;
        dp[r] = pv * (dp[r] * p.scale - dtl[qloc]);
      }
#pragma unroll
      for (int ks = 0; ks < A::KS32; ++ks) {
        const typename A::frag pb = A::pack(s, ks);
        const typename A::frag sb = A::pack(dp, ks);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          dv[dt] = A::mma(A::read_tr(dot, 0, ks, dt * 32, lane), pb, dv[dt]);
          dk[dt] = A::mma(A::read_tr(qt, 0, ks, dt * 32, lane), sb, dk[dt]);
        }
      }
    }
    __syncthreads();
    if (i + 1 < nstage) commit(i + 1);
    __syncthreads();
  }

  if (kvalid) {
    const int64_t slice = (int64_t)(b * p.Hkv + kvh) * p.C * p.D;
    float* ok = p.dk + slice + (int64_t)ki * p.dk_ss;
    float* ov = p.dv + slice + (int64_t)ki * p.dv_ss;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int d = oc0 + dt * 32 + 8 * g + 4 * hh + e;
          if (d < p.D) {
            ok[(int64_t)d * p.dk_sd] = dk[dt][4 * g + e] * p.dk_mul;
            ov[(int64_t)d * p.dv_sd] = dv[dt][4 * g + e];
          }
        }
  }
}

// ---------------------------------------------------------------------------------------
template <class A, int DC>
static hipError_t launch_fwd_bigd(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = BigTile<A, 128, DC>::bytes + 2 * BigTile<A, 32, DC>::bytes;
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const dim3 grid(q.nblk * p.B * p.H, (p.D + DC - 1) / DC);
  return launch(mfa_fwd_bigd_kernel<A, DC>, grid, dim3(256), LDS, stream, q);
}

template <class A, int DC, int DOS>
static hipError_t launch_bwd_bigd(const BwdParams& p, int kind, hipStream_t stream) {
  constexpr int LDS = 2 * BigTile<A, 128, DC>::bytes + 2 * BigTile<A, 32, DC>::bytes + 2 * 32 * 4;
  BwdParams q = p;
  const int nob = (p.D + DC - 1) / DC;
  if (kind == 0) {
    q.nblk = (p.R + 127) / 128;
    return launch(mfa_bwd_q_bigd_kernel<A, DC, DOS>, dim3(q.nblk * p.B * p.H, nob), dim3(256), LDS,
                  stream, q);
  }
  q.nblk = (p.C + 127) / 128;
  return launch(mfa_bwd_kv_bigd_kernel<A, DC, DOS>, dim3(q.nblk * p.B * p.Hkv, nob), dim3(256), LDS,
                stream, q);
}

hipError_t fwd_bigd_dispatch(const FwdParams& p, int elem, hipStream_t stream) {
  if (p.q.prec != p.k.prec || p.k.prec != p.v.prec || p.q.prec != elem)
    return hipErrorNotSupported;  // quantised operands arrive dequantised (kv_dequant.hip)
  switch (elem) {
    case P_FP32: return launch_fwd_bigd<Arith32<64>, 64>(p, stream);
    case P_FP16: return launch_fwd_bigd<Arith16<F16, 128>, 128>(p, stream);
    case P_BF16: return launch_fwd_bigd<Arith16<BF16, 128>, 128>(p, stream);
    default: return hipErrorNotSupported;
  }
}

hipError_t bwd_bigd_dispatch(const BwdParams& p, int kind, int elem, hipStream_t stream) {
  if (p.q.prec != p.k.prec || p.k.prec != p.v.prec || p.q.prec != elem)
    return hipErrorNotSupported;
  // dO in the compute precision, or FP32 in memory rounded on staging (16-bit compute only).
  const bool do_same = p.dO_op.prec == elem;
  if (!do_same && (elem == P_FP32 || p.dO_op.prec != P_FP32)) return hipErrorNotSupported;
  switch (elem) {
    case P_FP32: return launch_bwd_bigd<Arith32<64>, 64, SRC_SAME>(p, kind, stream);
    case P_FP16:
      return do_same ? launch_bwd_bigd<Arith16<F16, 128>, 128, SRC_SAME>(p, kind, stream)
                     : launch_bwd_bigd<Arith16<F16, 128>, 128, SRC_F32ANY>(p, kind, stream);
    case P_BF16:
      return do_same ? launch_bwd_bigd<Arith16<BF16, 128>, 128, SRC_SAME>(p, kind, stream)
                     : launch_bwd_bigd<Arith16<BF16, 128>, 128, SRC_F32ANY>(p, kind, stream);
    default: return hipErrorNotSupported;
  }
}

}  // namespace mfa
