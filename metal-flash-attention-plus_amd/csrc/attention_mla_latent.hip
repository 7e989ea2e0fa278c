// attention_mla_latent.hip — attention in the MLA latent space (the absorbed form of
// MLAOptimizedGEMMMFA, MLAOptimizedGEMMMFA.swift:158-240).
//
// The decompress path computes K_h = latent·W_k,h and V_h = latent·W_v,h, then attends per
// head.  Since Q_h·K_hᵀ = (Q_h·W_k,hᵀ)·latentᵀ and P·V_h = (P·latent)·W_v,h, the same result
// comes from
//     Q̃_h = Q_h·W_k,hᵀ                        (general GEMM, B transposed)
//     Õ_h = softmax(scale·Q̃_h·latentᵀ)·latent (this kernel: every head attends to ONE
//                                               [S_kv, LAT] latent, used as both K and V)
//     O_h = Õ_h·W_v,h                          (16-bit GEMM)
// with the softmax scale of the decompressed head dimension.  K/V are never materialised;
// the latent is read once per query block instead of two [S_kv, H·D] tensors.
//
// Kernel structure: all heads share the latent, so query rows of every head of a batch item
// are one flattened [H·S_q, LAT] problem (MQA with a single KV head).  A workgroup is 4 waves
// on 32 query rows; wave w owns latent dims [w·LAT/4, (w+1)·LAT/4) of both products:
//   * Sᵀ_w = latent[:, slice]·Q̃[:, slice]ᵀ on MFMA (key on the register, query on the lane),
//   * the four partial Sᵀ are summed through LDS (fixed order, so every wave holds the same
//     bits and runs the same online softmax),
//   * Õᵀ_w += latent[:, slice]ᵀ·Pᵀ with the latent tile read transposed (ds_read_b64_tr_b16).
// MFMA work is not duplicated; the cost is the partial-S exchange (16 KiB of LDS per tile).
// Latent tiles of 32 keys are register-staged into a double-buffered [32][LAT] LDS image.
// Softmax semantics are the reference forward's (AttentionKernel+Softmax.swift:641-892):
// base-2 online softmax, masked keys at (0.875/log2 e)·(−FLT_MAX) (causal) or −inf (past S_kv),
// L = m + log2 l.  Õ is written in the 16-bit element type for the final 16-bit GEMM.
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

template <class E, int LAT>
__global__ void __launch_bounds__(256, 2) mfa_mla_latent_kernel(LatentParams p) {
  constexpr int BK = 32, NT = 256;
  constexpr int WS = LAT / 4;              // latent dims per wave
  constexpr int DS = WS / 16;              // MFMA k-steps of the wave's QK^T slice
  constexpr int ND = WS / 32;              // O^T tiles per wave
  constexpr int CPR = LAT / 8;             // 16-byte chunks per latent row
  constexpr int CPT = BK * CPR / NT;       // chunks staged per thread
  constexpr int TILEB = BK * LAT * 2;
  constexpr int XST = 16;                  // floats per lane in the exchange area
  using A = Arith16<E, LAT>;
  using TT = Tile16<LAT>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const tb0 = smem;                              // 2 latent tiles
  float* const xb = reinterpret_cast<float*>(smem + 2 * TILEB);  // [4 waves][64 lanes][XST]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int split = blockIdx.x % p.nsplit;
  const int bq = blockIdx.x / p.nsplit;
  const int b = bq / p.nblk;
  const int r0 = (bq % p.nblk) * 32;
  const int r = r0 + l32;
  const bool rvalid = r < p.R;
  const int spos = rvalid ? r % p.Sq : 0;   // query position of the row (causal)

  // Keys this block needs: all of S_kv, or up to the largest query position it holds.
  int kend = p.Skv;
  if (p.causal) {
    const int rl = min(r0 + 31, p.R - 1);
    const int smax = (r0 / p.Sq == rl / p.Sq) ? rl % p.Sq : p.Sq - 1;
    kend = min(kend, smax + 1);
  }
  const int kbeg = split * p.chunk;
  kend = min(kend, kbeg + p.chunk);

  // Q̃ fragments of the wave's slice: d = w·WS + 16·ds + 8·hh + j.
  i16x8 qf[DS];
  {
    const uint16_t* qrow = (const uint16_t*)p.q + ((int64_t)b * p.R + (rvalid ? r : 0)) * LAT;
#pragma unroll
    for (int ds = 0; ds < DS; ++ds) {
      i16x8 v = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (rvalid) v = *reinterpret_cast<const i16x8*>(qrow + wave * WS + 16 * ds + 8 * hh);
      qf[ds] = v;
    }
  }

  const uint16_t* lat = (const uint16_t*)p.lat + (int64_t)b * p.Skv * LAT;
  uint4 stg[CPT];
  auto load = [&](int t) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int id = tid + NT * i;
      const int row = id / CPR, ch = id % CPR;
      stg[i] = (t + row < p.Skv)
                   ? *reinterpret_cast<const uint4*>(lat + (int64_t)(t + row) * LAT + 8 * ch)
                   : make_uint4(0u, 0u, 0u, 0u);
    }
  };
  auto store = [&](char* tile) {
#pragma unroll
    for (int i = 0; i < CPT; ++i) {
      const int id = tid + NT * i;
      *reinterpret_cast<uint4*>(tile + TT::off(id / CPR, id % CPR)) = stg[i];
    }
  };

  f32x16 o[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) o[dt] = zero16();
  float m = -kFltMax, lh = 0.f;
  const float c = p.c_log2;

  if (kbeg < kend) {
    load(kbeg);
    store(tb0);
  }
  __syncthreads();
  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool has_next = t + BK < kend;
    if (has_next) load(t + BK);
    const char* kt = tb0 + cur * TILEB;

    // Partial S^T over this wave's latent slice.
    f32x16 sp = zero16();
#pragma unroll
    for (int ds = 0; ds < DS; ++ds)
      sp = A::mma(A::read_row(kt, l32, wave * DS + ds, hh), qf[ds], sp);
    // Exchange: each lane's 16 partial values contiguous ([wave][lane][16 floats]); the four
    // 16-byte chunks are rotated by (lane >> 2) & 3 so the lanes of a ds_read_b128 group hit
    // distinct banks.
    const int xsw = (lane >> 2) & 3;
    {
      float* dst = xb + (wave * 64 + lane) * XST;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<f32x4*>(dst + 4 * (q ^ xsw)) =
            f32x4{sp[4 * q], sp[4 * q + 1], sp[4 * q + 2], sp[4 * q + 3]};
    }
    __syncthreads();
    f32x16 s;
    {
      f32x4 part[4][4];
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          part[w][q] = *reinterpret_cast<const f32x4*>(xb + (w * 64 + lane) * XST + 4 * (q ^ xsw));
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          s[4 * q + e] = ((part[0][q][e] + part[1][q][e]) + part[2][q][e]) + part[3][q][e];
    }

    if (t + BK > p.Skv || (p.causal && t + BK - 1 > spos)) {
      MFA_KEEP_BRANCH();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = t + acc_row(i, hh);
        if (p.causal && key > spos) s[i] = kMaskValue;
        if (key >= p.Skv) s[i] = -__builtin_inff();
      }
    }
    float mx = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[i]);
    const float m_tile = cross_half_max(mx) * c;
    if (m_tile > m) {
      const float corr = __builtin_amdgcn_exp2f(m - m_tile);
      m = m_tile;
      lh *= corr;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= corr;
    }
    float rs = 0.f;
    if (m < kMaskLevel) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = __builtin_amdgcn_exp2f(mul_rn(s[i], c) - m);
        rs += s[i];
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(s[i], c, -m));
        rs += s[i];
      }
    }
    lh += rs;
    // O^T += latent[:, slice]^T · P^T
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const i16x8 pb = A::pack(s, ks);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
        o[dt] = A::mma(A::read_tr(kt, 0, ks, wave * WS + 32 * dt, lane), pb, o[dt]);
    }
    if (has_next) store(tb0 + (cur ^ 1) * TILEB);
    __syncthreads();
    cur ^= 1;
  }

  if (p.nsplit > 1) {
    // Partial state of this key split: Õ unnormalised, (m, l) for the merge pass.
    const float lp = cross_half_sum(lh);
    if (!rvalid) return;
    const int64_t prow = ((int64_t)b * p.nsplit + split) * p.R + r;
    float* op = p.opart + prow * LAT + wave * WS;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(op + dt * 32 + 8 * g + 4 * hh) =
            make_float4(o[dt][4 * g], o[dt][4 * g + 1], o[dt][4 * g + 2], o[dt][4 * g + 3]);
    if (wave == 0 && hh == 0) p.mlpart[prow] = make_float2(m, lp);
    return;
  }
  float l = cross_half_sum(lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if (!rvalid) return;
  const float inv = 1.f / l;
  uint16_t* orow = (uint16_t*)p.olat + ((int64_t)b * p.R + r) * LAT + wave * WS;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = dt * 32 + 8 * g + 4 * hh;
      ushort4 v;
      v.x = E::from_f32(o[dt][4 * g] * inv);
      v.y = E::from_f32(o[dt][4 * g + 1] * inv);
      v.z = E::from_f32(o[dt][4 * g + 2] * inv);
      v.w = E::from_f32(o[dt][4 * g + 3] * inv);
      *reinterpret_cast<ushort4*>(orow + d) = v;
    }
  if (wave == 0 && hh == 0 && p.l) {
    const float L = m + __log2f(l);
    const int64_t li = (int64_t)b * p.R + r;
    if (p.l_f16)
      reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
    else
      reinterpret_cast<float*>(p.l)[li] = L;
  }
}

// Merge of the key splits (flash-decoding): M = max m_s, w_s = exp2(m_s − M),
// Õ = Σ w_s Õ_s / Σ w_s l_s, L = M + log2 Σ w_s l_s.  MNB rows (the same query row r of MNB
// consecutive batch items) per 256-thread workgroup, launched with MNB = 1.  The split states
// are combined per row into an FP32 Õ row image in LDS; with W_v, the projection then reads
// each W_v element once for the workgroup's rows, the latent dimension split over 16 k groups.
constexpr int MNT = 256;

template <class E, int LAT, int MNB>
__global__ void __launch_bounds__(MNT) mfa_mla_latent_merge_kernel(LatentParams p) {
  constexpr int TPR = LAT / 4;        // threads per row in the combine step (4 dims each)
  constexpr int RPI = MNT / TPR;      // rows combined per iteration
  // Õ rows [MNB][LAT], then (projection) 16 k groups' partial sums [16][MNB][128].
  __shared__ __attribute__((aligned(16))) float smf[MNB * LAT + 16 * MNB * 128];
  float (*orow)[LAT] = reinterpret_cast<float (*)[LAT]>(smf);
  const int r = blockIdx.x % p.R;
  const int b0 = (blockIdx.x / p.R) * MNB;
  const int tid = threadIdx.x;
  const int d = 4 * (tid % TPR);
  for (int nb = tid / TPR; nb < MNB; nb += RPI) {
    const int b = b0 + nb;
    if (b >= p.B) break;
    // SU splits' loads in flight at a time (a one-split-at-a-time loop is a chain of HBM
    // latencies), merged online: running max M, rescaled sum l and Õ accumulator.
    constexpr int SU = 16;
    float M = -kFltMax;
    float l = 0.f;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int s0 = 0; s0 < p.nsplit; s0 += SU) {
      float2 ml[SU];
      float4 x[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        ml[u] = make_float2(-kFltMax, 0.f);
        x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (s0 + u < p.nsplit) {
          const int64_t prow = ((int64_t)b * p.nsplit + s0 + u) * p.R + r;
          ml[u] = p.mlpart[prow];
          x[u] = *reinterpret_cast<const float4*>(p.opart + prow * LAT + d);
        }
      }
      float Mc = M;
#pragma unroll
      for (int u = 0; u < SU; ++u) Mc = fmaxf(Mc, ml[u].x);
      const float cr = __builtin_amdgcn_exp2f(M - Mc);
      M = Mc;
      l *= cr;
      acc.x *= cr; acc.y *= cr; acc.z *= cr; acc.w *= cr;
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const float w = __builtin_amdgcn_exp2f(ml[u].x - M);
        l += w * ml[u].y;
        acc.x += w * x[u].x; acc.y += w * x[u].y; acc.z += w * x[u].z; acc.w += w * x[u].w;
      }
    }
    l += kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    const float inv = 1.f / l;
    const int64_t row = (int64_t)b * p.R + r;
    if (p.wv) {
      *reinterpret_cast<float4*>(&orow[nb][d]) =
          make_float4(acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv);
    } else {
      ushort4 v;
      v.x = E::from_f32(acc.x * inv);
      v.y = E::from_f32(acc.y * inv);
      v.z = E::from_f32(acc.z * inv);
      v.w = E::from_f32(acc.w * inv);
      *reinterpret_cast<ushort4*>((uint16_t*)p.olat + row * LAT + d) = v;
    }
    if (d == 0 && p.l) {
      const float L = M + __log2f(l);
      if (p.l_f16)
        reinterpret_cast<uint16_t*>(p.l)[row] = f32_to_f16(L);
      else
        reinterpret_cast<float*>(p.l)[row] = L;
    }
  }
  if (!p.wv) return;
  __syncthreads();
  // Fused output projection O[b, r, :] = Õ[b, r, :]·W_v[:, h·D : (h+1)·D], per 128-dim chunk:
  // lane group dg (16 lanes) x k group kg (16 per workgroup) — each thread loads 8 consecutive
  // W_v dims (16 B) for LAT/16 latent rows, all loads independent, and keeps 8 x MNB partial
  // sums; the 16 k groups are summed through LDS.
  const int nbv = min(MNB, p.B - b0);
  const int hq = r / p.Sq;
  const uint16_t* w = (const uint16_t*)p.wv + (int64_t)hq * p.D;
  const int64_t ldw = (int64_t)p.H * p.D;
  const bool vec = (p.D % 8) == 0 && (ldw % 8) == 0 && ((uintptr_t)p.wv % 16) == 0;
  const int dg = tid & 15, kg = tid >> 4;
  constexpr int KPG = LAT / 16;
  float* red = smf + MNB * LAT;  // [16 k groups][MNB][128]
  for (int dd0 = 0; dd0 < p.D; dd0 += 128) {
    float acc[MNB][8];
#pragma unroll
    for (int nb = 0; nb < MNB; ++nb)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[nb][j] = 0.f;
    const int dd = dd0 + 8 * dg;
    if (dd < p.D) {
#pragma unroll 16
      for (int kk = 0; kk < KPG; ++kk) {
        const int k = kg * KPG + kk;
        const uint16_t* wr = w + (int64_t)k * ldw + dd;
        float wf[8];
        if (vec) {
          const i16x8 w8 = *reinterpret_cast<const i16x8*>(wr);
#pragma unroll
          for (int j = 0; j < 8; ++j) wf[j] = E::to_f32((uint16_t)w8[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) wf[j] = dd + j < p.D ? E::to_f32(wr[j]) : 0.f;
        }
#pragma unroll
        for (int nb = 0; nb < MNB; ++nb) {
          const float o = orow[nb][k];
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[nb][j] = __builtin_fmaf(o, wf[j], acc[nb][j]);
        }
      }
    }
#pragma unroll
    for (int nb = 0; nb < MNB; ++nb)
#pragma unroll
      for (int j = 0; j < 8; j += 4)
        *reinterpret_cast<float4*>(red + (kg * MNB + nb) * 128 + 8 * dg + j) =
            make_float4(acc[nb][j], acc[nb][j + 1], acc[nb][j + 2], acc[nb][j + 3]);
    __syncthreads();
    for (int o = tid; o < MNB * 128; o += MNT) {
      const int nb = o >> 7, dl = o & 127;
      if (nb < nbv && dd0 + dl < p.D) {
        float sum = 0.f;
#pragma unroll
        for (int g2 = 0; g2 < 16; ++g2) sum += red[(g2 * MNB + nb) * 128 + dl];
        p.out[((int64_t)(b0 + nb) * p.R + r) * p.D + dd0 + dl] = sum;
      }
    }
    __syncthreads();
  }
}

template <class E, int LAT>
static hipError_t launch_latent(const LatentParams& p, hipStream_t stream) {
  constexpr int LDS = 2 * 32 * LAT * 2 + 4 * 64 * 16 * 4;
  auto kern = mfa_mla_latent_kernel<E, LAT>;
  hipError_t e = launch(kern, dim3(p.nblk * p.B * p.nsplit), dim3(256), LDS, stream, p);
  if (e != hipSuccess || p.nsplit <= 1) return e;
  // One row per workgroup measured fastest (B32 S_q 1: MNB 1/2/4 = 14.5/15.6/17.9 us): the
  // W_v re-reads per batch item come from L2.
  return launch(mfa_mla_latent_merge_kernel<E, LAT, 1>, dim3(p.B * p.R), dim3(MNT), 0, stream, p);
}

// Decode query projection Q̃[b, h, :] = q[b, h, :] · W_k[:, h·D : (h+1)·D]ᵀ (S_q = 1): a workgroup
// takes one head, QC latent columns and 32 batch rows; the W_k slice [QC][D] and the query rows
// [32][D] sit in LDS (rows padded by 16 B), each thread accumulates QC/8 columns of one row in
// FP32 over D.  Replaces a 128x128-tile GEMM launch whose 64 workgroups were mostly padding
// (M = B rows per head).
constexpr int QC = 16;
template <class E>
__global__ void __launch_bounds__(256) mfa_mla_qproj_kernel(const uint16_t* __restrict__ q,
                                                            const uint16_t* __restrict__ wk,
                                                            uint16_t* __restrict__ qt, int B,
                                                            int H, int D, int Lat) {
  constexpr int NJ = QC / 8;  // columns per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int RS = D * 2 + 16;  // padded row stride (bytes)
  char* const wsl = smem;            // [QC][RS]
  char* const qsl = smem + QC * RS;  // [32][RS]
  const int h = blockIdx.x, l0 = blockIdx.y * QC, b0 = blockIdx.z * 32;
  const int tid = threadIdx.x;
  const int cpr = D / 8;  // 16-byte chunks per row
  for (int i = tid; i < QC * cpr; i += 256) {
    const int r = i / cpr, c = i % cpr;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (l0 + r < Lat)
      v = *reinterpret_cast<const uint4*>(wk + (int64_t)(l0 + r) * H * D + (int64_t)h * D + 8 * c);
    *reinterpret_cast<uint4*>(wsl + r * RS + 16 * c) = v;
  }
  for (int i = tid; i < 32 * cpr; i += 256) {
    const int r = i / cpr, c = i % cpr;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (b0 + r < B) v = *reinterpret_cast<const uint4*>(q + ((int64_t)(b0 + r) * H + h) * D + 8 * c);
    *reinterpret_cast<uint4*>(qsl + r * RS + 16 * c) = v;
  }
  __syncthreads();
  const int br = tid >> 3, lg = tid & 7;
  float acc[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) acc[j] = 0.f;
  for (int c = 0; c < cpr; ++c) {
    const uint4 qv = *reinterpret_cast<const uint4*>(qsl + br * RS + 16 * c);
    float qf[8];
    const uint32_t qw[4] = {qv.x, qv.y, qv.z, qv.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      qf[2 * e] = E::to_f32((uint16_t)(qw[e] & 0xffffu));
      qf[2 * e + 1] = E::to_f32((uint16_t)(qw[e] >> 16));
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const uint4 wv = *reinterpret_cast<const uint4*>(wsl + (lg * NJ + j) * RS + 16 * c);
      const uint32_t ww[4] = {wv.x, wv.y, wv.z, wv.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[j] = __builtin_fmaf(qf[2 * e], E::to_f32((uint16_t)(ww[e] & 0xffffu)), acc[j]);
        acc[j] = __builtin_fmaf(qf[2 * e + 1], E::to_f32((uint16_t)(ww[e] >> 16)), acc[j]);
      }
    }
  }
  const int b = b0 + br;
  if (b >= B) return;
  uint16_t* orow = qt + ((int64_t)b * H + h) * Lat + l0 + lg * NJ;
#pragma unroll
  for (int j = 0; j < NJ; ++j)
    if (l0 + lg * NJ + j < Lat) orow[j] = E::from_f32(acc[j]);
}

hipError_t mla_qproj_dispatch(const void* q, const void* wk, void* qt, int B, int H, int D,
                              int Lat, int elem, hipStream_t stream) {
  if (D % 8 != 0 || D > 256 || ((uintptr_t)q & 15) || ((uintptr_t)wk & 15))
    return hipErrorNotSupported;
  const dim3 grid(H, (Lat + QC - 1) / QC, (B + 31) / 32);
  const size_t lds = (size_t)(QC + 32) * (D * 2 + 16);
  if (elem == P_FP16)
    hipLaunchKernelGGL(mfa_mla_qproj_kernel<F16>, grid, dim3(256), lds, stream,
                       (const uint16_t*)q, (const uint16_t*)wk, (uint16_t*)qt, B, H, D, Lat);
  else if (elem == P_BF16)
    hipLaunchKernelGGL(mfa_mla_qproj_kernel<BF16>, grid, dim3(256), lds, stream,
                       (const uint16_t*)q, (const uint16_t*)wk, (uint16_t*)qt, B, H, D, Lat);
  else
    return hipErrorNotSupported;
  return hipGetLastError();
}

hipError_t mla_latent_dispatch(const LatentParams& p, int elem, int lat, hipStream_t stream) {
  if (lat == 512 && elem == P_FP16) return launch_latent<F16, 512>(p, stream);
  if (lat == 512 && elem == P_BF16) return launch_latent<BF16, 512>(p, stream);
  if (lat == 256 && elem == P_FP16) return launch_latent<F16, 256>(p, stream);
  if (lat == 256 && elem == P_BF16) return launch_latent<BF16, 256>(p, stream);
  return hipErrorNotSupported;
}

template __global__ void mfa_mla_latent_kernel<F16, 512>(LatentParams);
template __global__ void mfa_mla_latent_merge_kernel<F16, 512, 1>(LatentParams);
template __global__ void mfa_mla_latent_merge_kernel<BF16, 512, 1>(LatentParams);
template __global__ void mfa_mla_latent_merge_kernel<F16, 256, 1>(LatentParams);
template __global__ void mfa_mla_latent_merge_kernel<BF16, 256, 1>(LatentParams);
template __global__ void mfa_mla_latent_kernel<BF16, 512>(LatentParams);
template __global__ void mfa_mla_latent_kernel<F16, 256>(LatentParams);
template __global__ void mfa_mla_latent_kernel<BF16, 256>(LatentParams);

}  // namespace mfa
