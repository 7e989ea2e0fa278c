// gemm_general.hip — the general GEMMDescriptor surface (GEMMDescriptor.swift:11-47,
// GEMMKernel+Source.swift:9-85): C[M,N] = op(A)·op(B) (+ C when loadPreviousC), with
//   * A, B, C memory precisions chosen independently from FP32 / FP16 / BF16
//     (GEMMOperandPrecision.swift), C rounded once at the store;
//   * transposeState: A stored [K][M] when transposed (leading dimension ≥ M), B stored
//     [N][K] when transposed (leading dimension ≥ K), GEMMDescriptor.swift:344-372;
//   * any leading dimensions, batch (grid z) with element strides.
// The NN 16-bit case with equal A/B precisions goes to the tuned kernels in gemm.hip; this
// file covers everything else.
//
// Arithmetic (gfx950 register-precision policy, reported by mfa_gemm_kernel_descriptor):
//   * A and B both FP16 (or both BF16): v_mfma_f32_32x32x16_{f16,bf16}, FP32 accumulation.
//     The reference accumulates FP16 x FP16 -> FP16 in FP16 registers
//     (GEMMDescriptor.swift:204-210); accumulating in FP32 is strictly more accurate.
//   * every other combination: operands converted to FP32 on their way into LDS and
//     multiplied on the exact FP32 matrix core (v_mfma_f32_32x32x2_f32), as the reference's
//     FP32 register precision does for mixed inputs.
//
// Tiling: 128x128 outputs per workgroup of 4 waves (2x2, 64x64 per wave = 2x2 MFMA tiles).
// A k-contiguous operand (A untransposed, B transposed) sits in LDS as [128 rows][64 bytes]
// (32 16-bit or 16 FP32 values of k per row), 16-byte chunks XOR-swizzled by (row >> 2) & 3.
// A 16-bit m/n-contiguous operand keeps its memory layout ([32 k][128], Tile16<128>) and is
// read with the transposing LDS read (see the LAY parameter); an FP32 one is written to the
// k-contiguous image element by element.  Register-staged double buffering: the next
// k-step's chunks are loaded from HBM while the current one is multiplied.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mfa/mfa.h"
#include "mfa_device.h"
#include "mfa_params.h"
#include "mfa_dispatch.h"
#include <type_traits>

namespace mfa {

namespace {

constexpr int GBM = 128, GBN = 128;   // output tile
constexpr int GROWB = 64;             // bytes of k per LDS row
constexpr int GTILE = 128 * GROWB;    // 8 KiB per operand tile

__device__ __forceinline__ int goff(int r, int ch) { return r * GROWB + 16 * (ch ^ ((r >> 2) & 3)); }

__device__ __forceinline__ float load_elem(const char* base, int prec, int64_t i) {
  if (prec == P_FP32) return reinterpret_cast<const float*>(base)[i];
  const uint16_t b = reinterpret_cast<const uint16_t*>(base)[i];
  return prec == P_FP16 ? f16_to_f32(b) : bf16_to_f32(b);
}

}  // namespace

// CT: compute type — P_FP16 / P_BF16 (16-bit MFMA, A and B in that precision) or P_FP32.
// LAY (16-bit only): bit 0 = A is m-contiguous (transposed), bit 1 = B is n-contiguous
// (untransposed).  A 16-bit m/n-contiguous operand keeps its memory layout in LDS
// ([32 k][128 m/n], Tile16<128>) and is read with ds_read_b64_tr_b16; the k-contiguous
// operand is then read in the same permuted k order (two 8-byte reads), as gemm.hip does.
template <int CT, int LAY = 0>
__global__ void __launch_bounds__(256) mfa_gemm_general_kernel(GemmGParams p) {
  constexpr bool F32 = CT == P_FP32;
  constexpr int KT = F32 ? 16 : 32;                 // k per LDS tile
  constexpr int CPT = F32 ? 1 : 2;                  // 8-element chunks per thread per operand
  __shared__ __attribute__((aligned(16))) char smem[4 * GTILE];
  char* const abuf = smem;
  char* const bbuf = smem + 2 * GTILE;

  const int z = blockIdx.z;
  const char* A = (const char*)p.a + (int64_t)z * p.sa * p.esz_a;
  const char* B = (const char*)p.b + (int64_t)(p.bmod ? z % p.bmod : z) * p.sb * p.esz_b;
  char* C = (char*)p.c + (int64_t)z * p.sc * p.esz_c;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;

  // Operand view: rows along m (A) or n (B); `kc` = memory is k-contiguous.
  struct Op {
    const char* base;
    int prec, esz, ld, rows, r0;
    bool kc;
  };
  const Op opa{A, p.prec_a, p.esz_a, p.lda, p.M, m0, !p.trans_a};
  const Op opb{B, p.prec_b, p.esz_b, p.ldb, p.N, n0, (bool)p.trans_b};

  // Staged chunk values: 16-bit raw bits, or FP32.
  uint4 ra[CPT], rb[CPT];
  float fa[8], fb[8];

  // Element (row, k) of an operand lives at row*ld + k (k-contiguous) or k*ld + row.
  auto chunk_coords = [&](const Op& o, int id, int k0, int* row, int* k) {
    if (o.kc) {
      *row = id / (KT / 8);
      *k = k0 + (id % (KT / 8)) * 8;
    } else {
      *row = (id % 16) * 8;
      *k = k0 + id / 16;
    }
  };
  auto load16 = [&](const Op& o, int id, int k0) -> uint4 {
    int row, k;
    chunk_coords(o, id, k0, &row, &k);
    const int gr = o.r0 + row;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    // The chunk's 8 elements are consecutive in memory along k (kc) or along m/n.
    const uint16_t* src;
    int nvalid;
    if (o.kc) {
      if (gr >= o.rows) return v;
      src = (const uint16_t*)o.base + (int64_t)gr * o.ld + k;
      nvalid = p.K - k;
    } else {
      if (k >= p.K) return v;
      src = (const uint16_t*)o.base + (int64_t)k * o.ld + gr;
      nvalid = o.rows - gr;
    }
    if (nvalid >= 8 && (((uintptr_t)src) & 15) == 0) return *reinterpret_cast<const uint4*>(src);
    uint32_t w[4] = {0u, 0u, 0u, 0u};
    for (int j = 0; j < 8; ++j)
      if (j < nvalid) w[j >> 1] |= (uint32_t)src[j] << (16 * (j & 1));
    return make_uint4(w[0], w[1], w[2], w[3]);
  };
  auto loadf = [&](const Op& o, int id, int k0, float (&v)[8]) {
    int row, k;
    chunk_coords(o, id, k0, &row, &k);
    const int gr = o.r0 + row;
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = 0.f;
    int64_t first;
    int nvalid;
    if (o.kc) {
      if (gr >= o.rows) return;
      first = (int64_t)gr * o.ld + k;
      nvalid = p.K - k;
    } else {
      if (k >= p.K) return;
      first = (int64_t)k * o.ld + gr;
      nvalid = o.rows - gr;
    }
    if (nvalid > 8) nvalid = 8;
    if (o.prec == P_FP32 && nvalid == 8 && ((((uintptr_t)o.base) + first * 4) & 15) == 0) {
      const float4 x = *reinterpret_cast<const float4*>((const float*)o.base + first);
      const float4 y = *reinterpret_cast<const float4*>((const float*)o.base + first + 4);
      v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
      v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
      return;
    }
    for (int j = 0; j < 8; ++j)
      if (j < nvalid) v[j] = load_elem(o.base, o.prec, first + j);
  };
  auto load = [&](int k0) {
    if constexpr (F32) {
      loadf(opa, tid, k0, fa);
      loadf(opb, tid, k0, fb);
    } else {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        ra[i] = load16(opa, tid + 256 * i, k0);
        rb[i] = load16(opb, tid + 256 * i, k0);
      }
    }
  };
  auto store16 = [&](const Op& o, char* tile, int id, uint4 v) {
    int row, k;
    chunk_coords(o, id, 0, &row, &k);
    if constexpr (LAY != 0) {
      if (!o.kc) {  // memory layout kept: [k][128 m/n]
        *reinterpret_cast<uint4*>(tile + Tile16<128>::off(k, row / 8)) = v;
        return;
      }
    }
    if (o.kc) {
      *reinterpret_cast<uint4*>(tile + goff(row, k / 8)) = v;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<uint16_t*>(tile + goff(row + j, k / 8) + 2 * (k % 8)) =
            (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
    }
  };
  auto storef = [&](const Op& o, char* tile, int id, const float (&v)[8]) {
    int row, k;
    chunk_coords(o, id, 0, &row, &k);
    if (o.kc) {
      *reinterpret_cast<float4*>(tile + goff(row, k / 4)) = make_float4(v[0], v[1], v[2], v[3]);
      *reinterpret_cast<float4*>(tile + goff(row, k / 4 + 1)) =
          make_float4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        *reinterpret_cast<float*>(tile + goff(row + j, k / 4) + 4 * (k % 4)) = v[j];
    }
  };
  auto store = [&](int buf) {
    if constexpr (F32) {
      storef(opa, abuf + buf * GTILE, tid, fa);
      storef(opb, bbuf + buf * GTILE, tid, fb);
    } else {
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        store16(opa, abuf + buf * GTILE, tid + 256 * i, ra[i]);
        store16(opb, bbuf + buf * GTILE, tid + 256 * i, rb[i]);
      }
    }
  };

  f32x16 acc[2][2];
  if (p.load_prev) {
    // loadPreviousC (GEMMKernel+Caching.swift): the accumulators start from C.
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = n0 + wn * 64 + j * 32 + l32;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + wm * 64 + i * 32 + acc_row(r, hh);
          acc[i][j][r] = (m < p.M && n < p.N) ? load_elem(C, p.prec_c, (int64_t)m * p.ldc + n) : 0.f;
        }
      }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = zero16();
  }

  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < p.K; k0 += KT) {
    const bool has_next = k0 + KT < p.K;
    if (has_next) load(k0 + KT);
    const char* at = abuf + cur * GTILE;
    const char* bt = bbuf + cur * GTILE;
    if constexpr (F32) {
      // k-step s covers k = 4(s>>1) + 2hh + (s&1): one 8-byte read serves two steps.
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float2 af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const float2*>(at + goff(wm * 64 + i * 32 + l32, q) + 8 * hh);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[j] = *reinterpret_cast<const float2*>(bt + goff(wn * 64 + j * 32 + l32, q) + 8 * hh);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) {
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].x, bf[j].x, acc[i][j], 0, 0, 0);
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(af[i].y, bf[j].y, acc[i][j], 0, 0, 0);
          }
      }
    } else {
      using E = typename std::conditional<CT == P_FP16, F16, BF16>::type;
      using AT = Arith16<E, 128>;
      // k-contiguous operand read: standard k order, or the transposed reads' order.
      auto kc_read = [&](const char* t, int r, int s) -> i16x8 {
        if constexpr (LAY == 0) {
          return *reinterpret_cast<const i16x8*>(t + goff(r, 2 * s + hh));
        } else {
          const uint2 lo = *reinterpret_cast<const uint2*>(t + goff(r, 2 * s) + 8 * hh);
          const uint2 hi = *reinterpret_cast<const uint2*>(t + goff(r, 2 * s + 1) + 8 * hh);
          return __builtin_bit_cast(i16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
        }
      };
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        i16x8 af[2], bf[2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = (LAY & 1) ? AT::read_tr(at, 0, s, wm * 64 + i * 32, lane)
                            : kc_read(at, wm * 64 + i * 32 + l32, s);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[j] = (LAY & 2) ? AT::read_tr(bt, 0, s, wn * 64 + j * 32, lane)
                            : kc_read(bt, wn * 64 + j * 32 + l32, s);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = E::mma(af[i], bf[j], acc[i][j]);
      }
    }
    if (has_next) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // acc[i][j]: column n = lane, rows m = acc_row(r, hh).
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + wn * 64 + j * 32 + l32;
      if (n >= p.N) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + acc_row(r, hh);
        if (m >= p.M) continue;
        const int64_t ci = (int64_t)m * p.ldc + n;
        const float x = acc[i][j][r];
        if (p.prec_c == P_FP32)
          reinterpret_cast<float*>(C)[ci] = x;
        else
          reinterpret_cast<uint16_t*>(C)[ci] = p.prec_c == P_FP16 ? f32_to_f16(x) : f32_to_bf16(x);
      }
    }
}

int gemm_general_compute(int prec_a, int prec_b) {
  if (prec_a == prec_b && (prec_a == P_FP16 || prec_a == P_BF16)) return prec_a;
  return P_FP32;
}

hipError_t gemm_general_dispatch(const GemmGParams& p, int batch, hipStream_t stream) {
  const dim3 grid((p.N + GBN - 1) / GBN, (p.M + GBM - 1) / GBM, batch);
  const int lay = (p.trans_a ? 1 : 0) | (p.trans_b ? 0 : 2);
#define MFA_GG(CTV, L)                                                                      \
  case L: {                                                                                 \
    auto k = mfa_gemm_general_kernel<CTV, L>;                                               \
    hipLaunchKernelGGL(k, grid, dim3(256), 0, stream, p);                                   \
    break;                                                                                  \
  }
  switch (gemm_general_compute(p.prec_a, p.prec_b)) {
    case P_FP16:
      switch (lay) { MFA_GG(P_FP16, 0) MFA_GG(P_FP16, 1) MFA_GG(P_FP16, 2) MFA_GG(P_FP16, 3) }
      break;
    case P_BF16:
      switch (lay) { MFA_GG(P_BF16, 0) MFA_GG(P_BF16, 1) MFA_GG(P_BF16, 2) MFA_GG(P_BF16, 3) }
      break;
#undef MFA_GG
    default:
      hipLaunchKernelGGL(mfa_gemm_general_kernel<P_FP32>, grid, dim3(256), 0, stream, p);
      break;
  }
  return hipGetLastError();
}

#define MFA_GG_INST(CTV)                                                   \
  template __global__ void mfa_gemm_general_kernel<CTV, 0>(GemmGParams); \
  template __global__ void mfa_gemm_general_kernel<CTV, 1>(GemmGParams); \
  template __global__ void mfa_gemm_general_kernel<CTV, 2>(GemmGParams); \
  template __global__ void mfa_gemm_general_kernel<CTV, 3>(GemmGParams);
MFA_GG_INST(P_FP16)
MFA_GG_INST(P_BF16)
#undef MFA_GG_INST
template __global__ void mfa_gemm_general_kernel<P_FP32>(GemmGParams);

}  // namespace mfa
