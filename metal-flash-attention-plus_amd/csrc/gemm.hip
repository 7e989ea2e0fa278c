// gemm.hip — C[M,N] = A[M,K]·B[K,N] (+ C) on MFMA, the GEMM the reference uses on the hot path
// only for MLA decompression (MLAOptimizedGEMMMFA.swift:97-154: FP16 NN, K[B·S, H·D] =
// latent[B·S, 512]·W_k[512, H·D]).  The reference accumulates FP16xFP16 in FP16 registers
// (GEMMDescriptor.swift:204-210); here accumulation is FP32 and C is rounded once.
//
// Tiling: 128x128 output per workgroup of 4 waves (2x2, 64x64 per wave = 2x2 MFMA 32x32
// tiles), K staged 32 deep through double-buffered LDS.  B is row-major [K][N], so its MFMA
// operand (8 consecutive k of one column) is read with ds_read_b64_tr_b16; A is then read in
// the same permuted k order (two 8-byte reads per fragment) so the products pair up.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "../../include/mfa/mfa.h"
#include "mfa_device.h"
#include "mfa_params.h"
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

template <class E>
__global__ void __launch_bounds__(256) mfa_gemm_kernel(GemmParams p) {
  constexpr int BM = 128, BN = 128, BK = 32;
  using TA = Tile16<BK>;   // [BM][BK]
  using TB = Tile16<BN>;   // [BK][BN]
  using AB = Arith16<E, BN>;
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM * BK * 2 + BK * BN * 2)];
  char* const ab = smem;
  char* const bb = smem + 2 * BM * BK * 2;
  constexpr int ATILE = BM * BK * 2, BTILE = BK * BN * 2;

  const int z = blockIdx.z;
  const uint16_t* A = (const uint16_t*)p.a + (p.b[1] ? 0 : z * p.sa);
  const uint16_t* B = (const uint16_t*)(p.b[1] ? p.b[z] : p.b[0]) + (p.b[1] ? 0 : z * p.sb);
  char* C = (char*)(p.b[1] ? p.c[z] : p.c[0]);
  const int64_t coff = p.b[1] ? 0 : z * p.sc;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;

  // Each thread stages 2 A chunks and 2 B chunks (16 bytes = 8 elements each).
  uint4 ra[2], rb[2];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + i * 256;
      {  // A: 128 rows x 4 chunks
        const int r = id >> 2, c = id & 3;
        const int gm = m0 + r, gk = k0 + c * 8;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (gm < p.M) {
          const uint16_t* src = A + (int64_t)gm * p.lda + gk;
          if (gk + 8 <= p.K && ((((uintptr_t)src) & 15) == 0)) {
            v = *reinterpret_cast<const uint4*>(src);
          } else {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int j = 0; j < 8; ++j)
              if (gk + j < p.K) w[j >> 1] |= (uint32_t)src[j] << (16 * (j & 1));
            v = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
        ra[i] = v;
      }
      {  // B: 32 rows x 16 chunks
        const int r = id >> 4, c = id & 15;
        const int gk = k0 + r, gn = n0 + c * 8;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if (gk < p.K) {
          const uint16_t* src = B + (int64_t)gk * p.ldb + gn;
          if (gn + 8 <= p.N && ((((uintptr_t)src) & 15) == 0)) {
            v = *reinterpret_cast<const uint4*>(src);
          } else {
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int j = 0; j < 8; ++j)
              if (gn + j < p.N) w[j >> 1] |= (uint32_t)src[j] << (16 * (j & 1));
            v = make_uint4(w[0], w[1], w[2], w[3]);
          }
        }
        rb[i] = v;
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + i * 256;
      *reinterpret_cast<uint4*>(ab + buf * ATILE + TA::off(id >> 2, id & 3)) = ra[i];
      *reinterpret_cast<uint4*>(bb + buf * BTILE + TB::off(id >> 4, id & 15)) = rb[i];
    }
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    const bool has_next = k0 + BK < p.K;
    if (has_next) load(k0 + BK);
    const char* at = ab + cur * ATILE;
    const char* bt = bb + cur * BTILE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      i16x8 af[2], bf[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // A row (m), k = 16s + 8(j>>2) + 4h + (j&3): the order read_tr produces for B.
        const int r = wm * 64 + i * 32 + l32;
        const uint2 lo = *reinterpret_cast<const uint2*>(at + TA::off(r, 2 * s) + 8 * hh);
        const uint2 hi = *reinterpret_cast<const uint2*>(at + TA::off(r, 2 * s + 1) + 8 * hh);
        af[i] = __builtin_bit_cast(i16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) bf[j] = AB::read_tr(bt, 0, s, wn * 64 + j * 32, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = E::mma(af[i], bf[j], acc[i][j]);
    }
    if (has_next) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // acc[i][j]: column n = lane, rows m = acc_row(r, h).
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
        const int64_t ci = coff + (int64_t)m * p.ldc + n;
        float x = acc[i][j][r];
        if (p.prec_c == P_FP32) {
          float* cf = reinterpret_cast<float*>(C);
          cf[ci] = p.load_prev ? x + cf[ci] : x;
        } else {
          uint16_t* ch = reinterpret_cast<uint16_t*>(C);
          if (p.load_prev) x += (p.prec_c == P_FP16 ? f16_to_f32(ch[ci]) : bf16_to_f32(ch[ci]));
          ch[ci] = p.prec_c == P_FP16 ? f32_to_f16(x) : f32_to_bf16(x);
        }
      }
    }
}

// ---------------------------------------------------------------------------------------
// Tuned path for whole tiles: M % 128 == N % 128 == K % 64 == 0, 16-byte aligned rows, no
// load-previous (the MLA decompression shape: [B·S, 512] x [512, H·D]).
//   * computed transposed, D[n][m] = Σ_k B[k][n]·A[m][k]: the lane is m, the accumulator
//     registers run along n, so the epilogue stores 4 consecutive n per register group (8-byte
//     bf16 / 16-byte fp32 stores) instead of one element per store;
//   * A [128 m][64 k] and B [64 k][128 n] tiles land by LDS-DMA in the TileA image, double
//     buffered, one barrier per 64-deep k-step; B^T fragments by transposed reads, A fragments
//     in the matching k order as two 8-byte reads.
// LAY: 3 = NN (A by rows, B by transposed reads in the natural k order, TileA::tr_base_nat);
// 0 = NN with the permuted order of TileA::tr_base (A read as two 8-byte halves to match);
// 1 = NT (B stored [N][K]: its tile is a [128 n][64 k] image like A's, both operands read by
// rows); 2 = TN (A stored [K][M]: its tile is a [64 k][128 m] image like B's, both operands
// read transposed in the permuted k order).
template <class E, int LAY = 0>
__global__ void __launch_bounds__(256, 2) mfa_gemm2_kernel(GemmParams p) {
  constexpr int BM = 128, BN = 128, BK = 64;
  using TAa = TileA<BK>;   // A tile: 128 rows of 64 k (128 B)
  using TBb = TileA<BN>;   // B tile: 64 rows of 128 n (256 B)
  using AB = Arith16<E, BN>;
  constexpr int ATILE = BM * BK * 2, BTILE = BK * BN * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ab = smem;
  char* const bb = smem + 2 * ATILE;

  const int z = blockIdx.z;
  const char* A = (const char*)p.a + (p.b[1] ? 0 : z * p.sa * 2);
  const char* B = (const char*)(p.b[1] ? p.b[z] : p.b[0]) + (p.b[1] ? 0 : z * p.sb * 2);
  char* C = (char*)(p.b[1] ? p.c[z] : p.c[0]);
  const int64_t coff = p.b[1] ? 0 : z * p.sc;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int trb[2] = {TBb::tr_base(lane, 0), TBb::tr_base(lane, 1)};
  // A fragment in the k order of the transposed B read: element j of lane half h is
  // k = 16s + 8(j>>2) + 4h + (j&3), i.e. bytes 8h..8h+7 of chunks 2s and 2s+1 of row m.
  int abase[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) abase[c] = TAa::off(wm * 64 + l32, c) + 8 * hh;

  // Tile images: A [128 m][64 k] (NN, NT) or [64 k][128 m] (TN); B [64 k][128 n] (NN, TN) or
  // [128 n][64 k] (NT).  Same byte size either way.
  constexpr bool AK = LAY != 2, BKR = LAY == 1;  // A / B rows are k-contiguous (LAY 3 = NN)
  DmaA<AK ? BK : BM, AK ? BM : BK, 256> ad;
  DmaA<BKR ? BK : BN, BKR ? BN : BK, 256> bd;
  ad.init(p.lda * 2, AK ? BM : BK, (AK ? BK : BM) * 2, tid);
  bd.init(p.ldb * 2, BKR ? BN : BK, (BKR ? BK : BN) * 2, tid);
  const char* ahead = A + (AK ? (int64_t)m0 * p.lda * 2 : (int64_t)m0 * 2);
  const char* bhead = B + (BKR ? (int64_t)n0 * p.ldb * 2 : (int64_t)n0 * 2);
  const int64_t astep = AK ? 2 : (int64_t)p.lda * 2;   // bytes per k
  const int64_t bstep = BKR ? 2 : (int64_t)p.ldb * 2;
  const int rb[2] = {TAa::row_base(l32, hh, 0), TAa::row_base(l32, hh, 1)};
  const int trn[2] = {TBb::tr_base_nat(lane, 0), TBb::tr_base_nat(lane, 1)};

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  ad.issue(ahead, 0, ab);
  bd.issue(bhead, 0, bb);
  wait_vm();
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    if (k0 + BK < p.K) {
      ad.issue(ahead + (int64_t)(k0 + BK) * astep, 0, ab + (cur ^ 1) * ATILE);
      bd.issue(bhead + (int64_t)(k0 + BK) * bstep, 0, bb + (cur ^ 1) * BTILE);
    }
    const char* at = ab + cur * ATILE;
    const char* bt = bb + cur * BTILE;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      i16x8 af[2], bf[2];
      if constexpr (LAY == 3) {
        // NN, natural k order: A by 16-byte row reads, B by transposed reads whose lane halves
        // take rows 8h..8h+7 of the k-step (TileA::tr_base_nat).
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const i16x8*>(TAa::row_addr(at, rb, 2 * wm + i, s));
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = AB::read_tr_nat(bt, trn, 32 * (s >> 1), s & 1, wn * 64 + j * 32);
      } else if constexpr (LAY == 1) {
        // Both k-contiguous images: rows read in the natural k order (chunk 2s + hh).
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[i] = *reinterpret_cast<const i16x8*>(TAa::row_addr(at, rb, 2 * wm + i, s));
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[j] = *reinterpret_cast<const i16x8*>(TAa::row_addr(bt, rb, 2 * wn + j, s));
      } else {
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          if constexpr (LAY == 2) {
            af[i] = AB::read_tr_a(at, trb, 32 * (s >> 1), s & 1, wm * 64 + i * 32);
          } else {
            // rows wm*64 + 32i + l32: + 32 rows = 4 row blocks of TAa::RB; chunks 2s, 2s+1
            // live in column block s/2 (512 B) at chunk parities (2s)&3, (2s+1)&3.
            const int cb = 512 * ((2 * s) >> 2);
            const uint2 lo = *reinterpret_cast<const uint2*>(at + abase[(2 * s) & 3] + cb +
                                                             TAa::RB * 4 * i);
            const uint2 hi = *reinterpret_cast<const uint2*>(at + abase[(2 * s + 1) & 3] + cb +
                                                             TAa::RB * 4 * i);
            af[i] = __builtin_bit_cast(i16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
          }
        }
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bf[j] = AB::read_tr_a(bt, trb, 32 * (s >> 1), s & 1, wn * 64 + j * 32);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = E::mma(bf[j], af[i], acc[i][j]);
    }
    wait_vm();
    __syncthreads();
    cur ^= 1;
  }

  // acc[i][j][r] = C[m = m0 + wm*64 + 32i + l32][n = n0 + wn*64 + 32j + acc_row(r, hh)].
  if (p.c_img) {
    // 16-bit C: the waves write their quadrants into a [128 m][128 n] image (row pitch 272 B)
    // in the ring the loop has released, then the workgroup stores whole 256-B rows (16 lanes
    // per row) instead of one 8-B piece per row per lane.
    constexpr int CP = BN * 2 + 16;
    const bool f16c = p.prec_c == P_FP16;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16& a = acc[i][j];
          auto cv = [&](float x) -> uint32_t {
            return f16c ? (uint32_t)f32_to_f16(x) : (uint32_t)f32_to_bf16(x);
          };
          const uint32_t w0 = cv(a[4 * g]) | (cv(a[4 * g + 1]) << 16);
          const uint32_t w1 = cv(a[4 * g + 2]) | (cv(a[4 * g + 3]) << 16);
          const int row = wm * 64 + i * 32 + l32, col = wn * 64 + j * 32 + 8 * g + 4 * hh;
          *reinterpret_cast<uint2*>(smem + row * CP + col * 2) = make_uint2(w0, w1);
        }
    __syncthreads();
    const int c16 = tid & 15;
#pragma unroll
    for (int it = 0; it < BM / 16; ++it) {
      const int row = it * 16 + (tid >> 4);
      const uint4 v = *reinterpret_cast<const uint4*>(smem + row * CP + c16 * 16);
      *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(C) + coff +
                                (int64_t)(m0 + row) * p.ldc + n0 + c16 * 8) = v;
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 64 + i * 32 + l32;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 64 + j * 32 + 8 * g + 4 * hh;
        const int64_t ci = coff + (int64_t)m * p.ldc + n;
        const f32x16& a = acc[i][j];
        if (p.prec_c == P_FP32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + ci) =
              make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]);
        } else {
          // C's own 16-bit format (it may differ from the operands').
          auto cv = [&](float x) -> uint32_t {
            return p.prec_c == P_FP16 ? (uint32_t)f32_to_f16(x) : (uint32_t)f32_to_bf16(x);
          };
          const uint32_t w0 = cv(a[4 * g]) | (cv(a[4 * g + 1]) << 16);
          const uint32_t w1 = cv(a[4 * g + 2]) | (cv(a[4 * g + 3]) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + ci) = make_uint2(w0, w1);
        }
      }
  }
}

template <class E>
static hipError_t launch_gemm2(const GemmParams& p0, int batch, hipStream_t stream) {
  constexpr int LDS = 2 * (128 * 64 * 2) + 2 * (64 * 128 * 2);
  const dim3 grid(p0.N / 128, p0.M / 128, batch);
  // Whole-row C stores need 16-B aligned rows; MFA_GEMM_IMG=0 keeps the per-lane stores (A/B).
  GemmParams p = p0;
  const char* ie = mfa::dev_env("MFA_GEMM_IMG");
  auto al16 = [](const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; };
  p.c_img = p.prec_c != P_FP32 && (p.ldc & 7) == 0 && (p.b[1] || (p.sc & 7) == 0) &&
            al16(p.c[0]) && al16(p.c[1]) && !(ie && ie[0] == '0');
  if (p.trans_b) return launch(mfa_gemm2_kernel<E, 1>, grid, dim3(256), LDS, stream, p);
  if (p.trans_a) return launch(mfa_gemm2_kernel<E, 2>, grid, dim3(256), LDS, stream, p);
  // NN in the natural k order (4096^3 fp16: 856-959 vs 745-749 TF for the permuted order;
  // C4 151.3 vs 153.1 us).  MFA_GEMM_NN=0 keeps the permuted-order kernel (A/B).
  const char* nn = mfa::dev_env("MFA_GEMM_NN");
  if (nn && nn[0] == '0') return launch(mfa_gemm2_kernel<E, 0>, grid, dim3(256), LDS, stream, p);
  return launch(mfa_gemm2_kernel<E, 3>, grid, dim3(256), LDS, stream, p);
}

constexpr int64_t kGemm3MinTiles = 256;  // one workgroup per CU

// NN whole tiles of 256 x 256 (M % 256 == N % 256 == 0, K % 64 == 0), 16-bit operands: one
// 512-thread workgroup per CU, 8 waves of 128 m x 64 n (two per SIMD).  Same layout as
// mfa_gemm2_kernel<E, 3> (A by 16-byte row reads, B by transposed reads in the natural k
// order, D^T computed so the lane is m), with each staged 64-deep k-step serving 256 x 256
// outputs: half the LDS-DMA bytes per FLOP of the 128 x 128 kernel, and 8 MFMAs per 6 fragment
// reads instead of 4 per 4.  For the MLA decompression ([B·S, 512] x [512, H·D], two outputs)
// the grid is one round of the chip instead of two.
// LAY as in mfa_gemm2_kernel: 3 = NN, 1 = NT (B stored [N][K]: both operands k-contiguous
// images read by rows), 2 = TN (A stored [K][M]: both operands read transposed, permuted order).
template <class E, int LAY = 3>
__global__ void __launch_bounds__(512, 1) mfa_gemm3_kernel(GemmParams p) {
  constexpr int BM = 256, BN = 256, BK = 64;
  using TAa = TileA<BK>;   // k-contiguous tile: 256 rows of 64 k (128 B)
  using TBb = TileA<BN>;   // m/n-contiguous tile: 64 rows of 256 (512 B)
  using AB = Arith16<E, BN>;
  constexpr bool AK = LAY != 2, BKR = LAY == 1;  // A / B rows are k-contiguous
  constexpr int ATILE = BM * BK * 2, BTILE = BK * BN * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ab = smem;
  char* const bb = smem + 2 * ATILE;

  const int z = blockIdx.z;
  const char* A = (const char*)p.a + (p.b[1] ? 0 : z * p.sa * 2);
  const char* B = (const char*)(p.b[1] ? p.b[z] : p.b[0]) + (p.b[1] ? 0 : z * p.sb * 2);
  char* C = (char*)(p.b[1] ? p.c[z] : p.c[0]);
  const int64_t coff = p.b[1] ? 0 : z * p.sc;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int wm = wave >> 2, wn = wave & 3;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  const int rb[2] = {TAa::row_base(l32, hh, 0), TAa::row_base(l32, hh, 1)};
  const int trn[2] = {TBb::tr_base_nat(lane, 0), TBb::tr_base_nat(lane, 1)};
  const int trb[2] = {TBb::tr_base(lane, 0), TBb::tr_base(lane, 1)};

  DmaA<AK ? BK : BM, AK ? BM : BK, 512> ad;
  DmaA<BKR ? BK : BN, BKR ? BN : BK, 512> bd;
  ad.init(p.lda * 2, AK ? BM : BK, (AK ? BK : BM) * 2, tid);
  bd.init(p.ldb * 2, BKR ? BN : BK, (BKR ? BK : BN) * 2, tid);
  const char* ahead = A + (AK ? (int64_t)m0 * p.lda * 2 : (int64_t)m0 * 2);
  const char* bhead = B + (BKR ? (int64_t)n0 * p.ldb * 2 : (int64_t)n0 * 2);
  const int64_t astep = AK ? 2 : (int64_t)p.lda * 2;   // bytes per k
  const int64_t bstep = BKR ? 2 : (int64_t)p.ldb * 2;

  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = zero16();

  ad.issue(ahead, 0, ab);
  bd.issue(bhead, 0, bb);
  wait_vm();
  __syncthreads();
  int cur = 0;
  for (int k0 = 0; k0 < p.K; k0 += BK) {
    if (k0 + BK < p.K) {
      ad.issue(ahead + (int64_t)(k0 + BK) * astep, 0, ab + (cur ^ 1) * ATILE);
      bd.issue(bhead + (int64_t)(k0 + BK) * bstep, 0, bb + (cur ^ 1) * BTILE);
    }
    const char* at = ab + cur * ATILE;
    const char* bt = bb + cur * BTILE;
#pragma unroll
    for (int s = 0; s < BK / 16; ++s) {
      i16x8 af[4], bf[2];
      if constexpr (LAY == 2) {
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = AB::read_tr_a(at, trb, 32 * (s >> 1), s & 1, wm * 128 + i * 32);
#pragma unroll
        for (int j = 0; j < 2; ++j) bf[j] = AB::read_tr_a(bt, trb, 32 * (s >> 1), s & 1, wn * 64 + j * 32);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          af[i] = *reinterpret_cast<const i16x8*>(TAa::row_addr(at, rb, 4 * wm + i, s));
        if constexpr (LAY == 1) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bf[j] = *reinterpret_cast<const i16x8*>(TAa::row_addr(bt, rb, 2 * wn + j, s));
        } else {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bf[j] = AB::read_tr_nat(bt, trn, 32 * (s >> 1), s & 1, wn * 64 + j * 32);
        }
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = E::mma(bf[j], af[i], acc[i][j]);
    }
    wait_vm();
    __syncthreads();
    cur ^= 1;
  }

  // acc[i][j][r] = C[m = m0 + wm*128 + 32i + l32][n = n0 + wn*64 + 32j + acc_row(r, hh)].
  if (p.c_img) {
    // 16-bit C through a [256 m][256 n] LDS image (row pitch 528 B) over the released ring,
    // then whole 512-B rows from all 512 threads.
    constexpr int CP = BN * 2 + 16;
    const bool f16c = p.prec_c == P_FP16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x16& a = acc[i][j];
          auto cv = [&](float x) -> uint32_t {
            return f16c ? (uint32_t)f32_to_f16(x) : (uint32_t)f32_to_bf16(x);
          };
          const uint32_t w0 = cv(a[4 * g]) | (cv(a[4 * g + 1]) << 16);
          const uint32_t w1 = cv(a[4 * g + 2]) | (cv(a[4 * g + 3]) << 16);
          const int row = wm * 128 + i * 32 + l32, col = wn * 64 + j * 32 + 8 * g + 4 * hh;
          *reinterpret_cast<uint2*>(smem + row * CP + col * 2) = make_uint2(w0, w1);
        }
    __syncthreads();
    const int c16 = tid & 31;
    uint4 v[BM / 16];
#pragma unroll
    for (int it = 0; it < BM / 16; ++it)
      v[it] = *reinterpret_cast<const uint4*>(smem + (it * 16 + (tid >> 5)) * CP + c16 * 16);
    uint16_t* dst = reinterpret_cast<uint16_t*>(C) + coff + (int64_t)(m0 + (tid >> 5)) * p.ldc + n0 + c16 * 8;
#pragma unroll
    for (int it = 0; it < BM / 16; ++it)
      *reinterpret_cast<uint4*>(dst + (int64_t)it * 16 * p.ldc) = v[it];
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + wm * 128 + i * 32 + l32;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int n = n0 + wn * 64 + j * 32 + 8 * g + 4 * hh;
        const int64_t ci = coff + (int64_t)m * p.ldc + n;
        const f32x16& a = acc[i][j];
        if (p.prec_c == P_FP32) {
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(C) + ci) =
              make_float4(a[4 * g], a[4 * g + 1], a[4 * g + 2], a[4 * g + 3]);
        } else {
          auto cv = [&](float x) -> uint32_t {
            return p.prec_c == P_FP16 ? (uint32_t)f32_to_f16(x) : (uint32_t)f32_to_bf16(x);
          };
          const uint32_t w0 = cv(a[4 * g]) | (cv(a[4 * g + 1]) << 16);
          const uint32_t w1 = cv(a[4 * g + 2]) | (cv(a[4 * g + 3]) << 16);
          *reinterpret_cast<uint2*>(reinterpret_cast<uint16_t*>(C) + ci) = make_uint2(w0, w1);
        }
      }
  }
}

template <class E, int LAY = 3>
static hipError_t launch_gemm3(const GemmParams& p0, int batch, hipStream_t stream) {
  constexpr int RING = 2 * (256 * 64 * 2) + 2 * (64 * 256 * 2);
  constexpr int IMG = 256 * (256 * 2 + 16);
  constexpr int LDS = RING > IMG ? RING : IMG;
  static_assert(LDS <= 160 * 1024, "LDS");
  const dim3 grid(p0.N / 256, p0.M / 256, batch);
  GemmParams p = p0;
  auto al16 = [](const void* q) { return q == nullptr || ((uintptr_t)q & 15) == 0; };
  p.c_img = p.prec_c != P_FP32 && (p.ldc & 7) == 0 && (p.b[1] || (p.sc & 7) == 0) &&
            al16(p.c[0]) && al16(p.c[1]);
  return launch(mfa_gemm3_kernel<E, LAY>, grid, dim3(512), LDS, stream, p);
}

static bool gemm2_eligible(const GemmParams& p) {
  if (const char* e = mfa::dev_env("MFA_DISABLE_FAST")) {
    if (e[0] == '1') return false;
  }
  if (p.M % 128 || p.N % 128 || p.K % 64 || p.K == 0 || p.load_prev) return false;
  if (p.lda % 8 || p.ldb % 8 || p.ldc % 8) return false;
  auto al = [](const void* q) { return ((uintptr_t)q & 15) == 0; };
  if (!al(p.a) || !al(p.b[0]) || !al(p.c[0])) return false;
  if (p.b[1] && (!al(p.b[1]) || !al(p.c[1]))) return false;
  if (!p.b[1] && (p.sa % 8 || p.sb % 8 || p.sc % 8)) return false;
  if (p.trans_a && p.trans_b) return false;  // TT: the general kernel
  // 32-bit buffer offsets per tile stream.
  const int64_t arows = p.trans_a ? p.K : p.M, brows = p.trans_b ? p.N : p.K;
  if (arows * p.lda * 2 >= ((int64_t)1 << 31) || brows * p.ldb * 2 >= ((int64_t)1 << 31))
    return false;
  return true;
}

// 256 x 256 whole tiles filling at least one round of the chip run the 8-wave kernel (4096^3
// fp16 NN 1140 vs 932 TF; with fewer tiles than CUs the 128 x 128 kernel's 4x the workgroups
// win, e.g. a single [4096, 512] x [512, 2048] 15.0 vs 20.1 us).  MFA_GEMM3=0 / =1 forces
// gemm2 / gemm3 (A/B, tests).
static bool gemm3_pick(const GemmParams& p, int batch) {
  const char* g3 = mfa::dev_env("MFA_GEMM3");
  const int64_t tiles3 = (int64_t)(p.M / 256) * (p.N / 256) * batch;
  return p.M % 256 == 0 && p.N % 256 == 0 && (g3 ? g3[0] == '1' : tiles3 >= kGemm3MinTiles);
}

hipError_t gemm_dispatch(const GemmParams& p, int prec_ab, int batch, hipStream_t stream) {
  if (p.trans_a || p.trans_b) {  // NT / TN: whole tiles on gemm2, else the caller's fallback
    if (!gemm2_eligible(p)) return hipErrorNotSupported;
    if (gemm3_pick(p, batch)) {
      if (prec_ab == P_FP16)
        return p.trans_b ? launch_gemm3<F16, 1>(p, batch, stream) : launch_gemm3<F16, 2>(p, batch, stream);
      if (prec_ab == P_BF16)
        return p.trans_b ? launch_gemm3<BF16, 1>(p, batch, stream) : launch_gemm3<BF16, 2>(p, batch, stream);
    }
    if (prec_ab == P_FP16) return launch_gemm2<F16>(p, batch, stream);
    if (prec_ab == P_BF16) return launch_gemm2<BF16>(p, batch, stream);
    return hipErrorNotSupported;
  }
  if (gemm2_eligible(p)) {
    if (gemm3_pick(p, batch)) {
      if (prec_ab == P_FP16) return launch_gemm3<F16>(p, batch, stream);
      if (prec_ab == P_BF16) return launch_gemm3<BF16>(p, batch, stream);
    }
    if (prec_ab == P_FP16) return launch_gemm2<F16>(p, batch, stream);
    if (prec_ab == P_BF16) return launch_gemm2<BF16>(p, batch, stream);
  }
  const dim3 grid((p.N + 127) / 128, (p.M + 127) / 128, batch);
  if (prec_ab == P_FP16)
    hipLaunchKernelGGL(mfa_gemm_kernel<F16>, grid, dim3(256), 0, stream, p);
  else if (prec_ab == P_BF16)
    hipLaunchKernelGGL(mfa_gemm_kernel<BF16>, grid, dim3(256), 0, stream, p);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

template __global__ void mfa_gemm3_kernel<F16, 1>(GemmParams);
template __global__ void mfa_gemm3_kernel<BF16, 1>(GemmParams);
template __global__ void mfa_gemm3_kernel<F16, 2>(GemmParams);
template __global__ void mfa_gemm3_kernel<BF16, 2>(GemmParams);
template __global__ void mfa_gemm3_kernel<F16, 3>(GemmParams);
template __global__ void mfa_gemm3_kernel<BF16, 3>(GemmParams);
template __global__ void mfa_gemm2_kernel<F16, 0>(GemmParams);
template __global__ void mfa_gemm2_kernel<BF16, 0>(GemmParams);
template __global__ void mfa_gemm2_kernel<F16, 1>(GemmParams);
template __global__ void mfa_gemm2_kernel<BF16, 1>(GemmParams);
template __global__ void mfa_gemm2_kernel<F16, 2>(GemmParams);
template __global__ void mfa_gemm2_kernel<BF16, 2>(GemmParams);
template __global__ void mfa_gemm2_kernel<F16, 3>(GemmParams);
template __global__ void mfa_gemm2_kernel<BF16, 3>(GemmParams);

}  // namespace mfa

namespace {

struct GemmPlan {
  bool tuned;           // NN, equal 16-bit A/B: the kernels above
  int compute;          // P_FP16 / P_BF16 / P_FP32
  uint32_t lda, ldb, ldc;
};

int esize(int prec) { return prec == mfa::P_FP32 ? 4 : 2; }
bool gemm_prec_ok(int p) {
  return p == MFA_PRECISION_FP32 || p == MFA_PRECISION_FP16 || p == MFA_PRECISION_BF16;
}

// Validation and leading-dimension resolution of GEMMDescriptor.setFunctionConstants
// (GEMMDescriptor.swift:344-372): expected ld = rows when transposed, else columns.
mfa_status_t gemm_plan(const mfa_gemm_descriptor_t* d, GemmPlan* pl) {
  if (!gemm_prec_ok(d->precision_a) || !gemm_prec_ok(d->precision_b) ||
      !gemm_prec_ok(d->precision_c)) {
    mfa_api_set_error("mfa_gemm: memory precisions must be FP32, FP16 or BF16");
    return MFA_ERR_UNSUPPORTED;
  }
  if (d->M > 0x7fffffffu || d->N > 0x7fffffffu || d->K > 0x7fffffffu) {
    mfa_api_set_error("mfa_gemm: matrix dimensions exceed 2^31");
    return MFA_ERR_INVALID_ARGUMENT;
  }
  const uint32_t ea = d->transpose_a ? d->M : d->K;
  const uint32_t eb = d->transpose_b ? d->K : d->N;
  const uint32_t ec = d->N;
  pl->lda = d->lda ? d->lda : ea;
  pl->ldb = d->ldb ? d->ldb : eb;
  pl->ldc = d->ldc ? d->ldc : ec;
  if (pl->lda < ea || pl->ldb < eb || pl->ldc < ec) {
    mfa_api_set_error("mfa_gemm: Leading block dimension was too small.");
    return MFA_ERR_INVALID_DESCRIPTOR;
  }
  pl->compute = mfa::gemm_general_compute(d->precision_a, d->precision_b);
  pl->tuned = !d->transpose_a && !d->transpose_b && pl->compute != mfa::P_FP32;
  return MFA_SUCCESS;
}

}  // namespace

extern "C" mfa_status_t mfa_gemm_kernel_descriptor(const mfa_gemm_descriptor_t* d,
                                                   mfa_gemm_kernel_descriptor_t* out) {
  if (!d || !out) return MFA_ERR_INVALID_ARGUMENT;
  GemmPlan pl;
  mfa_status_t st = gemm_plan(d, &pl);
  if (st != MFA_SUCCESS) return st;
  memset(out, 0, sizeof(*out));
  out->block_m = 128;
  out->block_n = 128;
  out->block_k = pl.compute == mfa::P_FP32 ? 16 : 32;
  out->splits_m = 2;
  out->splits_n = 2;
  out->memory_precisions[0] = d->precision_a;
  out->memory_precisions[1] = d->precision_b;
  out->memory_precisions[2] = d->precision_c;
  out->register_precisions[0] = pl.compute;
  out->register_precisions[1] = pl.compute;
  out->register_precisions[2] = MFA_PRECISION_FP32;
  out->transpose_a = d->transpose_a;
  out->transpose_b = d->transpose_b;
  out->load_previous_c = d->load_previous_c;
  out->lda = pl.lda; out->ldb = pl.ldb; out->ldc = pl.ldc;
  out->threadgroup_size = 256;
  out->grid_x = (d->N + 127) / 128;
  out->grid_y = (d->M + 127) / 128;
  out->grid_z = d->batch ? d->batch : 1;
  const char* cn = pl.compute == mfa::P_FP16 ? "f16" : pl.compute == mfa::P_BF16 ? "bf16" : "f32";
  const bool tile_t = !pl.tuned && pl.compute != mfa::P_FP32 &&
                      (d->transpose_a != d->transpose_b) && !d->load_previous_c &&
                      d->M % 128 == 0 && d->N % 128 == 0 && d->K % 64 == 0 && d->K > 0 &&
                      pl.lda % 8 == 0 && pl.ldb % 8 == 0 && pl.ldc % 8 == 0;
  const bool big3 = d->M % 256 == 0 && d->N % 256 == 0 &&
                    (int64_t)(d->M / 256) * (d->N / 256) * (d->batch ? d->batch : 1) >= mfa::kGemm3MinTiles;
  if (tile_t && big3) {
    // Whole 256 x 256 tiles, one transpose, filling a round of the chip: the 8-wave kernel.
    out->block_m = 256;
    out->block_n = 256;
    out->block_k = 64;
    out->splits_m = 2;
    out->splits_n = 4;
    out->threadgroup_size = 512;
    out->grid_x = d->N / 256;
    out->grid_y = d->M / 256;
    out->threadgroup_memory_allocation = 256 * (256 * 2 + 16);
    snprintf(out->variant, sizeof(out->variant), "mfa_gemm3_kernel<%s,%s>/mfa_gemm_general_kernel",
             cn, d->transpose_a ? "TN" : "NT");
  } else if (tile_t) {
    // Whole tiles, one transpose: the LDS-DMA kernel (16-byte aligned buffers; the general
    // kernel otherwise).
    out->threadgroup_memory_allocation = 2 * (128 * 64 * 2 + 64 * 128 * 2);
    snprintf(out->variant, sizeof(out->variant), "mfa_gemm2_kernel<%s,%s>/mfa_gemm_general_kernel",
             cn, d->transpose_a ? "TN" : "NT");
  } else if (pl.tuned && !d->load_previous_c && big3 && d->K % 64 == 0 && d->K > 0 &&
             pl.lda % 8 == 0 && pl.ldb % 8 == 0 && pl.ldc % 8 == 0) {
    // Whole 256 x 256 tiles (16-byte aligned buffers): the 8-wave LDS-DMA kernel.
    out->block_m = 256;
    out->block_n = 256;
    out->block_k = 64;
    out->splits_m = 2;
    out->splits_n = 4;
    out->threadgroup_size = 512;
    out->grid_x = d->N / 256;
    out->grid_y = d->M / 256;
    out->threadgroup_memory_allocation = 256 * (256 * 2 + 16);
    snprintf(out->variant, sizeof(out->variant), "mfa_gemm3_kernel<%s>/mfa_gemm_kernel<%s>", cn, cn);
  } else if (pl.tuned) {
    out->threadgroup_memory_allocation = 2 * (128 * 32 * 2 + 32 * 128 * 2);
    snprintf(out->variant, sizeof(out->variant), "mfa_gemm_kernel<%s>/mfa_gemm2_kernel<%s>", cn, cn);
  } else {
    out->threadgroup_memory_allocation = 4 * 128 * 64;
    snprintf(out->variant, sizeof(out->variant), "mfa_gemm_general_kernel<%s,%s%s>", cn,
             d->transpose_a ? "T" : "N", d->transpose_b ? "T" : "N");
  }
  return MFA_SUCCESS;
}

extern "C" mfa_status_t mfa_gemm(const mfa_gemm_descriptor_t* d, const void* A, const void* B,
                                 void* C, void* stream) {
  using namespace mfa;
  if (!d || !A || !B || !C) return MFA_ERR_INVALID_ARGUMENT;
  GemmPlan pl;
  mfa_status_t st = gemm_plan(d, &pl);
  if (st != MFA_SUCCESS) return st;
  if (d->M == 0 || d->N == 0) return MFA_SUCCESS;
  const int batch = d->batch ? (int)d->batch : 1;
  hipError_t e = hipErrorNotSupported;
  // NT / TN with equal 16-bit operands and whole 128x128x64 tiles: the LDS-DMA kernel.
  if (!pl.tuned && pl.compute != P_FP32 && (d->transpose_a != d->transpose_b) &&
      !d->load_previous_c) {
    GemmParams p{};
    p.a = A;
    p.b[0] = B;
    p.b[1] = nullptr;
    p.c[0] = C;
    p.M = (int)d->M; p.N = (int)d->N; p.K = (int)d->K;
    p.lda = (int)pl.lda; p.ldb = (int)pl.ldb; p.ldc = (int)pl.ldc;
    p.sa = (int64_t)d->stride_a; p.sb = (int64_t)d->stride_b; p.sc = (int64_t)d->stride_c;
    p.prec_c = d->precision_c;
    p.trans_a = d->transpose_a ? 1 : 0;
    p.trans_b = d->transpose_b ? 1 : 0;
    e = gemm_dispatch(p, d->precision_a, batch, (hipStream_t)stream);
    if (e == hipSuccess) return MFA_SUCCESS;
    if (e != hipErrorNotSupported) {
      mfa_api_set_error("mfa_gemm: kernel launch failed");
      return MFA_ERR_LAUNCH;
    }
  }
  if (pl.tuned) {
    GemmParams p{};
    p.a = A;
    p.b[0] = B;
    p.b[1] = nullptr;
    p.c[0] = C;
    p.M = (int)d->M; p.N = (int)d->N; p.K = (int)d->K;
    p.lda = (int)pl.lda; p.ldb = (int)pl.ldb; p.ldc = (int)pl.ldc;
    p.sa = (int64_t)d->stride_a; p.sb = (int64_t)d->stride_b; p.sc = (int64_t)d->stride_c;
    p.prec_c = d->precision_c;
    p.load_prev = d->load_previous_c;
    e = gemm_dispatch(p, d->precision_a, batch, (hipStream_t)stream);
  } else {
    GemmGParams p{};
    p.a = A; p.b = B; p.c = C;
    p.M = (int)d->M; p.N = (int)d->N; p.K = (int)d->K;
    p.lda = (int)pl.lda; p.ldb = (int)pl.ldb; p.ldc = (int)pl.ldc;
    p.sa = (int64_t)d->stride_a; p.sb = (int64_t)d->stride_b; p.sc = (int64_t)d->stride_c;
    p.prec_a = d->precision_a; p.prec_b = d->precision_b; p.prec_c = d->precision_c;
    p.esz_a = esize(p.prec_a); p.esz_b = esize(p.prec_b); p.esz_c = esize(p.prec_c);
    p.trans_a = d->transpose_a ? 1 : 0;
    p.trans_b = d->transpose_b ? 1 : 0;
    p.load_prev = d->load_previous_c;
    e = gemm_general_dispatch(p, batch, (hipStream_t)stream);
  }
  if (e != hipSuccess) {
    mfa_api_set_error("mfa_gemm: kernel launch failed");
    return MFA_ERR_LAUNCH;
  }
  return MFA_SUCCESS;
}
