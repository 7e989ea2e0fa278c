// mfa_params.h — kernel argument structs shared by the host launcher (mfa_api.cpp) and the
// HIP kernels.  Plain data only: this is the layout of one kernarg segment per launch.
#pragma once
#include <stdint.h>

namespace mfa {

// One operand as a kernel sees it: base pointer + ELEMENT strides in BHSD order
// (MultiHeadAttention.swift:325-336 passes the same four strides; `sd` generalises the
// transposed layouts of AttentionKernelDescriptor.transposeState).
struct Operand {
  const void* ptr;
  int64_t sb, sh, ss, sd;
  int32_t prec;      // storage precision (mfa_precision_t)
  int32_t vec;       // 16-byte (8-byte for INT8) vector loads are legal for every row
  float scale;       // per-tensor quantisation scale (1 when folded / not quantised)
  int32_t zp;        // per-tensor zero point
  const float* bscale;    // blockwise scales (NULL: per-tensor)
  const int32_t* bzp;     // blockwise zero points (NULL: zero)
  int32_t bsize;          // block size (elements) of the 2-D [rows, cols] block grid
  int32_t bcols;          // ceil(cols / bsize)
  int32_t cols;           // columns of the 2-D quantisation view: the head dim, or S when qtr
  int32_t qtr;            // transposed quantised operand: the block grid is over the memory
                          // view [D rows][S cols] per head (AttentionKernel+Accumulate.swift:
                          // 461-472: row = d, col = seq, ceil(leadingDimension / BLOCK_SIZE_K))
};

struct MaskArgs {
  int32_t causal;
  int32_t window;          // sliding window active
  uint32_t window_size;
  int32_t skip_ok;         // fully masked causal/window tiles may be skipped exactly
  const float* amask;      // additive fp32 [B, H, R, C] (added to QK^T before scaling)
  const uint32_t* ranges;  // uint32x2 [B, H_kv, R] half-open key ranges
};

struct FwdParams {
  Operand q, k, v;
  float* o;
  int64_t o_sb, o_sh, o_ss, o_sd;  // O element strides (o_sd = R: transposeState.O)
  void* l;
  int32_t l_f16;           // L stored as FP16 (lowPrecisionIntermediates)
  int32_t B, H, Hkv, R, C, D;
  int32_t nblk;            // query blocks per (batch, head)
  float c_log2;            // softmax_scale * log2(e) * folded quant scales of Q and K
  float o_mul;             // folded quant scale of V
  MaskArgs mask;
  // Stream-split causal forward (attention_fwd_stream.hip): workspace = arrival counters
  // (sk_cnt_bytes, zero between launches) then two partial-state slots per range; ranges of
  // sk_len key tiles over sk_total tiles (sk_head per (batch, head)).
  void* ws;
  int32_t sk_len, sk_total, sk_head, sk_cnt_bytes;
  int32_t sk_flags;        // bit 0: closers always publish (tests)
  int32_t xcd_heads;       // adjacent shared-tile pairs: a head's pairs together on one XCD
  // Mirrored causal pairs: the light pairs (pair index >= pro_split) wait pro_delay rounds of
  // 512 shader cycles before their prologue loads, so the heavy pairs' prologue burst (the
  // kernel's critical path) has HBM to itself.
  int32_t pro_delay, pro_split;
};

struct BwdParams {
  Operand q, k, v;
  const float* o;          // forward output (fp32, dense [B, H, R, D])
  Operand dO_op;           // dO (input precision, or FP32 for the quantized API)
  const void* l;  int32_t l_f16;
  void* dD;       int32_t d_bf16;   // D in memory (FP32 or BF16-truncated)
  float* dq;  float* dk;  float* dv;
  // Row / column element strides inside one (batch, head) slice of O, dQ (slice R·D) and dK,
  // dV (slice C·D): D and 1 dense, 1 and R (or C) when transposed (AttentionDescriptor.swift:
  // 150-165 maps transposeState.O to O / dO and Q / K / V to dQ / dK / dV).
  int64_t o_ss, o_sd, dq_ss, dq_sd, dk_ss, dk_sd, dv_ss, dv_sd;
  int32_t B, H, Hkv, R, C, D;
  int32_t nblk;            // query blocks (bwd_q) or key blocks (bwd_kv) per slice
  int32_t group;           // H / Hkv (query heads per kv head)
  float c_log2;            // softmax_scale * log2(e) * quant(Q) * quant(K)
  float scale;             // softmax_scale · folded quant(V): dS = P∘(dP_int·scale - D)
  float dscale;            // softmax_scale (D = dscale · rowsum(dO∘O))
  float dq_mul;            // quant(K) folded into dQ
  float dk_mul;            // quant(Q) folded into dK
  MaskArgs mask;
};

// Split-KV decode forward (attention_decode.hip): INT8 K/V, few query rows per kv head.
struct DecodeParams {
  FwdParams f;
  int32_t rows;      // query rows per kv head: (H / H_kv) · R
  int32_t nrt;       // 32-row tiles per kv head
  int32_t nsplit;    // key splits per unit (unit = batch, kv head, row tile)
  int32_t chunk;     // keys per split (whole rounds of 4 waves x 32-key tiles)
  float* opart;      // [units][nsplit][32][D] unnormalised O of each workgroup (its 4 waves combined)
  float2* mlpart;    // [units][nsplit][32] (m, l)
  int32_t fused;     // nsplit == 1: the workgroup merges its 4 waves' partials in LDS
};

// MFMA GEMM (gemm.hip): C = A·B (+C); two (B, C) pairs share A when b[1] != nullptr.
struct GemmParams {
  const void* a;
  const void* b[2];
  void* c[2];
  int32_t M, N, K;
  int32_t lda, ldb, ldc;
  int64_t sa, sb, sc;     // batch strides (elements) when b[1] == nullptr
  int32_t prec_c;         // P_FP32 / P_FP16 / P_BF16
  int32_t load_prev;
  int32_t trans_a, trans_b;  // A stored [K][M] / B stored [N][K] (mfa_gemm2_kernel TN / NT)
  int32_t c_img;          // 16-bit C leaves through an LDS image as whole rows (set by the launcher)
};

// MLA latent-space attention (attention_mla_latent.hip): query rows of every head of a batch
// item flattened to [R = H·S_q][LAT]; the latent [S_kv][LAT] is both K and V.
struct LatentParams {
  const void* q;     // [B][R][LAT] 16-bit (Q·W_kᵀ)
  const void* lat;   // [B][S_kv][LAT] 16-bit
  void* olat;        // [B][R][LAT] 16-bit output (P·latent / l)
  void* l;           // [B][R] L = m + log2 l (FP16 when l_f16), nullable
  int32_t B, R, Sq, Skv, nblk;
  float c_log2;      // softmax scale · log2(e)
  int32_t causal, l_f16;
  // Split-KV (decode shapes): nsplit workgroups per query block, `chunk` keys each, partial
  // unnormalised Õ [B][nsplit][R][LAT] FP32 and (m, l) [B][nsplit][R] merged by a second pass.
  int32_t nsplit, chunk;
  float* opart;
  float2* mlpart;
  // Split path only: the merge also applies W_v (O[b,h,s,:] = Õ·W_v[:, h·D:(h+1)·D], FP32
  // output) when wv != nullptr, so no separate output GEMM runs.
  const void* wv;    // [LAT][H·D] 16-bit
  float* out;        // [B][H][S_q][D]
  int32_t H, D;
};

// General GEMM (gemm_general.hip): any FP32/FP16/BF16 mix, transposes, leading dimensions.
struct GemmGParams {
  const void* a;
  const void* b;
  void* c;
  int32_t M, N, K;
  int32_t lda, ldb, ldc;
  int64_t sa, sb, sc;       // batch strides (elements)
  int32_t prec_a, prec_b, prec_c;
  int32_t esz_a, esz_b, esz_c;
  int32_t trans_a, trans_b;
  int32_t load_prev;
  int32_t bmod;             // > 0: B's batch index is z % bmod (weights shared across an outer batch)
};

}  // namespace mfa
