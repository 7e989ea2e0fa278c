// mfa_dispatch.h — compile-time block configurations per kernel instantiation and the
// host-callable dispatch entry points of each kernel family.
#pragma once
#include <hip/hip_runtime.h>
#include "mfa_params.h"

// Sets the thread-local message mfa_last_error() returns (mfa_api.cpp).
void mfa_api_set_error(const char* msg);

namespace mfa {

template <class E, int DP> struct Arith16;
template <int DP> struct Arith32;
struct F16;
struct BF16;

template <int ELEM, int DP> struct ArithOf;
template <int DP> struct ArithOf<1, DP> { using type = Arith16<F16, DP>; };
template <int DP> struct ArithOf<2, DP> { using type = Arith16<BF16, DP>; };
template <int DP> struct ArithOf<0, DP> { using type = Arith32<DP>; };

// Forward: NW waves x 32 queries per workgroup, BK keys per K/V tile.
template <int ELEM, int DP> struct FwdCfg {
  static constexpr int BK = (ELEM == 0 || DP >= 256) ? 32 : 64;
  static constexpr int NW = 4;
};
// Backward (both phases): NW waves x 32 rows per workgroup, BT rows per traversal tile.
template <int ELEM, int DP> struct BwdCfg {
  static constexpr int BT = (ELEM == 0 || DP >= 128) ? 32 : 64;
  static constexpr int NW = 4;
};

inline void fwd_block_config(int elem, int DP, int* bq, int* bk, int* nw) {
  const int BK = (elem == 0 || DP >= 256) ? 32 : 64;
  *bq = 4 * 32; *bk = BK; *nw = 4;
}
inline int fwd_lds_bytes(int elem, int DP) {
  int bq, bk, nw; fwd_block_config(elem, DP, &bq, &bk, &nw);
  const int tile = elem == 0 ? bk * (DP + 1) * 4 : bk * DP * 2;
  return 4 * tile;
}
inline void bwd_block_config(int elem, int DP, int* bp, int* bt, int* nw) {
  const int BT = (elem == 0 || DP >= 128) ? 32 : 64;
  *bp = 4 * 32; *bt = BT; *nw = 4;
}

hipError_t fwd_dispatch(const FwdParams& p, int elem, int DP, int ksrc, int vsrc,
                        hipStream_t stream);
hipError_t bwd_q_dispatch(const BwdParams& p, int elem, int DP, int ksrc, int vsrc,
                          hipStream_t stream);
hipError_t bwd_kv_dispatch(const BwdParams& p, int elem, int DP, int ksrc, int vsrc,
                           hipStream_t stream);
int bwd_lds_bytes(int kind, int elem, int DP);
// Tuned 16-bit backward phases (attention_bwd_fast.hip); kind 0 = query, 1 = key/value.
hipError_t bwd_fast_dispatch(const BwdParams& p, int kind, int elem, int DP, hipStream_t stream);
// D-blocked forward / backward for head dimensions above 256 (attention_bigd.hip): any D,
// FP32 / FP16 / BF16 operands of one precision (quantised ones arrive dequantised).
constexpr int kBigChunk16 = 128, kBigChunk32 = 64;  // head-dimension chunk (DC) per element kind
inline int bigd_lds_bytes(int kind, int elem) {
  const int dc = elem == 0 ? kBigChunk32 : kBigChunk16;
  const int row = elem == 0 ? (dc + 1) * 4 : dc * 2;
  return kind == 0 ? (128 + 2 * 32) * row : 2 * (128 + 32) * row + 2 * 32 * 4;
}
hipError_t fwd_bigd_dispatch(const FwdParams& p, int elem, hipStream_t stream);
hipError_t bwd_bigd_dispatch(const BwdParams& p, int kind, int elem, hipStream_t stream);
// Split-KV decode forward for per-tensor INT8 K/V (attention_decode.hip) and the workspace it
// needs (partials of every wave).
size_t decode_workspace_bytes(int B, int Hkv, int rows, int C, int D);
int decode_keys(int R, int C, bool causal);
hipError_t fwd_decode_dispatch(const FwdParams& p, int elem, void* workspace, hipStream_t stream);
// FP16 Q with per-tensor INT8 / INT4 K/V (src SRC_I8 / SRC_I4) widened on load inside the
// shared-tile loop (attention_fwd_kv8.hip); D <= 128 padded to 128, no masks.
hipError_t fwd_kv8_dispatch(const FwdParams& p, int elem, int DP, int src, hipStream_t stream);
hipError_t fwd_share_kv8_dispatch(const FwdParams& p, int elem, int DP, int src,
                                  hipStream_t stream);
// Causal 16-bit forward over equal key-tile ranges (attention_fwd_stream.hip): the workspace
// it needs for p (0: p does not take it; the first *zero_bytes must be zero when allocated)
// and the launch (p.ws set).
size_t fwd_stream_workspace_bytes(const FwdParams& p, int elem, int DP, size_t* zero_bytes);
hipError_t fwd_stream_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream);
// Software-pipelined fp16 D = 128 forward (attention_fwd_pipe.hip); hipErrorNotSupported when
// the shape or mask is not covered.
hipError_t fwd_pipe_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream);
// Second-generation 16-bit forward (attention_fwd_v2.hip).
hipError_t fwd2_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream);
// Dense 16-bit copy [B, Hx, S, D] of a quantised operand holding the MFMA operands the
// dequantise-on-load staging would produce (kv_dequant.hip).
hipError_t kv_dequant_dispatch(const Operand& op, int B, int Hx, int S, int D, int elem,
                               void* out, hipStream_t stream);
// INT8 K/V on the integer matrix cores (attention_fwd_i8.hip); 128-query blocks.
hipError_t fwd_i8mma_dispatch(const FwdParams& p, int elem, hipStream_t stream);
hipError_t gemm_dispatch(const GemmParams& p, int prec_ab, int batch, hipStream_t stream);
// MLA latent-space attention (attention_mla_latent.hip); lat = 256 or 512.
hipError_t mla_latent_dispatch(const LatentParams& p, int elem, int lat, hipStream_t stream);
// Decode (S_q = 1) query projection of the absorbed MLA path; hipErrorNotSupported when the
// shapes or alignment do not fit (the caller falls back to the general GEMM).
hipError_t mla_qproj_dispatch(const void* q, const void* wk, void* qt, int B, int H, int D,
                              int Lat, int elem, hipStream_t stream);
// General GEMMDescriptor surface (gemm_general.hip); compute precision chosen from A and B.
int gemm_general_compute(int prec_a, int prec_b);
hipError_t gemm_general_dispatch(const GemmGParams& p, int batch, hipStream_t stream);

}  // namespace mfa
