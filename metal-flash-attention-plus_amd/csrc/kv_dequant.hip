// kv_dequant.hip — one-pass dequantisation of a quantised attention operand into a dense
// 16-bit copy, so the tuned 16-bit kernels (attention_fwd_v2.hip, attention_bwd_fast.hip) run
// quantised K/V (and Q) instead of the generic dequantise-on-load kernels.
//
// The copy holds exactly the MFMA operands the dequantise-on-load staging produces
// (mfa_stage.h convert_qchunk): per-tensor the integers q - zp (exact in FP16/BF16; the scale
// stays folded into the softmax / output multipliers), blockwise the dequantised value
// (q - zp)·s rounded to the element type — so results are bit-identical to staging every tile
// from the quantised tensor, while each element is converted once per call instead of once
// per query block that reads it (GEMMHeaders.swift:679-808, reference dequantize-on-load).
// HBM-bound: 1 (INT8) or 0.5 (INT4) byte read + 2 bytes written per element.
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

// Dense output [B, Hx, S, D] (row stride D elements); one 8-element chunk per thread step.
template <class E, int SRC>
__global__ void __launch_bounds__(256) mfa_kv_dequant_kernel(Operand op, int Hx, int S, int D,
                                                              uint64_t chunks, uint16_t* out) {
  const int cpr = (D + 7) / 8;
  for (uint64_t idx = blockIdx.x * 256ull + threadIdx.x; idx < chunks;
       idx += (uint64_t)gridDim.x * 256ull) {
    const uint64_t rowg = idx / cpr;
    const int c = (int)(idx - rowg * cpr);
    const int row = (int)(rowg % S);
    const uint64_t bh = rowg / S;
    const int hx = (int)(bh % Hx), b = (int)(bh / Hx);
    const int64_t rowoff = (int64_t)b * op.sb + (int64_t)hx * op.sh + (int64_t)row * op.ss;
    const int d0 = c * 8;
    const uint4 raw = load_qchunk<SRC>(op, rowoff, d0, D);
    const uint4 v = convert_qchunk<E, SRC>(raw, op, op.bscale ? quant_row(op, b, hx) : 0, row, d0,
                                           D, true);
    uint16_t* dst = out + rowg * D + d0;
    if (d0 + 8 <= D) {
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; d0 + j < D; ++j) dst[j] = (uint16_t)(w[j >> 1] >> (16 * (j & 1)));
    }
  }
}

hipError_t kv_dequant_dispatch(const Operand& op, int B, int Hx, int S, int D, int elem,
                               void* out, hipStream_t stream) {
  const uint64_t chunks = (uint64_t)B * Hx * S * ((D + 7) / 8);
  if (chunks == 0) return hipSuccess;
  const uint64_t want = (chunks + 255) / 256;
  const dim3 grid((unsigned)(want < 8192 ? want : 8192));
  const int src = op.prec == P_INT8 ? SRC_I8 : op.prec == P_INT4 ? SRC_I4 : -1;
#define MFA_KVD(EE, SS)                                                                    \
  return launch(mfa_kv_dequant_kernel<EE, SS>, grid, dim3(256), 0, stream, op, Hx, S, D,   \
                chunks, (uint16_t*)out);
  if (elem == P_FP16 && src == SRC_I8) MFA_KVD(F16, SRC_I8)
  if (elem == P_FP16 && src == SRC_I4) MFA_KVD(F16, SRC_I4)
  if (elem == P_BF16 && src == SRC_I8) MFA_KVD(BF16, SRC_I8)
  if (elem == P_BF16 && src == SRC_I4) MFA_KVD(BF16, SRC_I4)
#undef MFA_KVD
  return hipErrorNotSupported;
}

}  // namespace mfa
