// quantize.hip — GPU runtime quantisation, bit-exact with the reference's CPU quantiser
// (Sources/FlashAttention/GEMM/GEMMQuantization.swift):
//   tensor-wise  scale = absmax/127 (INT8) or absmax/7 (INT4), zero point 0      (:305-350)
//   block-wise   one scale per 2-D bs x bs block, row-major block order          (:353-421)
//   row-wise     one scale per row                                              (:424-479)
//   INT8  q = Int8(clamping: Int32(round(x / scale)) + zp)                       (:487-499)
//   INT4  nibble = clamp(q + 8, 0, 15), element 2i in the low nibble of byte i;  (:500-516)
//         tensor-wise pads an odd tail with nibble 8, block-wise with 0          (:600-619)
// The reference runs this on the host per call (QuantizedTensor.from, :720-860; GPU kernels in
// GEMMRuntimeQuantization.metal are only loaded when a default library exists).  Here the
// reduction and the element pass run on the device: absmax reductions are order-independent
// and the per-element arithmetic is IEEE division + round-half-away, so bytes and scales match
// the CPU oracle exactly.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "../../include/mfa/mfa.h"
#include "mfa_device.h"

namespace mfa {

__device__ __forceinline__ float load_any(const void* p, int prec, uint64_t i) {
  switch (prec) {
    case P_FP32: return reinterpret_cast<const float*>(p)[i];
    case P_FP16: return f16_to_f32(reinterpret_cast<const uint16_t*>(p)[i]);
    default: return bf16_to_f32(reinterpret_cast<const uint16_t*>(p)[i]);
  }
}

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o));
  return x;
}

// |x| as an order-preserving unsigned key (NaN-free inputs).
__device__ __forceinline__ unsigned abs_bits(float x) {
  return __builtin_bit_cast(unsigned, x) & 0x7fffffffu;
}

__global__ void qz_absmax_tensor(const void* in, int prec, uint64_t n, unsigned* ws) {
  float m = 0.f;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    m = fmaxf(m, fabsf(load_any(in, prec, i)));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) atomicMax(ws, abs_bits(m));
}

__global__ void qz_scale_tensor(const unsigned* ws, float* scale_out, float div) {
  if (threadIdx.x == 0 && blockIdx.x == 0) scale_out[0] = __builtin_bit_cast(float, ws[0]) / div;
}

// One workgroup per group: block (br, bc) of bsr x bsc elements, or a row (bsr = 1, bsc = cols).
__global__ void qz_absmax_groups(const void* in, int prec, uint64_t n, uint32_t rows,
                                 uint32_t cols, uint32_t bsr, uint32_t bsc, uint32_t nbc,
                                 float* scales, int32_t* zps, float div) {
  __shared__ float red[16];
  const uint32_t g = blockIdx.x;
  const uint32_t br = g / nbc, bc = g % nbc;
  const uint64_t r0 = (uint64_t)br * bsr, c0 = (uint64_t)bc * bsc;
  const uint64_t r1 = r0 + bsr < rows ? r0 + bsr : rows;
  const uint64_t c1 = c0 + bsc < cols ? c0 + bsc : cols;
  const uint64_t w = c1 - c0, cnt = (r1 - r0) * w;
  float m = 0.f;
  for (uint64_t t = threadIdx.x; t < cnt; t += blockDim.x) {
    const uint64_t idx = (r0 + t / w) * cols + c0 + t % w;
    if (idx < n) m = fmaxf(m, fabsf(load_any(in, prec, idx)));
  }
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float mm = 0.f;
    for (uint32_t i = 0; i < blockDim.x / 64; ++i) mm = fmaxf(mm, red[i]);
    scales[g] = mm / div;
    if (zps) zps[g] = 0;  // symmetric quantisation (GEMMQuantization.swift:410)
  }
}

__device__ __forceinline__ int32_t round_to_int(float v) {
  const float r = roundf(v);  // Swift round: half away from zero
  if (!(r == r)) return 0;
  if (r >= 2147483647.0f) return 2147483647;
  if (r <= -2147483648.0f) return (-2147483647 - 1);
  return (int32_t)r;
}
__device__ __forceinline__ int8_t clamp8(int64_t v) {
  return (int8_t)(v < -128 ? -128 : (v > 127 ? 127 : v));
}
__device__ __forceinline__ uint32_t nib(int64_t v) {
  return (uint32_t)(v < 0 ? 0 : (v > 15 ? 15 : v));
}

// mode 0 tensor-wise (scale_t[0]), 1 block-wise / 2 row-wise (scales[group]).
__global__ void qz_quantize(const void* in, int prec, uint64_t n, uint32_t cols, int target,
                            int mode, uint32_t bs, uint32_t nbc, const float* scale_t,
                            const float* scales, uint8_t* out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  auto group = [&](uint64_t i) -> uint64_t {
    const uint64_t r = i / cols, c = i % cols;
    return mode == 1 ? (r / bs) * nbc + c / bs : r;
  };
  if (target == P_INT8) {
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
      const float s = mode == 0 ? scale_t[0] : scales[group(i)];
      reinterpret_cast<int8_t*>(out)[i] = clamp8((int64_t)round_to_int(load_any(in, prec, i) / s));
    }
  } else {
    const uint64_t nbytes = (n + 1) / 2;
    for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < nbytes; t += stride) {
      const uint64_t i = 2 * t;
      const float s0 = mode == 0 ? scale_t[0] : scales[group(i)];
      const uint32_t lo = nib((int64_t)round_to_int(load_any(in, prec, i) / s0) + 8);
      uint32_t hi;
      if (i + 1 < n) {
        const float s1 = mode == 0 ? scale_t[0] : scales[group(i + 1)];
        hi = nib((int64_t)round_to_int(load_any(in, prec, i + 1) / s1) + 8);
      } else {
        hi = mode == 0 ? 8u : 0u;
      }
      out[t] = (uint8_t)((hi << 4) | lo);
    }
  }
}


// ---------------------------------------------------------------------------------------
// Vector forms (the common case: 16-byte aligned input, 8 elements per thread step).  The
// per-element arithmetic is the scalar kernels' (same division, rounding and clamping), so
// the bytes are identical; the tensor-wise absmax reduces through LDS to one atomic per
// workgroup (one atomic per wave on a single address serialised the reduction).
template <int PREC>
__device__ __forceinline__ void load8(const void* p, uint64_t v, float (&x)[8]) {
  if constexpr (PREC == P_FP32) {
    const float4 a = reinterpret_cast<const float4*>(p)[2 * v];
    const float4 b = reinterpret_cast<const float4*>(p)[2 * v + 1];
    x[0] = a.x; x[1] = a.y; x[2] = a.z; x[3] = a.w;
    x[4] = b.x; x[5] = b.y; x[6] = b.z; x[7] = b.w;
  } else {
    const uint4 a = reinterpret_cast<const uint4*>(p)[v];
    const uint32_t w[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint16_t lo = (uint16_t)(w[k] & 0xffffu), hi = (uint16_t)(w[k] >> 16);
      x[2 * k] = PREC == P_FP16 ? f16_to_f32(lo) : bf16_to_f32(lo);
      x[2 * k + 1] = PREC == P_FP16 ? f16_to_f32(hi) : bf16_to_f32(hi);
    }
  }
}

template <int PREC>
__global__ void __launch_bounds__(256) qz_absmax_tensor_v(const void* in, uint64_t n,
                                                          unsigned* ws) {
  __shared__ float red[4];
  float m = 0.f;
  const uint64_t n8 = n / 8, stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  // Four grid-stride steps' loads in flight at a time (one step at a time is a chain of HBM
  // latencies: 3.2 TB/s at 16.8 M FP32 elements).
  uint64_t v = gid;
  for (; v + 3 * stride < n8; v += 4 * stride) {
    float x[4][8];
#pragma unroll
    for (int u = 0; u < 4; ++u) load8<PREC>(in, v + u * stride, x[u]);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(x[u][k]));
  }
  for (; v < n8; v += stride) {
    float x[8];
    load8<PREC>(in, v, x);
#pragma unroll
    for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(x[k]));
  }
  for (uint64_t i = n8 * 8 + gid; i < n; i += stride) m = fmaxf(m, fabsf(load_any(in, PREC, i)));
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  // One partial per workgroup (no atomics, so no workspace reset launch): the quantise kernel
  // reduces them.
  if (threadIdx.x == 0)
    ws[blockIdx.x] = abs_bits(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3])));
}

// MODE 0 tensor-wise, 1 block-wise, 2 row-wise; requires cols % 8 == 0 (and bs % 8 == 0 for
// block-wise) so that the 8 elements of a step share one scale.
// Tensor-wise (MODE 0) with `ws`: every workgroup reduces qz_absmax_tensor_v's nws partial
// maxima (float bits of |x|, compared as unsigned like the atomicMax of the scalar path) and
// computes the scale absmax / div, as qz_scale_tensor does; thread 0 of the grid also stores it
// to scale_t.
template <int PREC, int TARGET, int MODE>
__global__ void __launch_bounds__(256) qz_quantize_v(const void* in, uint64_t n, uint32_t cols,
                                                     uint32_t bs, uint32_t nbc,
                                                     const float* scale_t, const float* scales,
                                                     uint8_t* out, const unsigned* ws, int nws,
                                                     float div) {
  const uint64_t n8 = n / 8, stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t gid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  float st = 0.f;
  if constexpr (MODE == 0) {
    if (ws) {
      __shared__ unsigned wred[4];
      unsigned mb = 0u;
      for (int i = threadIdx.x; i < nws; i += 256) mb = max(mb, ws[i]);
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mb = max(mb, (unsigned)__shfl_xor((int)mb, o));
      if ((threadIdx.x & 63) == 0) wred[threadIdx.x >> 6] = mb;
      __syncthreads();
      mb = max(max(wred[0], wred[1]), max(wred[2], wred[3]));
      st = __builtin_bit_cast(float, mb) / div;
      if (gid == 0) const_cast<float*>(scale_t)[0] = st;
    } else {
      st = scale_t[0];
    }
  }
  // One 8-element step: quantise x and store.
  auto step = [&](uint64_t v, const float (&x)[8]) {
    float s = st;
    if constexpr (MODE != 0) {
      const uint64_t i = v * 8, r = i / cols, c = i % cols;
      s = scales[MODE == 1 ? (r / bs) * nbc + c / bs : r];
    }
    if constexpr (TARGET == P_INT8) {
      uint32_t w[2] = {0u, 0u};
#pragma unroll
      for (int k = 0; k < 8; ++k)
        w[k >> 2] |= (uint32_t)(uint8_t)clamp8((int64_t)round_to_int(x[k] / s)) << (8 * (k & 3));
      reinterpret_cast<uint2*>(out)[v] = make_uint2(w[0], w[1]);
    } else {
      uint32_t w = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) w |= nib((int64_t)round_to_int(x[k] / s) + 8) << (4 * k);
      reinterpret_cast<uint32_t*>(out)[v] = w;
    }
  };
  for (uint64_t v = gid; v < n8; v += stride) {
    float x[8];
    load8<PREC>(in, v, x);
    step(v, x);
  }
  // Tail (n % 8 elements), element by element as in qz_quantize.
  const uint64_t i0 = n8 * 8;
  auto sc = [&](uint64_t i) -> float {
    if constexpr (MODE == 0) return st;
    const uint64_t r = i / cols, c = i % cols;
    return scales[MODE == 1 ? (r / bs) * nbc + c / bs : r];
  };
  if constexpr (TARGET == P_INT8) {
    for (uint64_t i = i0 + gid; i < n; i += stride)
      reinterpret_cast<int8_t*>(out)[i] =
          clamp8((int64_t)round_to_int(load_any(in, PREC, i) / sc(i)));
  } else {
    const uint64_t nbytes = (n + 1) / 2;
    for (uint64_t t = i0 / 2 + gid; t < nbytes; t += stride) {
      const uint64_t i = 2 * t;
      const uint32_t lo = nib((int64_t)round_to_int(load_any(in, PREC, i) / sc(i)) + 8);
      const uint32_t hi = i + 1 < n
                              ? nib((int64_t)round_to_int(load_any(in, PREC, i + 1) / sc(i + 1)) + 8)
                              : (MODE == 0 ? 8u : 0u);
      out[t] = (uint8_t)((hi << 4) | lo);
    }
  }
}

// Row-wise absmax when a row is L = cols/8 vectors with L a power of two <= 64: 64/L rows per
// wave, a row's vectors on L adjacent lanes, reduced by xor shuffles inside the lane group.
template <int PREC>
__global__ void __launch_bounds__(256) qz_absmax_rows_v(const void* in, uint32_t rows,
                                                        uint32_t cols, float* scales,
                                                        int32_t* zps, float div) {
  const uint32_t L = cols / 8;
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t wave = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) >> 6;
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const uint32_t rpw = 64 / L;
  for (uint64_t r0 = wave * rpw; r0 < rows; r0 += nwaves * rpw) {
    const uint64_t r = r0 + lane / L;
    float m = 0.f;
    if (r < rows) {
      float x[8];
      load8<PREC>(in, r * L + lane % L, x);
#pragma unroll
      for (int k = 0; k < 8; ++k) m = fmaxf(m, fabsf(x[k]));
    }
    for (uint32_t o = L / 2; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, (int)o));
    if (r < rows && lane % L == 0) {
      scales[r] = m / div;
      if (zps) zps[r] = 0;
    }
  }
}

__global__ void qz_dequantize(const uint8_t* in, int prec, uint64_t n, uint32_t cols, float scale,
                              int32_t zp, const float* bscale, const int32_t* bzp, uint32_t bs,
                              uint32_t nbc, float* out) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const int32_t q = prec == P_INT8 ? (int32_t)reinterpret_cast<const int8_t*>(in)[i]
                                     : (int32_t)((i & 1) ? (in[i / 2] >> 4) : (in[i / 2] & 15)) - 8;
    if (bscale) {
      const uint64_t b = (i / cols / bs) * nbc + (i % cols) / bs;
      out[i] = ((float)q - (float)(bzp ? bzp[b] : 0)) * bscale[b];
    } else {
      out[i] = ((float)q - (float)zp) * scale;
    }
  }
}

}  // namespace mfa

namespace {
thread_local char g_qerr[256];
int grid_for(uint64_t n) {
  const uint64_t g = (n + 255) / 256;
  return (int)(g < 8192 ? (g == 0 ? 1 : g) : 8192);
}
// Grid of the vector kernels: one thread per 8 elements, at most 1024 workgroups (4 per CU).
int grid_vec(uint64_t n) {
  const uint64_t g = (n / 8 + 255) / 256;
  return (int)(g < 1024 ? (g == 0 ? 1 : g) : 1024);
}
bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

template <int PREC>
void launch_absmax_v(const void* in, uint64_t n, unsigned* ws, hipStream_t s) {
  hipLaunchKernelGGL(mfa::qz_absmax_tensor_v<PREC>, dim3(grid_vec(n)), dim3(256), 0, s, in, n, ws);
}
template <int PREC, int TARGET>
void launch_quantize_v(int mode, const void* in, uint64_t n, uint32_t cols, uint32_t bs,
                       uint32_t nbc, const float* st, const float* sc, uint8_t* out,
                       const unsigned* ws, float div, hipStream_t s) {
  const dim3 g(grid_vec(n)), b(256);
  const int nws = grid_vec(n);  // qz_absmax_tensor_v's grid: one partial per workgroup
  if (mode == 0)
    hipLaunchKernelGGL((mfa::qz_quantize_v<PREC, TARGET, 0>), g, b, 0, s, in, n, cols, bs, nbc, st, sc, out, ws, nws, div);
  else if (mode == 1)
    hipLaunchKernelGGL((mfa::qz_quantize_v<PREC, TARGET, 1>), g, b, 0, s, in, n, cols, bs, nbc, st, sc, out, ws, nws, div);
  else
    hipLaunchKernelGGL((mfa::qz_quantize_v<PREC, TARGET, 2>), g, b, 0, s, in, n, cols, bs, nbc, st, sc, out, ws, nws, div);
}
template <int PREC>
void launch_quantize_vp(int target, int mode, const void* in, uint64_t n, uint32_t cols,
                        uint32_t bs, uint32_t nbc, const float* st, const float* sc, uint8_t* out,
                        const unsigned* ws, float div, hipStream_t s) {
  if (target == mfa::P_INT8)
    launch_quantize_v<PREC, mfa::P_INT8>(mode, in, n, cols, bs, nbc, st, sc, out, ws, div, s);
  else
    launch_quantize_v<PREC, mfa::P_INT4>(mode, in, n, cols, bs, nbc, st, sc, out, ws, div, s);
}
bool quantize_vec_ok(int target, int mode, const void* in, uint32_t cols, uint32_t bs,
                     const uint8_t* out) {
  if (!aligned16(in)) return false;
  if (((uintptr_t)out & (target == mfa::P_INT8 ? 7 : 3)) != 0) return false;
  return !(mode != 0 && (cols % 8 != 0 || (mode == 1 && bs % 8 != 0)));
}
// Vector quantise when the layout allows it; false: use the scalar kernel.  With `ws` (tensor-
// wise only) the kernel derives the scale from the absmax bits and writes it to `st`.
bool quantize_vec(int prec, int target, int mode, const void* in, uint64_t n, uint32_t cols,
                  uint32_t bs, uint32_t nbc, const float* st, const float* sc, uint8_t* out,
                  hipStream_t s, const unsigned* ws = nullptr, float div = 1.f) {
  if (!quantize_vec_ok(target, mode, in, cols, bs, out)) return false;
  if (prec == mfa::P_FP32) launch_quantize_vp<mfa::P_FP32>(target, mode, in, n, cols, bs, nbc, st, sc, out, ws, div, s);
  else if (prec == mfa::P_FP16) launch_quantize_vp<mfa::P_FP16>(target, mode, in, n, cols, bs, nbc, st, sc, out, ws, div, s);
  else launch_quantize_vp<mfa::P_BF16>(target, mode, in, n, cols, bs, nbc, st, sc, out, ws, div, s);
  return true;
}
}  // namespace

extern "C" size_t mfa_quantize_workspace_size(uint64_t count, uint32_t rows, uint32_t cols,
                                              int32_t mode, uint32_t block_size) {
  (void)count; (void)rows; (void)cols; (void)block_size;
  // Tensor-wise: one absmax partial per workgroup of the vector kernels (at most 1024), or the
  // scalar path's single atomic word.
  return mode == MFA_QUANT_TENSOR_WISE ? 4096 : 0;
}

extern "C" mfa_status_t mfa_quantize(const void* input, int32_t input_precision, uint64_t count,
                                     uint32_t rows, uint32_t cols, int32_t target_precision,
                                     int32_t mode, uint32_t block_size, void* output,
                                     float* scale_out, float* block_scales_out,
                                     int32_t* block_zero_points_out, void* workspace,
                                     void* stream) {
  using namespace mfa;
  if (!input || !output) return MFA_ERR_INVALID_ARGUMENT;
  if (input_precision != MFA_PRECISION_FP32 && input_precision != MFA_PRECISION_FP16 &&
      input_precision != MFA_PRECISION_BF16)
    return MFA_ERR_UNSUPPORTED;
  if (target_precision != MFA_PRECISION_INT8 && target_precision != MFA_PRECISION_INT4)
    return MFA_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const float div = target_precision == MFA_PRECISION_INT8 ? 127.0f : 7.0f;
  if (count == 0) return MFA_SUCCESS;
  if (mode == MFA_QUANT_TENSOR_WISE) {
    if (!workspace || !scale_out) return MFA_ERR_INVALID_ARGUMENT;
    const bool vec = aligned16(input) &&
                     quantize_vec_ok(target_precision, 0, input, cols ? cols : 1u, 1u,
                                     (const uint8_t*)output);
    if (!vec && hipMemsetAsync(workspace, 0, 16, s) != hipSuccess) return MFA_ERR_LAUNCH;
    if (vec) {
      if (input_precision == MFA_PRECISION_FP32)
        launch_absmax_v<P_FP32>(input, count, (unsigned*)workspace, s);
      else if (input_precision == MFA_PRECISION_FP16)
        launch_absmax_v<P_FP16>(input, count, (unsigned*)workspace, s);
      else
        launch_absmax_v<P_BF16>(input, count, (unsigned*)workspace, s);
    } else {
      hipLaunchKernelGGL(qz_absmax_tensor, dim3(grid_for(count)), dim3(256), 0, s, input,
                         input_precision, count, (unsigned*)workspace);
    }
    if (!quantize_vec(input_precision, target_precision, 0, input, count, cols ? cols : 1u, 1u,
                      1u, scale_out, nullptr, (uint8_t*)output, s, (const unsigned*)workspace,
                      div)) {
      hipLaunchKernelGGL(qz_scale_tensor, dim3(1), dim3(64), 0, s, (const unsigned*)workspace,
                         scale_out, div);
      hipLaunchKernelGGL(qz_quantize, dim3(grid_for(count)), dim3(256), 0, s, input,
                         input_precision, count, cols ? cols : 1u, target_precision, 0, 1u, 1u,
                         (const float*)scale_out, (const float*)nullptr, (uint8_t*)output);
    }
  } else if (mode == MFA_QUANT_BLOCKWISE || mode == MFA_QUANT_ROW_WISE) {
    if (!block_scales_out || rows == 0 || cols == 0) return MFA_ERR_INVALID_ARGUMENT;
    uint32_t bsr, bsc, nbr, nbc;
    if (mode == MFA_QUANT_BLOCKWISE) {
      if (block_size == 0) return MFA_ERR_INVALID_ARGUMENT;
      bsr = bsc = block_size;
      nbr = (rows + block_size - 1) / block_size;
      nbc = (cols + block_size - 1) / block_size;
    } else {
      bsr = 1; bsc = cols; nbr = rows; nbc = 1;
    }
    const uint32_t L = cols / 8;
    const bool rows_v = mode == MFA_QUANT_ROW_WISE && cols % 8 == 0 && L <= 64 &&
                        (L & (L - 1)) == 0 && aligned16(input) && (uint64_t)rows * cols == count;
    if (rows_v) {
      const uint64_t waves = ((uint64_t)rows * L + 63) / 64;
      const int grid = (int)std::min<uint64_t>((waves + 3) / 4, 4096);
      if (input_precision == MFA_PRECISION_FP32)
        hipLaunchKernelGGL(qz_absmax_rows_v<P_FP32>, dim3(grid), dim3(256), 0, s, input, rows, cols,
                           block_scales_out, block_zero_points_out, div);
      else if (input_precision == MFA_PRECISION_FP16)
        hipLaunchKernelGGL(qz_absmax_rows_v<P_FP16>, dim3(grid), dim3(256), 0, s, input, rows, cols,
                           block_scales_out, block_zero_points_out, div);
      else
        hipLaunchKernelGGL(qz_absmax_rows_v<P_BF16>, dim3(grid), dim3(256), 0, s, input, rows, cols,
                           block_scales_out, block_zero_points_out, div);
    } else {
      hipLaunchKernelGGL(qz_absmax_groups, dim3(nbr * nbc), dim3(256), 0, s, input,
                         input_precision, count, rows, cols, bsr, bsc, nbc, block_scales_out,
                         block_zero_points_out, div);
    }
    const int qmode = mode == MFA_QUANT_BLOCKWISE ? 1 : 2;
    const uint32_t bsz = block_size ? block_size : 1u;
    if (!quantize_vec(input_precision, target_precision, qmode, input, count, cols, bsz, nbc,
                      nullptr, block_scales_out, (uint8_t*)output, s))
      hipLaunchKernelGGL(qz_quantize, dim3(grid_for(count)), dim3(256), 0, s, input,
                         input_precision, count, cols, target_precision, qmode, bsz, nbc,
                         (const float*)nullptr, (const float*)block_scales_out, (uint8_t*)output);
  } else {
    return MFA_ERR_INVALID_DESCRIPTOR;
  }
  return hipGetLastError() == hipSuccess ? MFA_SUCCESS : MFA_ERR_LAUNCH;
}

extern "C" mfa_status_t mfa_dequantize(const mfa_quantized_tensor_t* t, uint64_t count,
                                       uint32_t cols, float* output, void* stream) {
  using namespace mfa;
  if (!t || !t->data || !output) return MFA_ERR_INVALID_ARGUMENT;
  if (t->precision != MFA_PRECISION_INT8 && t->precision != MFA_PRECISION_INT4)
    return MFA_ERR_UNSUPPORTED;
  if (count == 0) return MFA_SUCCESS;
  const uint32_t bs = t->block_size ? t->block_size : 1u;
  const uint32_t c = cols ? cols : 1u;
  hipLaunchKernelGGL(qz_dequantize, dim3(grid_for(count)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)t->data, t->precision, count, c, t->scale, t->zero_point,
                     t->block_scales, t->block_zero_points, bs, (c + bs - 1) / bs, output);
  return hipGetLastError() == hipSuccess ? MFA_SUCCESS : MFA_ERR_LAUNCH;
}
