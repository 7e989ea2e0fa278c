// hadamard.hip — group-wise Hadamard rotation (HadamardRotation.swift:43-151): an in-place
// Fast Walsh-Hadamard Transform over each power-of-two block (size ≤ 1024) of an FP32 buffer
// [num_blocks][block_size], then a scale by 1/√block_size.
//
// The reference runs one thread per block, stage by stage: at stage s every pair
// (i, i + 2^s) becomes (a + b, a − b) (:118-129).  Every output element of a stage depends
// only on the stage's two inputs, so any schedule that keeps the stage order gives the same
// bits.  Blocks of 4 or more elements use mfa_hadamard_wave_kernel (coalesced wave layout,
// below); blocks of 1 or 2 use mfa_hadamard_kernel, where each lane holds R = block
// consecutive elements (with R = 16, stages with stride < R run in registers and the rest
// exchange whole registers with the lane `stride / R` away).  The lower element of a pair computes mine + other, the upper other − mine:
// the reference's a + b and a − b operand for operand.
//
// Scale: the reference multiplies by Metal's rsqrt((float)N) (:132-135).  Here it is the
// correctly rounded FP32 value of 1/√N (exact for N = 4^k), computed on the host.
//
// HBM-bound: 8 bytes per element (one read, one write); no LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mfa/mfa.h"
#include "mfa_dispatch.h"

namespace mfa {

template <int R>
__global__ void __launch_bounds__(256) mfa_hadamard_kernel(float* __restrict__ data, int log2n,
                                                          uint64_t total, float scale) {
  const uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t base = t * R;
  const bool live = base < total;  // whole blocks are live or not: their lanes stay in step
  float v[R];
  if (live) {
    if constexpr (R >= 4) {
#pragma unroll
      for (int i = 0; i < R / 4; ++i) {
        const float4 x = reinterpret_cast<const float4*>(data + base)[i];
        v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < R; ++i) v[i] = data[base + i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = 0.f;
  }
  // In-register stages: stride 1 .. R/2 (all of them when the block is ≤ R).
#pragma unroll
  for (int st = 1; st < R; st <<= 1) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      if (i & st) continue;
      const float a = v[i], b = v[i + st];
      v[i] = a + b;
      v[i + st] = a - b;
    }
  }
  // Cross-lane stages: stride R .. N/2, lane distance stride / R.
  const int lane = threadIdx.x & 63;
  for (int s = 0; (R << s) < (1 << log2n); ++s) {
    const int d = 1 << s;
    const bool upper = (lane & d) != 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const float o = __shfl_xor(v[i], d);
      v[i] = upper ? o - v[i] : v[i] + o;
    }
  }
  if (!live) return;
  if constexpr (R >= 4) {
#pragma unroll
    for (int i = 0; i < R / 4; ++i)
      reinterpret_cast<float4*>(data + base)[i] =
          make_float4(v[4 * i] * scale, v[4 * i + 1] * scale, v[4 * i + 2] * scale,
                      v[4 * i + 3] * scale);
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) data[base + i] = v[i] * scale;
  }
}

// Blocks of N >= 4: each wave owns 256·I consecutive elements (I = max(1, N/256)) and reads
// them with I fully coalesced 16-byte-per-lane instructions (instruction i, lane l: elements
// 256·i + 4·l .. +3), so lane l holds v[4i + k] = element 256·i + 4·l + k.  The element-index
// bits are then k (strides 1, 2: in registers), lane (strides 4 .. 128: __shfl_xor by
// stride / 4) and i (strides 256, 512: in registers), and the stages still run in increasing
// stride order with the reference's operands (lower: a + b, upper: a − b).  (Measured on a
// 1 GiB buffer: 5.6-6.0 TB/s vs 5.0-5.1 for 16 consecutive elements per lane.)
template <int I>
__global__ void __launch_bounds__(256) mfa_hadamard_wave_kernel(float* __restrict__ data,
                                                                int log2n, uint64_t total,
                                                                float scale) {
  const int lane = threadIdx.x & 63;
  const uint64_t wbase = ((uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * (256 * I);
  const int n = 1 << log2n;
  float v[4 * I];
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const uint64_t e = wbase + 256 * i + 4 * lane;
    float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < total) x = *reinterpret_cast<const float4*>(data + e);
    v[4 * i] = x.x; v[4 * i + 1] = x.y; v[4 * i + 2] = x.z; v[4 * i + 3] = x.w;
  }
  // Strides 1 and 2 (k bits).
#pragma unroll
  for (int st = 1; st <= 2; st <<= 1) {
    if (st >= n) break;
#pragma unroll
    for (int j = 0; j < 4 * I; ++j) {
      if (j & st) continue;
      const float a = v[j], b = v[j + st];
      v[j] = a + b;
      v[j + st] = a - b;
    }
  }
  // Strides 4 .. 128 (lane bits).
  for (int d = 1; d <= 32 && 4 * d < n; d <<= 1) {
    const bool upper = (lane & d) != 0;
#pragma unroll
    for (int j = 0; j < 4 * I; ++j) {
      const float o = __shfl_xor(v[j], d);
      v[j] = upper ? o - v[j] : v[j] + o;
    }
  }
  // Strides 256 and 512 (i bits: register groups of 4).
#pragma unroll
  for (int e = 1; e < I; e <<= 1) {
#pragma unroll
    for (int i = 0; i < I; ++i) {
      if (i & e) continue;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float a = v[4 * i + k], b = v[4 * (i + e) + k];
        v[4 * i + k] = a + b;
        v[4 * (i + e) + k] = a - b;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const uint64_t e = wbase + 256 * i + 4 * lane;
    if (e < total)
      *reinterpret_cast<float4*>(data + e) = make_float4(v[4 * i] * scale, v[4 * i + 1] * scale,
                                                         v[4 * i + 2] * scale, v[4 * i + 3] * scale);
  }
}

hipError_t hadamard_dispatch(float* data, int log2n, uint64_t num_blocks, float scale,
                             hipStream_t stream) {
  const uint64_t n = 1ull << log2n;
  const uint64_t total = n * num_blocks;
  if (n >= 4) {
    const int I = n >= 1024 ? 4 : (n >= 512 ? 2 : 1);
    const uint64_t grid = (total + 1024 * I - 1) / (1024 * I);
    if (grid > 0x7fffffffull) return hipErrorInvalidValue;
    if (I == 4)
      hipLaunchKernelGGL(mfa_hadamard_wave_kernel<4>, dim3((unsigned)grid), dim3(256), 0, stream,
                         data, log2n, total, scale);
    else if (I == 2)
      hipLaunchKernelGGL(mfa_hadamard_wave_kernel<2>, dim3((unsigned)grid), dim3(256), 0, stream,
                         data, log2n, total, scale);
    else
      hipLaunchKernelGGL(mfa_hadamard_wave_kernel<1>, dim3((unsigned)grid), dim3(256), 0, stream,
                         data, log2n, total, scale);
    return hipGetLastError();
  }
  const int R = (int)n;  // 1 or 2
  const uint64_t threads = total / R;
  const uint64_t grid = (threads + 255) / 256;
  if (grid > 0x7fffffffull) return hipErrorInvalidValue;
  switch (R) {
#define MFA_HAD(RR)                                                                        \
  case RR:                                                                                 \
    hipLaunchKernelGGL(mfa_hadamard_kernel<RR>, dim3((unsigned)grid), dim3(256), 0, stream, \
                       data, log2n, total, scale);                                         \
    break;
    MFA_HAD(1) MFA_HAD(2)
#undef MFA_HAD
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace mfa

namespace {

// HadamardRotation.rotate preconditions (:49-52).
mfa_status_t hadamard_check(const float* buffer, uint32_t block_size, uint32_t num_blocks,
                            int* log2n) {
  if (!buffer) {
    mfa_api_set_error("mfa_hadamard_rotate: null buffer");
    return MFA_ERR_INVALID_ARGUMENT;
  }
  if (block_size == 0 || (block_size & (block_size - 1)) != 0) {
    mfa_api_set_error("mfa_hadamard_rotate: blockSize must be power of 2");
    return MFA_ERR_INVALID_ARGUMENT;
  }
  if (block_size > 1024) {
    mfa_api_set_error("mfa_hadamard_rotate: blockSize must be <= 1024");
    return MFA_ERR_INVALID_ARGUMENT;
  }
  if (num_blocks == 0) {
    mfa_api_set_error("mfa_hadamard_rotate: numBlocks must be > 0");
    return MFA_ERR_INVALID_ARGUMENT;
  }
  if (block_size >= 4 && (((uintptr_t)buffer) & 15) != 0) {
    mfa_api_set_error("mfa_hadamard_rotate: buffer must be 16-byte aligned");
    return MFA_ERR_UNSUPPORTED;
  }
  int l = 0;
  while ((1u << l) < block_size) ++l;
  *log2n = l;
  return MFA_SUCCESS;
}

}  // namespace

extern "C" float mfa_hadamard_scale(uint32_t block_size) {
  return (float)(1.0 / __builtin_sqrt((double)block_size));
}

extern "C" mfa_status_t mfa_hadamard_rotate(float* buffer, uint32_t block_size,
                                            uint32_t num_blocks, void* stream) {
  int log2n;
  mfa_status_t st = hadamard_check(buffer, block_size, num_blocks, &log2n);
  if (st != MFA_SUCCESS) return st;
  if (mfa::hadamard_dispatch(buffer, log2n, num_blocks, mfa_hadamard_scale(block_size),
                             (hipStream_t)stream) != hipSuccess) {
    mfa_api_set_error("mfa_hadamard_rotate: kernel launch failed");
    return MFA_ERR_LAUNCH;
  }
  return MFA_SUCCESS;
}

extern "C" mfa_status_t mfa_hadamard_rotate_batch(const mfa_hadamard_item_t* items,
                                                  uint32_t count, void* stream) {
  if (count && !items) return MFA_ERR_INVALID_ARGUMENT;
  // Validate every item before enqueuing any (the reference traps on the first bad one).
  for (uint32_t i = 0; i < count; ++i) {
    int l;
    mfa_status_t st = hadamard_check(items[i].buffer, items[i].block_size, items[i].num_blocks, &l);
    if (st != MFA_SUCCESS) return st;
  }
  for (uint32_t i = 0; i < count; ++i) {
    mfa_status_t st =
        mfa_hadamard_rotate(items[i].buffer, items[i].block_size, items[i].num_blocks, stream);
    if (st != MFA_SUCCESS) return st;
  }
  return MFA_SUCCESS;
}
