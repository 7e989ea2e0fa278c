// hadamard.hip — group-wise Hadamard rotation (HadamardRotation.swift:43-151): an in-place
// Fast Walsh-Hadamard Transform over each power-of-two block (size ≤ 1024) of an FP32 buffer
// [num_blocks][block_size], then a scale by 1/√block_size.
//
// The reference runs one thread per block, stage by stage: at stage s every pair
// (i, i + 2^s) becomes (a + b, a − b) (:118-129).  Every output element of a stage depends
// only on the stage's two inputs, so any schedule that keeps the stage order gives the same
// bits.  Here each lane holds R = min(block, 16) consecutive elements (four 16-byte loads), a
// block spans block/R lanes of one wave, stages with stride < R run in registers and the
// rest exchange whole registers with the lane `stride / R` away (ds_swizzle-free
// __shfl_xor).  The lower element of a pair computes mine + other, the upper other − mine:
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

hipError_t hadamard_dispatch(float* data, int log2n, uint64_t num_blocks, float scale,
                             hipStream_t stream) {
  const uint64_t n = 1ull << log2n;
  const uint64_t total = n * num_blocks;
  const int R = n >= 16 ? 16 : (int)n;
  const uint64_t threads = total / R;
  const uint64_t grid = (threads + 255) / 256;
  if (grid > 0x7fffffffull) return hipErrorInvalidValue;
  switch (R) {
#define MFA_HAD(RR)                                                                        \
  case RR:                                                                                 \
    hipLaunchKernelGGL(mfa_hadamard_kernel<RR>, dim3((unsigned)grid), dim3(256), 0, stream, \
                       data, log2n, total, scale);                                         \
    break;
    MFA_HAD(1) MFA_HAD(2) MFA_HAD(4) MFA_HAD(8) MFA_HAD(16)
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
