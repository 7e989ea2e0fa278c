// mfa_device.h — gfx950 (CDNA4) device building blocks shared by every attention kernel.
//
// The reference builds its kernels from `simdgroup_matrix_storage<T>` 8x8 tiles with two
// elements per lane (Sources/FlashAttention/GEMM/GEMMHeaders.swift:586-820).  On CDNA4 the
// unit of work is a 64-lane wave issuing 32x32 MFMAs, so the building blocks here are:
//
//   * Arith16<F16|BF16>: v_mfma_f32_32x32x16_{f16,bf16}; an operand fragment is 8 16-bit
//     elements per lane (lane l holds row l&31, k = 8*(l>>5) + j).
//   * Arith32: v_mfma_f32_32x32x2_f32 (exact fp32, the FP32 path of the reference); a
//     fragment is one float per lane (row l&31, k = l>>5).
//
// Every product in the attention kernels is arranged "swapped" so that the accumulator of
// one MFMA chain is directly the B operand of the next (cdna_hip_programming.md §3, "An
// accumulator tile as the next MFMA's operand"): S^T = K·Q^T puts the query on the lane and
// the key in registers, so P^T feeds O^T += V^T·P^T without a trip through LDS.  The
// A operand of that second product (V^T) is read from a row-major LDS tile with the
// gfx950 transposing LDS read ds_read_b64_tr_b16.
//
// LDS tiles of 16-bit data are [rows][DP] with DP*2-byte rows split into 16-byte chunks;
// chunk `ch` of row `r` lives at r*ROWB + 16*(ch ^ swz(r)).  The XOR swizzle makes both
// the row reads (ds_read_b128, 32 lanes = 32 rows at one chunk) and the transposed reads
// (ds_read_b64_tr_b16, 4 rows x 4 chunks per 32-lane half) bank-conflict free.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mfa {

typedef short i16x8 __attribute__((ext_vector_type(8)));
typedef short i16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __fp16 fp16x4_tr __attribute__((__vector_size__(4 * sizeof(__fp16))));
typedef short i16x4_tr __attribute__((__vector_size__(4 * sizeof(short))));

constexpr float kLog2E = 1.442695041f;  // AttentionKernel+Softmax.swift:18
constexpr float kFltMax = 3.402823466e+38f;
constexpr float kFltMin = 1.175494351e-38f;
// Masked-element value in S: (0.875 / log2(e)) * -FLT_MAX (AttentionKernel+Softmax.swift:257).
constexpr float kMaskValue = -(0.875f / 1.442695041f) * 3.402823466e+38f;
// Running maxima / log-sum-exps below this are at "mask level" (every key seen so far masked).
constexpr float kMaskLevel = -1e30f;

// Precision codes mirror mfa_precision_t.
enum Prec : int { P_FP32 = 0, P_FP16 = 1, P_BF16 = 2, P_INT8 = 3, P_INT4 = 4 };

__device__ __forceinline__ float f16_to_f32(uint16_t b) {
  return (float)__builtin_bit_cast(_Float16, b);
}
__device__ __forceinline__ uint16_t f32_to_f16(float x) {
  return __builtin_bit_cast(uint16_t, (_Float16)x);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __builtin_bit_cast(float, (uint32_t)b << 16);
}
__device__ __forceinline__ uint16_t f32_to_bf16(float x) {
  return __builtin_bit_cast(uint16_t, (__bf16)x);
}

struct F16 {
  static constexpr int prec = P_FP16;
  __device__ static __forceinline__ float to_f32(uint16_t b) { return f16_to_f32(b); }
  __device__ static __forceinline__ uint16_t from_f32(float x) { return f32_to_f16(x); }
  __device__ static __forceinline__ f32x16 mma(i16x8 a, i16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
};
struct BF16 {
  static constexpr int prec = P_BF16;
  __device__ static __forceinline__ float to_f32(uint16_t b) { return bf16_to_f32(b); }
  __device__ static __forceinline__ uint16_t from_f32(float x) { return f32_to_bf16(x); }
  __device__ static __forceinline__ f32x16 mma(i16x8 a, i16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
};

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// ------------------------------------------------------------------------------------
// LDS tile geometry for 16-bit data.
template <int DP>
struct Tile16 {
  static constexpr int NC = DP / 8;       // 16-byte chunks per row
  static constexpr int ROWB = DP * 2;     // bytes per row
  __device__ static __forceinline__ int swz(int r) {
    if constexpr (NC == 4) {
      return (r >> 2) & 3;
    } else if constexpr (NC == 8) {
      return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
    } else {
      return ((r & 3) << 2) | ((r >> 2) & 3);
    }
  }
  __device__ static __forceinline__ int off(int r, int ch) {
    return r * ROWB + 16 * (ch ^ swz(r));
  }
  static constexpr int bytes(int rows) { return rows * ROWB; }
};

// "Sub-tiled" LDS image of a [rows][DP] 16-bit tile (cdna_hip_programming.md T10, image (a)):
// 8-row x 32-column sub-tiles of 512 B, ordered [row / 8][column / 32]; inside a sub-tile,
// row r's four 16-byte chunks sit at 64*(r & 7) + 16*(c ^ ((r >> 2) & 3)).  Every fragment
// read of a 32x32x16 operand, by rows (ds_read_b128) or transposed (ds_read_b64_tr_b16), is
// then one per-lane base register plus an immediate: 2 bases cover all row reads of a
// 32-row tile and 2 all transposed reads, where the plain swizzled rows of Tile16 need
// a register per chunk.  Both reads are bank-conflict free.
template <int DP>
struct TileA {
  static constexpr int NC = DP / 8;        // 16-byte chunks per row
  static constexpr int RB = 16 * DP;       // bytes per 8-row block
  static_assert(DP % 32 == 0, "TileA needs whole 32-column sub-tiles");
  __device__ static __forceinline__ int off(int r, int ch) {
    return RB * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
  }
  // Row-read bases for lane (l32, hh): parity `par` of the k-step s (chunk 2s + hh).
  __device__ static __forceinline__ int row_base(int l32, int hh, int par) {
    return RB * (l32 >> 3) + 64 * (l32 & 7) + 16 * ((2 * par + hh) ^ ((l32 >> 2) & 3));
  }
  // Row operand of k-step s for rows 32*j + l32: base row_base(.., s & 1).
  __device__ static __forceinline__ const char* row_addr(const char* tile, const int (&rbase)[2],
                                                         int j, int s) {
    return tile + rbase[s & 1] + RB * 4 * j + 512 * (s >> 1);
  }
  // Transposed-read bases for lane: 16-lane group g, row q = i >> 2, columns 4*(i & 3).
  // `half` 0 reads rows 4h + q of an 8-row block, half 1 the rows 8 further (the block after
  // it), whose chunk swizzle differs by 2.
  __device__ static __forceinline__ int tr_base(int lane, int half) {
    const int h = (lane >> 5) & 1, g = (lane >> 4) & 1, i = lane & 15;
    return 64 * (4 * h + (i >> 2)) + 16 * ((2 * g + ((i >> 1) & 1)) ^ (h ^ (2 * half))) +
           8 * (i & 1);
  }
  // Natural-order variant: lane half h receives rows 8h..8h+3 (half 0) and 8h+4..8h+7 (half 1)
  // of a 16-row k-step, i.e. k = 8h + j in register order, as a row read of a k-contiguous
  // image gives.  Each 32-lane half still reads 256 contiguous bytes (conflict-free).
  __device__ static __forceinline__ int tr_base_nat(int lane, int half) {
    const int h = (lane >> 5) & 1, g = (lane >> 4) & 1, i = lane & 15;
    return RB * h + 64 * (4 * half + (i >> 2)) +
           16 * ((2 * g + ((i >> 1) & 1)) ^ (2 * h + half)) + 8 * (i & 1);
  }
};

// Arithmetic policy for 16-bit operands (f16 or bf16 MFMA, K = 16 per instruction).
template <class E, int DP>
struct Arith16 {
  using Elem = E;
  using frag = i16x8;
  using TileT = Tile16<DP>;
  static constexpr int KSTEP = 16;          // contraction depth per MFMA
  static constexpr int DSTEPS = DP / 16;    // MFMAs along the head dimension
  static constexpr int KS32 = 2;            // k-steps per 32 keys
  static constexpr bool is_f32 = false;
  static constexpr int ESIZE = 2;

  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return E::mma(a, b, c);
  }
  // Row operand: row `r` of a [rows][DP] tile, elements d = 16*s + 8*h + j (j < 8).
  __device__ static __forceinline__ frag read_row(const char* tile, int r, int s, int h) {
    return *reinterpret_cast<const i16x8*>(tile + TileT::off(r, 2 * s + h));
  }
  // Transposed operand for the second product of a swapped chain: for k-step `s` of a
  // 32-key sub-tile starting at row `kb`, lane l (column dcol + (l&31)) receives
  // rows kb + 16*s + 8*(j>>2) + 4*h + (j&3), j = 0..7 — the k order of `pack` below.
  __device__ static __forceinline__ frag read_tr(const char* tile, int kb, int s, int dcol,
                                                 int lane) {
    const int h = (lane >> 5) & 1;
    const int g = (lane >> 4) & 1;
    const int i = lane & 15;
    const int col = dcol + 16 * g + 4 * (i & 3);
    const int ch = col >> 3;
    const int ra = kb + 16 * s + 4 * h + (i >> 2);
    const char* pa = tile + TileT::off(ra, ch) + 8 * (i & 1);
    const char* pb = tile + TileT::off(ra + 8, ch) + 8 * (i & 1);
    i16x4_tr lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)pa);
    i16x4_tr hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)pb);
    frag f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
  // read_tr on a TileA image: k-step s of the 32-key sub-tile at row kb, columns dcol..+31.
  // trb = {TileA::tr_base(lane, 0), TileA::tr_base(lane, 1)}.
  __device__ static __forceinline__ frag read_tr_a(const char* tile, const int (&trb)[2], int kb,
                                                  int s, int dcol) {
    constexpr int RB = TileA<DP>::RB;
    const int o = RB * (kb / 8 + 2 * s) + 512 * (dcol / 32);
    i16x4_tr lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)(tile + trb[0] + o));
    i16x4_tr hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)(tile + trb[1] + o + RB));
    frag f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
  // read_tr_a with tr_base_nat bases: k-step s of the 32-key sub-tile at row kb, natural k
  // order (k = 16s + 8h + j).
  __device__ static __forceinline__ frag read_tr_nat(const char* tile, const int (&trn)[2], int kb,
                                                    int s, int dcol) {
    constexpr int RB = TileA<DP>::RB;
    const int o = RB * (kb / 8 + 2 * s) + 512 * (dcol / 32);
    i16x4_tr lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)(tile + trn[0] + o));
    i16x4_tr hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) i16x4_tr*)(tile + trn[1] + o));
    frag f;
    f[0] = lo[0]; f[1] = lo[1]; f[2] = lo[2]; f[3] = lo[3];
    f[4] = hi[0]; f[5] = hi[1]; f[6] = hi[2]; f[7] = hi[3];
    return f;
  }
  __device__ static __forceinline__ frag read_row_a(const char* tile, const int (&rbase)[2],
                                                   int j, int s) {
    return *reinterpret_cast<const i16x8*>(TileA<DP>::row_addr(tile, rbase, j, s));
  }
  // Accumulator registers 8s..8s+7 rounded to 16-bit: the B operand of k-step s.
  __device__ static __forceinline__ frag pack(const f32x16& p, int s) {
    frag f;
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = (short)E::from_f32(p[8 * s + j]);
    return f;
  }
  // Global fragment load (row operand held in registers, e.g. Q): elements
  // d = 16*s + 8*h + j of a row, `vec` when the row is 16-byte aligned and in-bounds.
  template <class LoadElem>
  __device__ static __forceinline__ frag load_row_global(const uint16_t* row, int s, int h,
                                                         int D, bool valid, bool vec,
                                                         int64_t sd, LoadElem&& conv) {
    frag f;
    const int d0 = 16 * s + 8 * h;
    if (valid && vec && d0 + 8 <= D) {
      f = *reinterpret_cast<const i16x8*>(row + d0);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int d = d0 + j;
        f[j] = (valid && d < D) ? (short)row[(int64_t)d * sd] : (short)0;
      }
    }
    (void)conv;
    return f;
  }
};

// Arithmetic policy for exact fp32 (v_mfma_f32_32x32x2_f32, K = 2 per instruction).
template <int DP>
struct Arith32 {
  using frag = float;
  static constexpr int KSTEP = 2;
  static constexpr int DSTEPS = DP / 2;
  static constexpr int KS32 = 16;
  static constexpr bool is_f32 = true;
  static constexpr int ESIZE = 4;
  static constexpr int LD = DP + 1;   // padded row (floats): conflict-free column reads

  __device__ static __forceinline__ f32x16 mma(frag a, frag b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
  }
  __device__ static __forceinline__ frag read_row(const char* tile, int r, int s, int h) {
    return reinterpret_cast<const float*>(tile)[r * LD + 2 * s + h];
  }
  // Key of accumulator register s in lane half h: (s&3) + 8*(s>>2) + 4*h.
  __device__ static __forceinline__ frag read_tr(const char* tile, int kb, int s, int dcol,
                                                 int lane) {
    const int h = (lane >> 5) & 1;
    const int k = kb + (s & 3) + 8 * (s >> 2) + 4 * h;
    return reinterpret_cast<const float*>(tile)[k * LD + dcol + (lane & 31)];
  }
  __device__ static __forceinline__ frag pack(const f32x16& p, int s) { return p[s]; }
  static constexpr int tile_bytes(int rows) { return rows * LD * 4; }
};

// Rounded product that the compiler may not contract into a following add (hipcc's default
// -ffp-contract=fast-honor-pragmas would otherwise fuse x*c - m into one FMA).
__device__ __forceinline__ float mul_rn(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}

// Two FP32 values rounded to FP16 (round to nearest even) and packed, a in the low half.  An
// explicit instruction: hipcc otherwise turns some fptrunc(fmul) pairs into v_fma_mixlo_f16, one
// rounding of the exact product instead of FP32 then FP16, and different code paths then
// disagree at FP16 ties (the block-wise dequantisation pass vs the on-load widening).
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
  uint32_t r;
  asm("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Keeps a rarely taken, wave-uniform branch (edge / diagonal tile masking) a branch: without
// it the compiler if-converts the body into per-element selects that then run on every tile.
#define MFA_KEEP_BRANCH() asm volatile("" ::: "memory")

// Workgroup -> (unit, block) map that keeps each unit's blocks on one XCD, in order
// (cdna_hip_programming.md T1).  Workgroups are dealt round-robin over the 8 XCDs, so with
// units % 8 == 0 the XCD that receives workgroups x, x+8, x+16, ... walks the blocks of units
// x, x+8, ... one unit at a time: the unit's shared operands (K/V of a head in the forward,
// Q/dO or K/V in the backward) stay in that XCD's L2.  Placement only changes speed.
__device__ __forceinline__ void xcd_unit_block(int bid, int units, int nblk, int* unit,
                                               int* blk) {
  if ((units & 7) == 0) {
    const int j = bid >> 3;
    *unit = (j / nblk) * 8 + (bid & 7);
    *blk = j % nblk;
  } else {
    *unit = bid % units;
    *blk = bid / units;
  }
}

// Row index (within a 32-row MFMA output tile) of accumulator register i in lane half h.
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// Masks a tile of NJ 32x32 accumulators whose element (j, i) sits at offset
// j*32 + acc_row(i, hh) along the accumulator row axis: elements whose offset (relative to
// the lane's half-wave base, i.e. without the 4·hh term) lies outside [lo, hi] become `val`.
// Compile-time offsets against two per-lane bounds: compares and selects, no branches.
template <int NJ>
__device__ __forceinline__ void mask_outside(f32x16 (&s)[NJ], int lo, int hi, float val) {
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kk = j * 32 + (i & 3) + 8 * (i >> 2);
      s[j][i] = (kk < lo || kk > hi) ? val : s[j][i];
    }
}

// Max / sum across the two 32-lane halves (lanes l and l^32 hold the same column).
__device__ __forceinline__ float xhalf_max(float x) { return fmaxf(x, __shfl_xor(x, 32)); }
__device__ __forceinline__ float xhalf_sum(float x) { return x + __shfl_xor(x, 32); }

// The same reductions through v_permlane32_swap (no LDS round trip; lanes l and l^32 swap).
__device__ __forceinline__ float cross_half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
// The same with IEEE maximum (v_maximum_f32: no operand canonicalisation; NaN propagates).
__device__ __forceinline__ float cross_half_maximum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_elementwise_maximum(__builtin_bit_cast(float, (unsigned)r[0]),
                                       __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float cross_half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

}  // namespace mfa
