// mfa_stage.h — global -> register -> LDS staging of [ROWS][DP] operand tiles, and the
// per-lane register fragments of operands held for a whole kernel (Q in the forward pass).
//
// Staging is split into load() (issue the global loads into registers) and store()
// (dequantise/convert and write the swizzled LDS image), so a kernel can issue the next
// tile's loads before its MFMA work and write them after (cdna_hip_programming.md T14).
//
// Quantised sources follow the reference's dequantize-on-load semantics
// (GEMMHeaders.swift:679-808): value = (q - zero_point) * scale, INT4 nibble n -> n - 8 with
// element 2i in the low nibble (GEMMQuantization.swift:500-515), blockwise scale index
// (row / bs) * ceil(cols / bs) + col / bs over the 2-D [rows, cols] view
// (GEMMQuantization.swift:561-575, AttentionKernel+OuterProduct.swift:301-316).
// A per-tensor scale is folded into the softmax / output multipliers by the host so the
// staged integers (q - zp) are exact in the 16-bit MFMA operand.
#pragma once
#include "mfa_device.h"
#include "mfa_params.h"
#include "mfa_launch.h"

namespace mfa {

// SRC_SAME: storage = MFMA element type.  SRC_I8/SRC_I4: quantised integers.
// SRC_F32ANY: runtime choice between the MFMA element type and FP32 storage that is rounded
// to the element type (dO is FP32 in memory unless lowPrecisionInputs,
// AttentionDescriptor+Precisions.swift:17-26).
enum SrcKind : int { SRC_SAME = 0, SRC_I8 = 1, SRC_I4 = 2, SRC_F32ANY = 3 };

__device__ __forceinline__ int8_t ld_i4(const uint8_t* base, int64_t e) {
  const uint8_t byte = base[e >> 1];
  const int nib = (e & 1) ? (byte >> 4) : (byte & 15);
  return (int8_t)(nib - 8);
}

// First row of head (b, hx) in the 2-D [rows, cols] quantisation view of a quantised operand.
// Quantised operands are dense (row-major or transposed within each head, make_operand), so the
// head starts at view row (b·sb + hx·sh) / cols whatever the layout inside the head.  The view
// is the operand's memory layout, as the reference's factory quantises a buffer
// (GEMMQuantization.swift:561-575): row-major [S][D] rows (cols = D), or, for a transposed
// operand, [D][S] rows (cols = S; AttentionKernel+Accumulate.swift:461-472 and
// AttentionKernel+OuterProduct.swift:301-316 index it with row = d, col = seq).
__device__ __forceinline__ int64_t quant_row(const Operand& op, int b, int hx) {
  return ((int64_t)b * op.sb + (int64_t)hx * op.sh) / op.cols;
}

// Dequantised value of quantised element (sequence row `row`, column `col`) of the head whose
// first view row is `hrow`, with integer payload qv.
__device__ __forceinline__ float dequant(const Operand& op, int qv, int64_t hrow, int64_t row,
                                         int col) {
  if (op.bscale) {
    const int64_t vr = op.qtr ? hrow + col : hrow + row;
    const int64_t vc = op.qtr ? row : col;
    const int64_t bi = (vr / op.bsize) * op.bcols + vc / op.bsize;
    const int zp = op.bzp ? op.bzp[bi] : 0;
    // One FP32 rounding of the product, then (at the caller) one rounding to the 16-bit type:
    // mul_rn keeps hipcc from contracting the multiply and the conversion into v_fma_mixlo_f16
    // (a single rounding), so every path holds the same values (kv_bytes.h widen_block).
    return mul_rn((float)(qv - zp), op.bscale[bi]);
  }
  return (float)(qv - op.zp);  // per-tensor scale folded by the host
}

typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

// 8 quantised elements (INT8 in raw.x/raw.y, or 8 INT4 nibbles in raw.x) -> 8 MFMA elements
// holding q - zp.  FP16: build 1024 + u in the fp16 bit pattern (0x6400 | u, u = q + 128 via
// v_perm_b32) and subtract 1152 + zp with packed fp16 math — exact for |q - zp| <= 1024.
template <class E, int SRC>
__device__ __forceinline__ uint4 dequant_fast(const uint4 raw, float zp) {
  uint32_t w[4];
  if constexpr (E::prec == P_FP16) {
    if constexpr (SRC == SRC_I8) {
      const uint32_t u0 = raw.x ^ 0x80808080u, u1 = raw.y ^ 0x80808080u;
      w[0] = __builtin_amdgcn_perm(0x64646464u, u0, 0x04010400u);
      w[1] = __builtin_amdgcn_perm(0x64646464u, u0, 0x04030402u);
      w[2] = __builtin_amdgcn_perm(0x64646464u, u1, 0x04010400u);
      w[3] = __builtin_amdgcn_perm(0x64646464u, u1, 0x04030402u);
      const _Float16 m = (_Float16)(1152.0f + zp);
      const f16x2 mm = {m, m};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, w[k]) - mm);
    } else {  // INT4 nibble n encodes n - 8
      // Even elements (low nibbles) and odd ones (high nibbles) masked out once, then each
      // pair's two bytes placed as the low bytes of its halfwords by one v_perm (0x0C selects
      // a zero byte) and the 0x64 exponent bytes OR-ed in: 15 VALU per 8 elements, not 20.
      const uint32_t lo = raw.x & 0x0F0F0F0Fu, hi = (raw.x >> 4) & 0x0F0F0F0Fu;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = __builtin_amdgcn_perm(hi, lo, 0x0C040C00u + 0x00010001u * k) | 0x64006400u;
      const _Float16 m = (_Float16)(1032.0f + zp);
      const f16x2 mm = {m, m};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, w[k]) - mm);
    }
  } else if constexpr (E::prec == P_BF16) {
    // BF16: q - zp in f32 (v_cvt_f32_ubyte of the biased byte, one subtract), then the two
    // upper halves packed by one v_perm.  The host holds |zp| <= 128, so |q - zp| <= 256 has
    // at most 8 significant bits: the f32 low halves are zero and the truncation is exact
    // (the value f32_to_bf16 gives).
    const float m = (SRC == SRC_I8 ? 128.0f : 8.0f) + zp;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a, b;
      if constexpr (SRC == SRC_I8) {
        const uint32_t u = (k < 2 ? raw.x : raw.y) ^ 0x80808080u;
        a = (float)((u >> (16 * (k & 1))) & 0xffu) - m;
        b = (float)((u >> (16 * (k & 1) + 8)) & 0xffu) - m;
      } else {
        a = (float)((raw.x >> (8 * k)) & 15u) - m;
        b = (float)((raw.x >> (8 * k + 4)) & 15u) - m;
      }
      w[k] = __builtin_amdgcn_perm(__builtin_bit_cast(uint32_t, b), __builtin_bit_cast(uint32_t, a),
                                   0x07060302u);
    }
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      int q0, q1;
      if constexpr (SRC == SRC_I8) {
        const uint32_t word = k < 2 ? raw.x : raw.y;
        q0 = (int)(int8_t)(word >> (16 * (k & 1)));
        q1 = (int)(int8_t)(word >> (16 * (k & 1) + 8));
      } else {
        q0 = (int)((raw.x >> (8 * k)) & 15u) - 8;
        q1 = (int)((raw.x >> (8 * k + 4)) & 15u) - 8;
      }
      w[k] = (uint32_t)E::from_f32((float)q0 - zp) | ((uint32_t)E::from_f32((float)q1 - zp) << 16);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// One 8-element chunk (columns d0..d0+7 of the row at element offset rowoff) of a quantised
// operand: INT8 bytes in .x/.y, or eight INT4 nibbles in .x (columns past D decode to 0).
template <int SRC>
__device__ __forceinline__ uint4 load_qchunk(const Operand& op, int64_t rowoff, int d0, int D) {
  uint4 v = make_uint4(0u, 0u, 0u, 0u);
  if constexpr (SRC == SRC_I8) {
    const int8_t* base = (const int8_t*)op.ptr + rowoff;
    if (op.vec && d0 + 8 <= D) {
      const uint2 t = *reinterpret_cast<const uint2*>(base + d0);
      v.x = t.x; v.y = t.y;
    } else {
      uint32_t w[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (d0 + j < D) w[j >> 2] |= (uint32_t)(uint8_t)base[(int64_t)(d0 + j) * op.sd] << (8 * (j & 3));
      v.x = w[0]; v.y = w[1];
    }
  } else {  // SRC_I4: element index e -> byte e/2, low nibble = even element
    const uint8_t* base = (const uint8_t*)op.ptr;
    uint32_t w = 0u;
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (d0 + j < D) {
        const int64_t e = rowoff + (int64_t)(d0 + j) * op.sd;
        const uint8_t byte = base[e >> 1];
        const uint32_t nib = (e & 1) ? (byte >> 4) : (byte & 15);
        w |= nib << (4 * j);
      } else {
        w |= 8u << (4 * j);  // decodes to 0
      }
    v.x = w;
  }
  return v;
}

// The MFMA-type chunk of a quantised chunk: per-tensor the exact integers q - zp (the scale is
// folded by the host); blockwise the dequantised value (q - zp)·s rounded to the element type.
// `hrow` is the head's first view row (quant_row), `row` the sequence row; invalid rows give
// zeros.
template <class E, int SRC>
__device__ __forceinline__ uint4 convert_qchunk(const uint4 raw, const Operand& op, int64_t hrow,
                                                int64_t row, int d0, int D, bool valid) {
  if (!op.bscale) return dequant_fast<E, SRC>(raw, (float)op.zp);
  uint32_t w[4];
#pragma unroll
  for (int jj = 0; jj < 4; ++jj) {
    uint32_t packed = 0u;
    float xs[2] = {0.f, 0.f};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * jj + e;
      int qv;
      if constexpr (SRC == SRC_I8) {
        const uint32_t word = j < 4 ? raw.x : raw.y;
        qv = (int)(int8_t)((word >> (8 * (j & 3))) & 0xff);
      } else {
        qv = (int)((raw.x >> (4 * j)) & 15u) - 8;
      }
      float x = 0.f;
      if (valid && d0 + j < D) x = dequant(op, qv, hrow, row, d0 + j);
      if constexpr (E::prec == P_FP16)
        xs[e] = x;
      else
        packed |= (uint32_t)E::from_f32(x) << (16 * e);
    }
    // (FP16: the explicit conversion of kv_bytes.h widen_block, so both hold the same bits.)
    if constexpr (E::prec == P_FP16) packed = pack_f16x2(xs[0], xs[1]);
    w[jj] = packed;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Eight 16-bit elements d0..d0+7 of a row at element stride sd (zero past D), packed.
__device__ __forceinline__ uint4 gather16(const uint16_t* p, int d0, int D, int64_t sd) {
  auto e = [&](int j) -> uint32_t { return d0 + j < D ? (uint32_t)p[(int64_t)(d0 + j) * sd] : 0u; };
  return make_uint4(e(0) | (e(1) << 16), e(2) | (e(3) << 16), e(4) | (e(5) << 16),
                    e(6) | (e(7) << 16));
}

template <class A, int ROWS, int DP, int NT, int SRC>
struct Stager {
  static constexpr int CE = 16 / A::ESIZE;   // output elements per 16-byte chunk
  static constexpr int CPR = DP / CE;        // chunks per row
  static constexpr int NCH = ROWS * CPR;
  static constexpr int PER = (NCH + NT - 1) / NT;
  uint4 raw[PER];
  uint4 raw2[SRC == SRC_F32ANY ? PER : 1];  // upper 16 bytes of an FP32-stored chunk

  // coff: element offset of the first column (a column chunk [c0, c0 + DP) of a wider
  // operand: coff = c0 * op.sd, D = columns left from c0); non-quantised sources only.
  __device__ __forceinline__ void load(const Operand& op, int b, int hx, int row0, int nrows,
                                       int D, int64_t coff = 0) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + i * NT;
      const int r = id / CPR, c = id % CPR;
      const int grow = row0 + r;
      const int d0 = c * CE;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      uint4 v2 = make_uint4(0u, 0u, 0u, 0u);  // upper half of an FP32-stored chunk
      if ((NCH % NT == 0 || id < NCH) && grow < nrows && d0 < D) {
        const int64_t rowoff =
            (int64_t)b * op.sb + (int64_t)hx * op.sh + (int64_t)grow * op.ss + coff;
        // Element-wise fallbacks (strided / unaligned rows, the row's last partial chunk)
        // build the chunk from scalar loads without a local array, so the staging registers
        // never go through scratch.
        if constexpr (SRC == SRC_F32ANY) {
          if (op.prec == P_FP32) {
            const float* base = (const float*)op.ptr + rowoff;
            if (op.vec && d0 + 8 <= D) {
              v = *reinterpret_cast<const uint4*>(base + d0);
              v2 = *reinterpret_cast<const uint4*>(base + d0 + 4);
            } else {
              auto e = [&](int j) -> uint32_t {
                return d0 + j < D ? __builtin_bit_cast(uint32_t, base[(int64_t)(d0 + j) * op.sd]) : 0u;
              };
              v = make_uint4(e(0), e(1), e(2), e(3));
              v2 = make_uint4(e(4), e(5), e(6), e(7));
            }
          } else {
            const uint16_t* p = (const uint16_t*)op.ptr + rowoff;
            if (op.vec && d0 + 8 <= D) {
              v = *reinterpret_cast<const uint4*>(p + d0);
            } else {
              v = gather16(p, d0, D, op.sd);
            }
          }
        } else if constexpr (SRC == SRC_SAME) {
          const char* base = (const char*)op.ptr + rowoff * A::ESIZE;
          if (op.vec && d0 + CE <= D) {
            v = *reinterpret_cast<const uint4*>(base + (int64_t)d0 * A::ESIZE);
          } else if constexpr (A::ESIZE == 2) {
            v = gather16((const uint16_t*)base, d0, D, op.sd);
          } else {
            const uint32_t* p = (const uint32_t*)base;
            auto e = [&](int j) -> uint32_t { return d0 + j < D ? p[(int64_t)(d0 + j) * op.sd] : 0u; };
            v = make_uint4(e(0), e(1), e(2), e(3));
          }
        } else {
          v = load_qchunk<SRC>(op, rowoff, d0, D);
        }
      }
      // One unconditional assignment per register array (assignments in the branches above
      // made hipcc keep raw2 in scratch).
      raw[i] = v;
      if constexpr (SRC == SRC_F32ANY) raw2[i] = v2;
    }
  }

  __device__ __forceinline__ void store(char* tile, const Operand& op, int b, int hx, int row0,
                                        int nrows, int D) const {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + i * NT;
      if (NCH % NT != 0 && id >= NCH) continue;
      const int r = id / CPR, c = id % CPR;
      if constexpr (A::is_f32) {
        float* t = reinterpret_cast<float*>(tile) + r * (DP + 1) + c * 4;
        t[0] = __builtin_bit_cast(float, raw[i].x);
        t[1] = __builtin_bit_cast(float, raw[i].y);
        t[2] = __builtin_bit_cast(float, raw[i].z);
        t[3] = __builtin_bit_cast(float, raw[i].w);
      } else {
        uint4 out;
        if constexpr (SRC == SRC_SAME) {
          out = raw[i];
        } else if constexpr (SRC == SRC_F32ANY) {
          if (op.prec == P_FP32) {
            const uint32_t f[8] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w,
                                   raw2[i].x, raw2[i].y, raw2[i].z, raw2[i].w};
            uint32_t w[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              w[jj] = (uint32_t)A::Elem::from_f32(__builtin_bit_cast(float, f[2 * jj])) |
                      ((uint32_t)A::Elem::from_f32(__builtin_bit_cast(float, f[2 * jj + 1])) << 16);
            out = make_uint4(w[0], w[1], w[2], w[3]);
          } else {
            out = raw[i];
          }
        } else {
          // Per-tensor: the exact integers (q - zp); zero-filled loads beyond the tile edge
          // only ever meet zero Q columns or masked keys.
          const int grow = row0 + r;
          const int64_t hrow = op.bscale ? quant_row(op, b, hx) : 0;
          out = convert_qchunk<typename A::Elem, SRC>(raw[i], op, hrow, grow, c * 8, D, grow < nrows);
        }
        *reinterpret_cast<uint4*>(tile + A::TileT::off(r, c)) = out;
      }
    }
  }
};

// Register fragments of a row operand kept for the whole kernel (B operand of S^T = K·Q^T):
// lane l holds row `row` (= its query), elements d = KSTEP*s + (KSTEP/2)*h + j.
template <class A, int DP>
__device__ __forceinline__ void load_row_frags(typename A::frag (&f)[A::DSTEPS],
                                               const Operand& op, int b, int hx, int row,
                                               bool valid, int h, int D) {
  const int64_t rowoff = (int64_t)b * op.sb + (int64_t)hx * op.sh + (int64_t)row * op.ss;
  if constexpr (A::is_f32) {
    const float* base = (const float*)op.ptr + rowoff;
#pragma unroll
    for (int s = 0; s < A::DSTEPS; ++s) {
      const int d = 2 * s + h;
      f[s] = (valid && d < D) ? base[(int64_t)d * op.sd] : 0.f;
    }
  } else {
    const int64_t hrow = (op.prec == P_INT8 || op.prec == P_INT4) ? quant_row(op, b, hx) : 0;
#pragma unroll
    for (int s = 0; s < A::DSTEPS; ++s) {
      const int d0 = 16 * s + 8 * h;
      i16x8 v;
      if (op.prec == P_INT8 || op.prec == P_INT4) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float x = 0.f;
          if (valid && d0 + j < D) {
            const int64_t e = rowoff + (int64_t)(d0 + j) * op.sd;
            const int qv = op.prec == P_INT8 ? (int)((const int8_t*)op.ptr)[e]
                                             : (int)ld_i4((const uint8_t*)op.ptr, e);
            x = dequant(op, qv, hrow, row, d0 + j);
          }
          v[j] = (short)A::Elem::from_f32(x);
        }
      } else if (op.prec == P_FP32) {
        const float* base = (const float*)op.ptr + rowoff;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          v[j] = (short)A::Elem::from_f32((valid && d0 + j < D) ? base[(int64_t)(d0 + j) * op.sd] : 0.f);
      } else {
        const uint16_t* base = (const uint16_t*)op.ptr + rowoff;
        if (valid && op.vec && d0 + 8 <= D) {
          v = *reinterpret_cast<const i16x8*>(base + d0);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            v[j] = (valid && d0 + j < D) ? (short)base[(int64_t)(d0 + j) * op.sd] : (short)0;
        }
      }
      f[s] = v;
    }
  }
}


// LDS-DMA of one [BK rows][ROWB bytes] tile (buffer_load ... lds, one 1-KiB piece per
// wave-instruction) straight into the Tile16 XOR-swizzled layout: no staging registers, no
// ds_write.  A piece covers RP = 1024/ROWB rows; lane l lands at byte 16*l of it (row
// n*RP + l/CPR, physical chunk l%CPR) and so fetches the logical chunk (l%CPR) ^ swz(row).
// Wave w of the NT/64 staging waves issues pieces n = w + NW*i; the swizzle depends only on
// row & 15, so each wave needs a single lane offset.  Rows past the end and chunks past the
// row's valid bytes read as zeros: the range-checked descriptor is rebuilt per piece from
// wave-uniform values (base at the piece's first row, num_records = bytes left).
// One LDS-DMA wave-instruction: 16 bytes per lane from base + voff (range-checked against
// nrec bytes; out of range reads zero) into dst + 16*lane.  Issued as inline asm so that
// hipcc knows nothing of the LDS write: with the builtin it guards later ds_reads with
// vmcnt(0) (it cannot tell the ring slot being filled from the slot being read), which exposes
// the prefetch latency every tile; callers order tiles with wait_vm() + a barrier.
__device__ __forceinline__ void lds_dma16(const void* base, int nrec, int voff, char* dst) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t a = (uint64_t)(uintptr_t)base;
  u32x4 rs;
  rs[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  rs[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);
  rs[2] = __builtin_amdgcn_readfirstlane((unsigned)nrec);
  rs[3] = 0x00020000u;
  // The low 32 bits of a generic LDS pointer are its LDS address; an explicit address-space
  // cast here can make the selector emit a null check on the shared aperture it then fails
  // to encode ("V_CMP_NE_U32 0, $src_shared_base").
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rs), "s"(lds)
               : "memory", "m0");
}

template <int ROWB, int BK, int NT>
struct TileDMA {
  using T = Tile16<ROWB / 2>;
  static constexpr int NW = NT / 64;
  static constexpr int CPR = ROWB / 16;
  static constexpr int RP = 1024 / ROWB;
  static constexpr int NPIECE = BK * ROWB / 1024;
  static constexpr int PPW = NPIECE / NW;
  static_assert(NPIECE % NW == 0 && (NW * RP) % 16 == 0, "DMA geometry");
  const char* base;
  int step, bytes, off, w;

  // head: first byte of the (batch, head) slice; step: bytes per row; rowbytes: valid bytes
  // per row (D * element size); gt: thread index within the staging waves.
  __device__ __forceinline__ void init(const char* head, int step_, int C, int rowbytes, int gt) {
    base = head;
    step = step_;
    bytes = (int)((int64_t)(C - 1) * step_ + rowbytes);
    w = __builtin_amdgcn_readfirstlane(gt >> 6);
    const int l = gt & 63;
    const int rl = l / CPR, pc = l % CPR;
    const int ch = pc ^ T::swz(w * RP + rl);
    off = ch * 16 < rowbytes ? rl * step + ch * 16 : 0x40000000;
  }
  __device__ __forceinline__ void issue(int t, char* dst) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int n = w + NW * i;
      const int rb = (t + n * RP) * step;
      lds_dma16(base + rb, max(bytes - rb, 0), off, dst + n * 1024);
    }
  }
};

// LDS-DMA of one [ROWS][DP] 16-bit tile into the TileA image (buffer_load ... lds, one 1-KiB
// piece per wave-instruction, lane l landing at byte 16*l of its piece), for a base pointer
// that may change from tile to tile (the kv group's query heads).  Piece n is half of 8-row
// block n / (DP/64): its two 512-B sub-tiles (column blocks 2*(n % (DP/64)) and +1), so lane
// l fetches row 8*(n / (DP/64)) + (l & 31)/4, logical chunk 4*sub + ((l & 3) ^ ((row>>2)&3)).
// Rows past nrows and chunks past rowbytes read as zeros (range-checked descriptor rebuilt
// per piece from wave-uniform values; out-of-row chunks get an out-of-range offset).
template <int DP, int ROWS, int NT>
struct DmaA {
  static constexpr int NW = NT / 64;
  static constexpr int PPRB = DP / 64;                 // pieces per 8-row block
  static constexpr int NPIECE = ROWS * DP * 2 / 1024;
  static constexpr int PPW = NPIECE / NW;
  static_assert(DP % 64 == 0 && NPIECE % NW == 0 && PPW >= 1, "DMA geometry");
  int step, bytes, w;
  int off[PPW];

  __device__ __forceinline__ void init(int step_, int nrows, int rowbytes, int gt) {
    step = step_;
    bytes = (int)((int64_t)(nrows - 1) * step_ + rowbytes);
    w = __builtin_amdgcn_readfirstlane(gt >> 6);
    const int l = gt & 63;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int n = w + NW * i;
      const int rblk = n / PPRB, sub = 2 * (n % PPRB) + (l >> 5);
      const int r7 = (l & 31) >> 2;
      const int ch = 4 * sub + ((l & 3) ^ ((2 * rblk + (r7 >> 2)) & 3));
      off[i] = ch * 16 < rowbytes ? (rblk * 8 + r7) * step + ch * 16 : 0x40000000;
    }
  }
  __device__ __forceinline__ void issue(const char* head, int t, char* dst) const {
#pragma unroll
    for (int i = 0; i < PPW; ++i) issue_piece(head, t, dst, i);
  }
  // Piece i (< PPW) of this wave's share alone: spread over the MFMAs of a chain, each
  // piece's issue cost hides in an MFMA gap instead of queueing behind the others.
  __device__ __forceinline__ void issue_piece(const char* head, int t, char* dst, int i) const {
    const int n = w + NW * i;
    const int rb = t * step;
    lds_dma16(head + rb, max(bytes - rb, 0), off[i], dst + n * 1024);
  }
};

// Forward masks on NJ 32-key accumulators of S^T (key in registers, query qi on the lane):
// keys past C -> -inf; additive mask; causal / window / sparse-range predicates -> the
// reference's finite mask value (AttentionKernel+Softmax.swift:243-336).
template <int NJ>
__device__ __forceinline__ void apply_masks(f32x16 (&s)[NJ], int kbase, int qi, int hh,
                                            const FwdParams& p, int b, int h, uint2 range) {
  const bool qvalid = qi < p.R;
  const float* arow =
      (p.mask.amask && qvalid) ? p.mask.amask + ((int64_t)(b * p.H + h) * p.R + qi) * p.C : nullptr;
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int key = kbase + j * 32 + acc_row(i, hh);
      float x = s[j][i];
      if (key >= p.C) {
        x = -__builtin_inff();
      } else {
        if (arow) x += arow[key];
        bool m = false;
        if (p.mask.causal && key > qi) m = true;
        if (p.mask.window && (int64_t)qi > (int64_t)key + (int64_t)p.mask.window_size) m = true;
        if (p.mask.ranges && ((uint32_t)key < range.x || (uint32_t)key >= range.y)) m = true;
        if (m) x = kMaskValue;
      }
      s[j][i] = x;
    }
  }
}

// Wait for this wave's outstanding vector-memory operations (LDS-DMA included): vmcnt(0),
// expcnt / lgkmcnt untouched (gfx9 s_waitcnt encoding).
__device__ __forceinline__ void wait_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

}  // namespace mfa
