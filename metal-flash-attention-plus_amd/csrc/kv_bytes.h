// kv_bytes.h — per-tensor quantised K/V tiles widened into the 16-bit TileA image inside the
// tuned loops (attention_fwd_kv8.hip, attention_bwd_fast.hip): the reference dequantises K/V
// tiles as it loads them (GEMMHeaders.swift:679-808).  Shared pieces: one chunk's widening
// (mfa_stage.h dequant_fast), the chunk geometry of a tile over 512 thread slots, a 4-byte
// LDS-DMA, and KvBytes, the LDS byte ring (LDS-DMA of the stored bytes, widened LDS -> LDS).
#pragma once
#include "mfa_stage.h"

namespace mfa {

// 8 quantised elements -> 16-byte chunk `ch` of row r of the TileA image.
// INT8: raw holds up to 16 bytes (half h: dwords 2h, 2h+1); INT4: up to 16 nibbles in raw.x,
// raw.y (half h: dword h, element 2i in the low nibble).
template <class E, int DP, int SRC, int HALF>
__device__ __forceinline__ void widen_store(char* img, int r, int ch, const uint4 raw, float zp) {
  uint4 q;
  if constexpr (SRC == SRC_I8)
    q = HALF ? make_uint4(raw.z, raw.w, 0u, 0u) : make_uint4(raw.x, raw.y, 0u, 0u);
  else
    q = make_uint4(HALF ? raw.y : raw.x, 0u, 0u, 0u);
  *reinterpret_cast<uint4*>(img + TileA<DP>::off(r, ch)) = dequant_fast<E, SRC>(q, zp);
}

// Blockwise-scaled chunk (round 6): 8 quantised elements of one scale block -> the 16-bit
// TileA chunk holding (q - zp) * s rounded to E, as the dequantisation pass writes it
// (mfa_stage.h convert_qchunk / dequant: (float)(q - zp) exact, one FP32 multiply, one rounding
// to FP16 / BF16), so the MFMA operands are bit-identical to the pass's.  An invalid chunk (rows
// past the operand's end, columns past D) is zero, as the pass's zero-filled copy reads.
//   FP16, |zp| <= 896: q - zp exact in FP16 by dequant_fast (|q - zp| <= 1024), then
//     v_fma_mix_f32 (FP16 operand x FP32 scale + 0: the FP32-rounded product) and one packed
//     conversion: about 2 VALU per element;
//   otherwise (BF16, or a zero point past that): q - zp in FP32 (byte -> float, subtract), the
//     FP32 multiply, the conversion: about 3.5 per element.
template <class E, int SRC, int HALF>
__device__ __forceinline__ uint4 widen_block(const uint4 raw, float s, float zp, bool valid) {
  uint32_t o[4];
  // (Both forms give the same bits, so the choice is made per wave: a branch, not a select.)
  if (E::prec == P_FP16 && __all(fabsf(zp) <= 896.f)) {
    uint4 q;
    if constexpr (SRC == SRC_I8)
      q = HALF ? make_uint4(raw.z, raw.w, 0u, 0u) : make_uint4(raw.x, raw.y, 0u, 0u);
    else
      q = make_uint4(HALF ? raw.y : raw.x, 0u, 0u, 0u);
    const uint4 n = dequant_fast<F16, SRC>(q, zp);
    const uint32_t nw[4] = {n.x, n.y, n.z, n.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f16x2 v = __builtin_bit_cast(f16x2, nw[k]);
      o[k] = pack_f16x2(__builtin_fmaf((float)v[0], s, 0.f), __builtin_fmaf((float)v[1], s, 0.f));
    }
  } else {
    const float m = (SRC == SRC_I8 ? 128.f : 8.f) + zp;
    float f[8];
    if constexpr (SRC == SRC_I8) {
      const uint32_t u0 = (HALF ? raw.z : raw.x) ^ 0x80808080u;
      const uint32_t u1 = (HALF ? raw.w : raw.y) ^ 0x80808080u;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f[k] = (float)((u0 >> (8 * k)) & 0xffu) - m;
        f[4 + k] = (float)((u1 >> (8 * k)) & 0xffu) - m;
      }
    } else {
      const uint32_t w = HALF ? raw.y : raw.x;
#pragma unroll
      for (int k = 0; k < 8; ++k) f[k] = (float)((w >> (4 * k)) & 15u) - m;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // (mul_rn: no contraction with the conversion into one rounding; see mfa_stage.h dequant.)
      const float a = mul_rn(f[2 * k], s), b = mul_rn(f[2 * k + 1], s);
      if constexpr (E::prec == P_FP16)
        o[k] = pack_f16x2(a, b);  // round to nearest even, as convert_qchunk
      else
        o[k] = (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);  // v_cvt_pk_bf16_f32
    }
  }
  return valid ? make_uint4(o[0], o[1], o[2], o[3]) : make_uint4(0u, 0u, 0u, 0u);
}

// Scale-block row index of a chunk's row, advanced one key tile (bk rows) at a time: the row
// block q = row / bs and the row's place r = row % bs in it, without a division per tile.
struct BlockRow {
  int q, r;
  __device__ __forceinline__ void init(int64_t row, int bs) {
    q = (int)(row / bs);
    r = (int)(row - (int64_t)q * bs);
  }
  __device__ __forceinline__ void advance(int bk, int bs) {
    r += bk;
    if (bs >= bk) {  // at most one block boundary per tile: no loop
      const bool w = r >= bs;
      r -= w ? bs : 0;
      q += w ? 1 : 0;
    } else {
      while (r >= bs) {
        r -= bs;
        ++q;
      }
    }
  }
};

// One LDS-DMA wave-instruction of 4 bytes per lane (buffer_load_dword ... lds): lane l's dword
// from base + voff lands at dst + 4·l (range-checked against nrec bytes, zeros past it).
__device__ __forceinline__ void lds_dma4(const void* base, int nrec, int voff, char* dst) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const uint64_t a = (uint64_t)(uintptr_t)base;
  u32x4 rs;
  rs[0] = __builtin_amdgcn_readfirstlane((unsigned)a);
  rs[1] = __builtin_amdgcn_readfirstlane((unsigned)(a >> 32) & 0xffffu);
  rs[2] = __builtin_amdgcn_readfirstlane((unsigned)nrec);
  rs[3] = 0x00020000u;
  const unsigned lds = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)dst);
  asm volatile("s_mov_b32 m0, %2\n\tbuffer_load_dword %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(rs), "s"(lds)
               : "memory", "m0");
}

// Geometry of one thread's share of a staged tile: CE = BK·DP / 512 elements (16: one 16-byte
// INT8 chunk = two TileA chunks; 8 at D = 64: one TileA chunk), at row `r`, TileA chunks
// ch0 (and ch0 + 1).  Each 16-lane quarter of a wave writes 8 rows x 2 chunks whose slots
// (64·(r & 7) + 16·(chunk & 3 ^ (r >> 2 & 3)) within a 512-byte sub-tile) are 16 distinct bank
// groups: chunk pairs {2c, 2c + 1} x 2 c-parities for CE = 16, {j, j + 2} for CE = 8.
template <int DP, int BK>
struct Kv8Geo {
  static constexpr int NT = 512;
  static constexpr int CE = BK * DP / NT;
  static_assert(CE == 16 || CE == 8, "8 or 16 elements per thread per tile");
  static_assert(CE == 8 || (BK % 8 == 0 && NT / 64 % (BK / 8) == 0), "row groups");
  int r, ch0, col;
  __device__ __forceinline__ Kv8Geo(int tid) {
    const int lane = tid & 63, w = tid >> 6;
    if constexpr (CE == 16) {
      constexpr int RG = BK / 8;  // 8-row groups per tile; waves beyond them take the next
                                  // 8 chunks of the same rows
      const int cc = (((lane >> 3) & 1) | ((lane >> 4) << 1)) + 8 * (w / RG);
      r = (w % RG) * 8 + (lane & 7);
      ch0 = 2 * cc;
      col = 16 * cc;
    } else {
      r = w * 8 + (lane & 7);
      ch0 = ((lane >> 3) & 1) * 2 + ((lane >> 4) & 1) + 4 * (lane >> 5);
      col = 8 * ch0;
    }
  }
};

// LDS byte ring of quantised K/V tiles for an NT-thread workgroup (NT = 256 or 512): each
// thread owns 512 / NT of the 512 chunk slots of Kv8Geo.  A slot's bytes move by LDS-DMA
// (one 16-byte piece per lane, or 4-byte pieces) into a region only its own wave reads, so a
// counted vmcnt wait orders them; the widening then writes the 16-bit image (a barrier orders
// that for the readers).  Rows past the operand's end and chunks past D widen to 0 (the
// stored-byte zero fill would decode to -zp), as the 16-bit tiles' zero fill gives.
template <class E, int DP, int BK, int SRC, int NT>
struct KvBytes {
  static constexpr int NV = 512 / NT;
  using G = Kv8Geo<DP, BK>;
  static constexpr int CE = G::CE;
  static constexpr int SH = SRC == SRC_I8 ? 0 : 1;
  static constexpr int CB = CE >> SH;               // stored bytes per chunk
  static constexpr int NPC = CB == 16 ? 1 : CB / 4; // DMA wave-instructions per chunk slot
  static constexpr int SLOT = 512 * CB;             // bytes per staged tile of one operand
  static constexpr int NH = CE / 8;                 // TileA chunks per slot
  static constexpr int NPIECE = NV * NH;            // widening pieces per operand per tile
  int r[NV], ch0[NV], off[NV], vw[NV];
  bool cv[NV];
  int lane;

  // ss: stored bytes per row.
  __device__ __forceinline__ void init(int tid, int D, int ss) {
    lane = tid & 63;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int vt = tid + k * NT;
      const G g(vt);
      r[k] = g.r;
      ch0[k] = g.ch0;
      cv[k] = g.col < D;
      vw[k] = __builtin_amdgcn_readfirstlane(vt >> 6);
      off[k] = cv[k] ? g.r * ss + (g.col >> SH) : 0x40000000;
    }
  }
  // Tile starting at row t of the head at `head` (bytes `bytes` in all, `ss` per row) -> slot.
  __device__ __forceinline__ void dma(const char* head, int ss, int bytes, int t, char* slot) const {
    const int tb = t * ss;
    const int left = max(bytes - tb, 0);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if constexpr (CB == 16) {
        lds_dma16(head + tb, left, off[k], slot + vw[k] * 1024);
      } else {
#pragma unroll
        for (int j = 0; j < NPC; ++j)
          lds_dma4(head + tb, left, off[k] + 4 * j, slot + j * 2048 + vw[k] * 256);
      }
    }
  }
  // Piece m (slot k = m / NH, half hf = m % NH): its stored bytes, as widen_store's half 0.
  __device__ __forceinline__ uint4 read(const char* slot, int m) const {
    const int k = m / NH, hf = m % NH;
    if constexpr (CB == 16) {
      const uint2 a = *reinterpret_cast<const uint2*>(slot + vw[k] * 1024 + lane * 16 + 8 * hf);
      return make_uint4(a.x, a.y, 0u, 0u);
    } else {
      // 4-byte pieces: a half spans NPC / NH of them (INT8 at CE = 8: both of the chunk's).
      constexpr int PH = NPC / NH;
      uint32_t w[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < PH; ++j)
        w[j] = *reinterpret_cast<const uint32_t*>(slot + (hf * PH + j) * 2048 + vw[k] * 256 +
                                                  lane * 4);
      return make_uint4(w[0], w[1], 0u, 0u);
    }
  }
  // Piece m widened into the 16-bit image; rows at or past `rows` (rows left in the operand
  // from the tile's first row) and chunks past D give zeros.
  __device__ __forceinline__ void widen(char* img, const uint4 raw, float zp, int m, int rows) const {
    const int k = m / NH, hf = m % NH;
    uint4 w = dequant_fast<E, SRC>(raw, zp);
    if (!(cv[k] && r[k] < rows)) w = make_uint4(0u, 0u, 0u, 0u);
    *reinterpret_cast<uint4*>(img + TileA<DP>::off(r[k], ch0[k] + hf)) = w;
  }
};

}  // namespace mfa
