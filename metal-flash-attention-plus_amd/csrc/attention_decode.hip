// attention_decode.hip — split-KV forward for INT8 K/V with few query rows per kv head
// (decode / KV-cache shapes): QuantizedAttention.forward (QuantizedAttention.swift:135-263)
// with the reference's dequantise-on-load semantics (GEMMHeaders.swift:679-738): every K/V
// element enters the product as (q - zp) exactly, the per-tensor scales folded into the
// softmax and output multipliers, as in the other dequant-exact kernels.
//
// A decode step reads the whole K/V cache to serve 1-16 query rows per head, so the kernel is
// HBM-bound: 2·D bytes per key.  Layout of the work:
//   * unit = (batch, kv head, 32-row tile of the kv group's query rows); the group's rows
//     (H/H_kv query heads x R rows) share every K/V byte, so a tile reads them once;
//   * each unit's keys are split over `nsplit` workgroups of 4 waves; inside a workgroup the
//     waves take 32-key tiles round-robin, each wave with its own 2-slot LDS ring filled by
//     LDS-DMA of the INT8 bytes (1 KiB per wave-instruction; no staging registers, no
//     barriers: a wave waits for its own DMA with a counted vmcnt);
//   * S^T = K·Q^T on v_mfma_f32_32x32x16 with K fragments widened from INT8 in registers
//     (the exact fp16 magic-number conversion of mfa_stage.h); online softmax per wave; V^T
//     fragments read transposed from the INT8 tile (ds_read_b64_tr_b8) and widened the same
//     way for O^T += V^T·P^T;
//   * the 4 waves' partials (m, l, unnormalised O) meet in LDS; with several key splits the
//     workgroup writes one combined partial per valid row, and a merge pass combines the
//     nsplit partials of each row into O = Σ w_s O_s / Σ w_s l_s and L = m + log2 l
//     (w_s = exp2(m_s - m)), one row per wave (batched loads), or per 4-wave workgroup above
//     32 splits.  With one split per unit (the B32 H16 decode rows) the workgroup merges its
//     waves into O and L itself: one launch, the same arithmetic in the same order.
// Units with at most 16 rows (the usual decode step) run mfa_fwd_decode16_kernel below: the
// same layout on 16x16x32 MFMAs, K rows straight from HBM to registers (see its comment).
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

typedef int i32x2d __attribute__((ext_vector_type(2)));

template <class E>
__device__ __forceinline__ i16x8 widen_i8(uint32_t lo, uint32_t hi, float zp) {
  return __builtin_bit_cast(i16x8, dequant_fast<E, SRC_I8>(make_uint4(lo, hi, 0u, 0u), zp));
}

// INT4 K fragments straight from the packed tile: 8 nibbles (n0 in the low nibble) -> 8 MFMA
// elements n - 8 - zp (zk4 = zp + 8).  FP16: v_perm places the even nibbles n0 n2 n4 n6 and
// the odd ones n1 n3 n5 n7 as the low bytes of 1024 + n (0x64nn) — one v_perm per pair, then a
// packed subtract: the fragment holds the elements in the order kI4Perm, which the Q fragments
// are loaded in too (the contraction over d does not care which lane slot holds which d, only
// that Q and K agree).  BF16: natural order, f32 route as in mfa_stage.h dequant_fast.
template <class E>
__device__ __forceinline__ i16x8 nib_widen(uint32_t x, float zk4) {
  if constexpr (E::prec == P_FP16) {
    const uint32_t lo = x & 0x0F0F0F0Fu, hi = (x >> 4) & 0x0F0F0F0Fu;
    uint32_t w[4] = {__builtin_amdgcn_perm(0x64646464u, lo, 0x04010400u),
                     __builtin_amdgcn_perm(0x64646464u, lo, 0x04030402u),
                     __builtin_amdgcn_perm(0x64646464u, hi, 0x04010400u),
                     __builtin_amdgcn_perm(0x64646464u, hi, 0x04030402u)};
    const _Float16 m = (_Float16)(1024.0f + zk4);
    const f16x2 mm = {m, m};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      w[k] = __builtin_bit_cast(uint32_t, __builtin_bit_cast(f16x2, w[k]) - mm);
    return __builtin_bit_cast(i16x8, make_uint4(w[0], w[1], w[2], w[3]));
  } else {
    return __builtin_bit_cast(i16x8, dequant_fast<E, SRC_I4>(make_uint4(x, 0u, 0u, 0u), zk4 - 8.0f));
  }
}

// Q fragment slot j holds element kI4Perm[j] of its 8-element group (FP16 INT4 K: the order
// nib_widen produces).
template <class E>
__device__ __forceinline__ i16x8 i4_order(i16x8 v) {
  if constexpr (E::prec == P_FP16)
    return __builtin_shufflevector(v, v, 0, 2, 4, 6, 1, 3, 5, 7);
  else
    return v;
}

// Merge of split partials (m_s, l_s, O_s) of one query row, columns d .. d+3:
// O = Σ w_s O_s / (Σ w_s l_s + FLT_MIN), w_s = exp2(m_s - max m), L = max m + log2 l.  Partial s
// is ml[s·mls] and the D floats at op + s·ops (global memory for the merge pass, LDS for the
// in-workgroup merge).  Loads go in batches of SB partials, all issued before any is used (a
// one-partial-at-a-time loop is a chain of memory latencies: the merge pass took as long as the
// split kernel at 64 partials per row); partials are summed in order.
constexpr int kMergeSB = 16;

__device__ __forceinline__ float merge_max(const float2* ml, int64_t mls, int np) {
  float mx = -kFltMax;
  for (int s0 = 0; s0 < np; s0 += kMergeSB) {
    float mb[kMergeSB];
#pragma unroll
    for (int u = 0; u < kMergeSB; ++u) mb[u] = s0 + u < np ? ml[(s0 + u) * mls].x : -kFltMax;
#pragma unroll
    for (int u = 0; u < kMergeSB; ++u) mx = fmaxf(mx, mb[u]);
  }
  return mx;
}

__device__ __forceinline__ void merge_sum(const FwdParams& p, const float2* ml, int64_t mls,
                                          const float* op, int64_t ops, int np, float mx, int d,
                                          float& l, float4& acc) {
  for (int s0 = 0; s0 < np; s0 += kMergeSB) {
    float2 mlb[kMergeSB];
    float4 vb[kMergeSB];
#pragma unroll
    for (int u = 0; u < kMergeSB; ++u) {
      const bool in = s0 + u < np;
      mlb[u] = in ? ml[(s0 + u) * mls] : make_float2(-kFltMax, 0.f);
      vb[u] = in && d < p.D ? *reinterpret_cast<const float4*>(op + (s0 + u) * ops + d)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kMergeSB; ++u) {
      if (s0 + u < np) {
        const float w = __builtin_amdgcn_exp2f(mlb[u].x - mx);
        l += mlb[u].y * w;
        if (d < p.D) {
          acc.x += vb[u].x * w; acc.y += vb[u].y * w; acc.z += vb[u].z * w; acc.w += vb[u].w * w;
        }
      }
    }
  }
}

__device__ __forceinline__ void merge_store(const FwdParams& p, float4 acc, float l, float mx,
                                            int b, int h, int q, int d, bool write_l) {
  l += kFltMin;
  const float inv = p.o_mul / l;
  float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)q * p.o_ss;
  const float vals[4] = {acc.x * inv, acc.y * inv, acc.z * inv, acc.w * inv};
#pragma unroll
  for (int e = 0; e < 4; ++e)
    if (d + e < p.D) orow[(int64_t)(d + e) * p.o_sd] = vals[e];
  if (write_l) {
    const float L = mx + __log2f(l);
    const int64_t li = (int64_t)(b * p.H + h) * p.R + q;
    if (p.l_f16)
      reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
    else
      reinterpret_cast<float*>(p.l)[li] = L;
  }
}

__device__ __forceinline__ void merge_partials(const FwdParams& p, const float2* ml, int64_t mls,
                                               const float* op, int64_t ops, int np, int b,
                                               int h, int q, int d, bool write_l) {
  const float mx = merge_max(ml, mls, np);
  float l = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  merge_sum(p, ml, mls, op, ops, np, mx, d, l, acc);
  merge_store(p, acc, l, mx, b, h, q, d, write_l);
}

// The workgroup's partial of one row (split `split` of unit u) from its 4 waves' partials in
// LDS: (max m, Σ w l, Σ w O) with the merge's weights and order, columns d .. d+3.
__device__ __forceinline__ void store_split_partial(const FwdParams& p, const DecodeParams& dp,
                                                    const float2* ml, int64_t mls,
                                                    const float* op, int64_t ops, int u,
                                                    int split, int r, int d) {
  const float mx = merge_max(ml, mls, 4);
  float l = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  merge_sum(p, ml, mls, op, ops, 4, mx, d, l, acc);
  const int64_t pidx = ((int64_t)u * dp.nsplit + split) * 32 + r;
  if (d < p.D) *reinterpret_cast<float4*>(dp.opart + pidx * p.D + d) = acc;
  if (d == 0) dp.mlpart[pidx] = make_float2(mx, l);
}

// s_waitcnt immediate for vmcnt(n) alone (n < 64: bits 3:0 and 15:14).
constexpr int vm_wait(int n) { return 0x0F70 | (n & 15) | ((n >> 4) << 14); }

// SRC_I8: one byte per element.  SRC_I4: two per byte (element 2i in the low nibble,
// GEMMQuantization.swift:500-515), staged by LDS-DMA as stored.  K fragments are widened from
// the packed tile in registers (nib_widen; each lane reads 16 consecutive elements = 8 bytes
// for two k-steps, so the lane's k-step st covers d = 32·(st / 2) + 16·hh + 8·(st % 2) + j and
// Q is loaded in that order; the packed K rows land XOR-swizzled by 16-byte chunk); V^T
// fragments come straight from the packed V tile (same swizzle) by ds_read_b64_tr_b4 and are
// widened in registers the same way (the zero point raised by 8: the nibble encodes n - 8).
template <class E, int DP, int SRC = SRC_I8>
__global__ void __launch_bounds__(256, DP >= 256 ? 1 : 2) mfa_fwd_decode_kernel(DecodeParams dp) {
  const FwdParams& p = dp.f;
  constexpr bool I4 = SRC == SRC_I4;
  // INT4 keeps three tiles in flight (four ring slots in the INT8 ring's bytes: the packed
  // tiles are half as large, and V is read from the packed tile too).
  constexpr int BK = 32, NSLOT = SRC == SRC_I4 ? 4 : 2, ND = DP / 32;
  constexpr int ROWB = DP;                  // INT8 compute tile: one byte per element
  using T = Tile16<ROWB / 2>;               // [BK][ROWB bytes], 16-byte chunks XOR-swizzled
  constexpr int TILEB = BK * ROWB;          // one K or V compute tile
  constexpr int ROWBS = I4 ? DP / 2 : DP;   // bytes per stored row
  constexpr int TILEBS = BK * ROWBS;        // one stored (DMA) tile
  constexpr int NPC = TILEBS / 1024;        // 1-KiB DMA pieces per tile
  constexpr int RP = 1024 / ROWBS;          // rows per piece
  static_assert(NPC >= 1 && NPC <= 8, "decode tile geometry");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  // Per wave: NSLOT DMA slots (K at 2s·TILEBS, V after it): 4·TILEB in all for both.
  constexpr int WREG = NSLOT * 2 * TILEBS;
  static_assert(WREG == 4 * TILEB, "per-wave LDS region");
  char* const ring = smem + wave * WREG;

  const int split = blockIdx.x;
  const int u = blockIdx.y + gridDim.y * blockIdx.z;    // (b·H_kv + kvh)·nrt + rt
  const int rt = u % dp.nrt;
  const int bk = u / dp.nrt;
  const int kvh = bk % p.Hkv, b = bk / p.Hkv;
  const float c = p.c_log2;

  // The lane's query row of this tile: row = g·R + q of kv head kvh's group (h = kvh + g·H_kv).
  const int row = rt * 32 + l32;
  const bool rvalid = row < dp.rows;
  i16x8 qf[DP / 16];
  // Causal: the lane's query index sees keys 0 .. qcol (the host caps C at R, past which no
  // row sees a key).
  const int qcol = rvalid ? row % p.R : 0x3fffffff;
  // Sliding window (mask row > key + window): the lane's first visible key (host: skip_ok).
  const int wlo = p.mask.window ? qcol - (int)min(p.mask.window_size, 0x3fffffffu) : -0x40000000;
  {
    const int g = rvalid ? row / p.R : 0, q = rvalid ? row % p.R : 0;
    const int h = kvh + g * p.Hkv;
    const uint16_t* qrow =
        (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh + (int64_t)q * p.q.ss;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const int d0 = I4 ? 32 * (s >> 1) + 16 * hh + 8 * (s & 1) : 16 * s + 8 * hh;
      i16x8 v = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (rvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
      qf[s] = I4 ? i4_order<E>(v) : v;
    }
  }

  // Keys of this split: [k0, k1); this wave's tiles k0 + 32·(wave + 4i).
  const int k0 = split * dp.chunk;
  const int k1 = min(p.C, k0 + dp.chunk);
  const int nt = k1 > k0 ? (k1 - k0 + BK - 1) / BK : 0;
  const int mine = nt > wave ? (nt - wave + 3) / 4 : 0;

  // LDS-DMA of one 32-row tile: piece n holds rows n·RP .. n·RP + RP - 1 (Tile16 rows are
  // contiguous); lane l lands at byte 16·l of it = row n·RP + l / CPR, physical chunk l % CPR,
  // so it fetches logical chunk (l % CPR) ^ swz(row).  Rows past C and chunks past D read as
  // zeros (range-checked descriptor per piece, out-of-row chunks out of range).
  constexpr int CPR = ROWBS / 16;
  constexpr int SH = I4 ? 1 : 0;  // element -> byte offsets
  // Packed INT4 K rows: 16-byte chunk c of row r at physical chunk c ^ swz4(r), so the 8-byte
  // fragment reads of a half-wave (32 rows, one chunk) spread over 16 slots (2-way at most).
  auto swz4 = [](int r) {
    if constexpr (CPR == 2) return (r >> 3) & 1;
    else if constexpr (CPR == 4) return (r >> 2) & 3;
    else return (((r >> 1) & 1) << 2) | ((r >> 2) & 3);
  };
  const int ssb = (int)(p.k.ss >> SH);
  int poff[NPC], voff[NPC];
#pragma unroll
  for (int n = 0; n < NPC; ++n) {
    const int r = n * RP + lane / CPR;
    const int ch = I4 ? (lane % CPR) ^ swz4(r) : (lane % CPR) ^ T::swz(r);
    poff[n] = ch * 16 < (p.D >> SH) ? r * ssb + ch * 16 : 0x40000000;
    // V: the same chunk placement as K (INT4: the transposed 4-bit reads below).
    voff[n] = ch * 16 < (p.D >> SH) ? r * ssb + ch * 16 : 0x40000000;
  }
  const char* khead = (const char*)p.k.ptr + (((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) >> SH);
  const char* vhead = (const char*)p.v.ptr + (((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) >> SH);
  const int kbytes = (int)((int64_t)(p.C - 1) * ssb + (p.D >> SH));
  const int vbytes = (int)((int64_t)(p.C - 1) * (p.v.ss >> SH) + (p.D >> SH));
  auto issue = [&](int i, int slot) {
    const int t = k0 + BK * (wave + 4 * i);
    char* kdst = ring + slot * 2 * TILEBS;
#pragma unroll
    for (int n = 0; n < NPC; ++n) {
      const int rk = t * ssb;
      lds_dma16(khead + rk, max(kbytes - rk, 0), poff[n], kdst + n * 1024);
    }
#pragma unroll
    for (int n = 0; n < NPC; ++n) {
      const int rv = t * ssb;
      // V rows share the K piece geometry when the row strides agree (host-checked).
      lds_dma16(vhead + rv, max(vbytes - rv, 0), voff[n], kdst + TILEBS + n * 1024);
    }
  };
  // ds_read_b64_tr_b8 lanes (see attention_fwd_i8.hip): in each 16-lane group, lane 2j supplies
  // the row of key acc_row(j + 8s, hh) and receives column d0 + (lane & 15) of the 8 rows.
  const int trj = (lane & 15) >> 1;
  const int trg = (lane >> 4) & 1;
  const int trow0 = acc_row(trj, hh), trow1 = acc_row(trj + 8, hh);
  // INT4 V^T fragments by ds_read_b64_tr_b4: in each 16-lane group lane r supplies row r (16
  // nibbles = 16 d's of one key) and receives nibble (lane & 15) of all 16 rows, i.e. d =
  // dt·32 + l32 for 16 keys: nibbles 0-7 are k-step 0's fragment, 8-15 k-step 1's.  The rows
  // are chosen so that, after nib_widen's slot order (FP16: slot j <- nibble pi(j), pi = 0 2 4 6
  // 1 3 5 7; BF16: natural), slot j of k-step ks holds key acc_row(8·ks + j, hh), the key order
  // of the packed P.
  int v4off = 0, v4sw = 0;
  if constexpr (I4) {
    const int r = lane & 15;
    constexpr int PINV[8] = {0, 4, 1, 5, 2, 6, 3, 7};  // pi^-1
    const int jj = E::prec == P_FP16 ? PINV[r & 7] : (r & 7);
    const int key = acc_row(8 * (r >> 3) + jj, hh);
    v4off = key * ROWBS + 8 * ((lane >> 4) & 1);
    v4sw = swz4(key);
  }
  const float zk = (float)(p.k.zp + (I4 ? 8 : 0)), zv = (float)(p.v.zp + (I4 ? 8 : 0));

  f32x16 o[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) o[dt] = zero16();
  float m = -kFltMax, lh = 0.f;

#pragma unroll
  for (int n = 0; n < NSLOT - 1; ++n)
    if (mine > n) issue(n, n);
  for (int i = 0; i < mine; ++i) {
    const int slot = i % NSLOT;
    if (i + NSLOT - 1 < mine) {
      issue(i + NSLOT - 1, (i + NSLOT - 1) % NSLOT);
      __builtin_amdgcn_s_waitcnt(vm_wait((NSLOT - 1) * 2 * NPC));  // tile i landed
    } else if (NSLOT >= 4 && i + 2 < mine) {
      __builtin_amdgcn_s_waitcnt(vm_wait(4 * NPC));  // tiles i + 1, i + 2 still in flight
    } else if (NSLOT >= 3 && i + 1 < mine) {
      __builtin_amdgcn_s_waitcnt(vm_wait(2 * NPC));  // tile i + 1 still in flight
    } else {
      wait_vm();
    }
    const char* kt = ring + slot * 2 * TILEBS;
    const char* vt = kt + TILEBS;
    const int t = k0 + BK * (wave + 4 * i);

    // S^T = K·Q^T: key l32 on the A operand's row, elements d = 16s + 8hh + j (INT4: the lane
    // order above, two k-steps per 8-byte read of the packed row).
    f32x16 sa[1];
    sa[0] = zero16();
    if constexpr (I4) {
      const char* kp = ring + slot * 2 * TILEBS;
#pragma unroll
      for (int a = 0; a < DP / 32; ++a) {
        const uint2 kb =
            *reinterpret_cast<const uint2*>(kp + l32 * ROWBS + 16 * (a ^ swz4(l32)) + 8 * hh);
        sa[0] = E::mma(nib_widen<E>(kb.x, zk), qf[2 * a], sa[0]);
        sa[0] = E::mma(nib_widen<E>(kb.y, zk), qf[2 * a + 1], sa[0]);
      }
    } else {
#pragma unroll
      for (int st = 0; st < DP / 16; ++st) {
        const uint2 kb = *reinterpret_cast<const uint2*>(kt + T::off(l32, st) + 8 * hh);
        sa[0] = E::mma(widen_i8<E>(kb.x, kb.y, zk), qf[st], sa[0]);
      }
    }
    if (t + BK > p.C || (p.mask.causal && t + BK - 1 > qcol) || t < wlo) {
      // Keys past C, (causal) keys past the lane's query index and (window) keys below
      // qcol - window: -inf (key offset acc_row(r, hh) within the tile).
      const int last = p.mask.causal ? min(p.C - 1, qcol) : p.C - 1;
      mask_outside<1>(sa, wlo - t - 4 * hh, last - t - 4 * hh, -__builtin_inff());
    }
    f32x16& s = sa[0];
    float mx = s[0];
#pragma unroll
    for (int r = 1; r < 16; ++r) mx = fmaxf(mx, s[r]);
    mx = cross_half_max(mx) * c;
    if (__any(mx > m)) {
      const float m_new = fmaxf(m, mx);
      const float corr = __builtin_amdgcn_exp2f(m - m_new);
      m = m_new;
      lh *= corr;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[dt][r] *= corr;
    }
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[r], c, -m));
      s[r] = pv;
      rs += pv;
    }
    lh += rs;
    i16x8 pb[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[ks][j] = (short)E::from_f32(s[8 * ks + j]);
    // O^T += V^T·P^T.
    if constexpr (I4) {
      const char* vp = ring + slot * 2 * TILEBS + TILEBS;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const i32x2d w = __builtin_amdgcn_ds_read_tr4_b64_v2i32(
            (__attribute__((address_space(3))) i32x2d*)(vp + v4off + 16 * (dt ^ v4sw)));
        o[dt] = E::mma(nib_widen<E>((uint32_t)w[0], zv), pb[0], o[dt]);
        o[dt] = E::mma(nib_widen<E>((uint32_t)w[1], zv), pb[1], o[dt]);
      }
    } else {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt) {
        const int col = dt * 32 + 16 * trg + 8 * (lane & 1);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const char* pa = vt + T::off(ks ? trow1 : trow0, col >> 4) + (col & 15);
          const i32x2d w = __builtin_amdgcn_ds_read_tr8_b64_v2i32(
              (__attribute__((address_space(3))) i32x2d*)pa);
          o[dt] = E::mma(widen_i8<E>((uint32_t)w[0], (uint32_t)w[1], zv), pb[ks], o[dt]);
        }
      }
    }
  }

  const float l = cross_half_sum(lh);
  // The 4 waves' partials meet in LDS ([4][32][DP] O, then [4][32] (m, l)) over the ring once
  // every wave is done with it.  One split: 256 threads merge them into O and L.  Several
  // splits: they combine them into the workgroup's one partial per row (a quarter of the
  // partial traffic and merge work of a partial per wave), in the merge's arithmetic, so the
  // merge pass of a single split reproduces the in-workgroup result bit for bit.
  __syncthreads();
  float* po = reinterpret_cast<float*>(smem);
  float2* pml = reinterpret_cast<float2*>(smem + 4 * 32 * DP * 4);
  float* prow = po + (wave * 32 + l32) * DP;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(prow + dt * 32 + 8 * g + 4 * hh) =
          make_float4(o[dt][4 * g], o[dt][4 * g + 1], o[dt][4 * g + 2], o[dt][4 * g + 3]);
  if (hh == 0) pml[wave * 32 + l32] = make_float2(m, l);
  __syncthreads();
  constexpr int CH = DP / 4, RPI = 256 / CH;  // 16-byte chunks per row, rows per pass
  const int ch = tid % CH;
#pragma unroll
  for (int k = 0; k < 32 / RPI; ++k) {
    const int r = tid / CH + k * RPI;
    const int qr = rt * 32 + r;
    if (qr < dp.rows) {
      if (dp.fused) {
        const int g = qr / p.R, q = qr % p.R;
        merge_partials(p, pml + r, 32, po + r * DP, 32 * DP, 4, b, kvh + g * p.Hkv, q, 4 * ch,
                       ch == 0);
      } else {
        store_split_partial(p, dp, pml + r, 32, po + r * DP, 32 * DP, u, split, r, 4 * ch);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// At most 16 query rows per kv head (the usual decode step: S_q 1-16, GQA groups up to 16
// rows), D <= 256 (INT4 at D = 256 at one wave per SIMD): the same split / partial / merge
// layout on v_mfma_f32_16x16x32, whose
// 16-query output halves the per-key softmax work of the 32-row tile (a lane holds one score
// per 4 keys instead of per 2) and whose K operand rows are contiguous reads:
//   * key tiles of BK = 64 (INT4) / 32 (INT8), each wave its own; K goes from HBM straight to
//     registers (lane: key l16 of a 16-key block, bytes g·ROWBS/4 .. (g+1)·ROWBS/4 of its
//     row: one wave load is 16 whole rows), double-buffered one tile ahead; V by LDS-DMA into a
//     3-slot ring, two tiles ahead, its 16-byte chunks XOR-swizzled per row (vsw);
//   * S^T = K·Q^T: k-step dt of a lane covers d = g·DP/4 + 8·dt + j (INT4: + kI4Perm[j],
//     nib_widen's order; Q loaded to match); the output holds key 16·kb + 4·g + e, query l16;
//   * O^T += V^T·P^T with V^T fragments read transposed from the V tile (INT4
//     ds_read_b64_tr_b4: lane r of each 16-lane group supplies the row of nibble slot r, key
//     32·c + 16·(j >> 2) + 4·g + (j & 3) for r = 8·c + pi(j); INT8 ds_read_b64_tr_b8: lanes
//     2j, 2j + 1 supply key 16·(j >> 2) + 4·g + (j & 3)), so the P fragments are the S
//     registers as they lie.
template <class E>
__device__ __forceinline__ f32x4 mma16(i16x8 a, i16x8 b, f32x4 c) {
  if constexpr (E::prec == P_FP16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}

// Max / sum over lanes l, l ^ 16, l ^ 32, l ^ 48 (one query column of a 16x16 output).
__device__ __forceinline__ float xgroup_max(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return cross_half_max(
      fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1])));
}
__device__ __forceinline__ float xgroup_sum(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return cross_half_sum(__builtin_bit_cast(float, (unsigned)r[0]) +
                        __builtin_bit_cast(float, (unsigned)r[1]));
}

template <int DP, int SRC>
constexpr int decode16_lds() {
  constexpr int tile = (SRC == SRC_I4 ? 64 * (DP / 2) : 32 * DP);
  constexpr int ring = 4 * (DP == 256 ? 2 : 3) * tile, merge = 4 * 16 * DP * 4 + 4 * 16 * 8;
  return ring > merge ? ring : merge;
}

template <class E, int DP, int SRC>
__global__ void __launch_bounds__(256, DP == 256 && SRC == SRC_I4 ? 1 : 2)
    mfa_fwd_decode16_kernel(DecodeParams dp) {
  const FwdParams& p = dp.f;
  constexpr bool I4 = SRC == SRC_I4;
  // V ring slots: 3 (two tiles ahead); 2 at D = 256 (one ahead: two workgroups per CU).
  constexpr int BK = I4 ? 64 : 32, NKB = BK / 16, NV = DP == 256 ? 2 : 3, NDT = DP / 32;
  constexpr int NDB = DP / 16;
  constexpr int SH = I4 ? 1 : 0;            // element -> byte offsets
  constexpr int ROWBS = DP >> SH;           // stored bytes per row
  constexpr int TILEBS = BK * ROWBS;        // one stored key tile
  constexpr int NPV = TILEBS / 1024;        // V DMA pieces per tile
  constexpr int RP = 1024 / ROWBS;          // rows per piece
  constexpr int CPR = ROWBS / 16;           // 16-byte chunks per row
  constexpr int KLB = ROWBS / 4;            // K bytes per lane per 16-key block
  constexpr int NKL = KLB >= 16 ? KLB / 16 : 1;  // K loads per block (b128, or one b64)
  constexpr int NI = NPV + NKB * NKL;       // vm operations per tile
  static_assert(DP == 64 || DP == 128 || DP == 256, "decode16 widths");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, g = lane >> 4;
  char* const ring = smem + wave * NV * TILEBS;

  const int split = blockIdx.x;
  const int u = blockIdx.y + gridDim.y * blockIdx.z;    // b·H_kv + kvh (one row tile)
  const int kvh = u % p.Hkv, b = u / p.Hkv;
  const float c = p.c_log2;

  // Q^T fragments: lane (query l16, group g), k-step dt: d = g·DP/4 + 8·dt + (kI4Perm)[j].
  const int row = l16;
  const bool rvalid = row < dp.rows;
  const int qcol = rvalid ? row % p.R : 0x3fffffff;
  const int wlo = p.mask.window ? qcol - (int)min(p.mask.window_size, 0x3fffffffu) : -0x40000000;
  i16x8 qf[NDT];
  {
    const int gq = rvalid ? row / p.R : 0, q = rvalid ? row % p.R : 0;
    const int h = kvh + gq * p.Hkv;
    const uint16_t* qrow =
        (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh + (int64_t)q * p.q.ss;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const int d0 = g * (DP / 4) + 8 * dt;
      i16x8 v = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (rvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
      qf[dt] = I4 ? i4_order<E>(v) : v;
    }
  }

  // Keys of this split: [k0, k1); this wave's tiles k0 + BK·(wave + 4i).
  const int k0 = split * dp.chunk;
  const int k1 = min(p.C, k0 + dp.chunk);
  const int nt = k1 > k0 ? (k1 - k0 + BK - 1) / BK : 0;
  const int mine = nt > wave ? (nt - wave + 3) / 4 : 0;

  const int ssb = (int)(p.k.ss >> SH);
  const char* khead = (const char*)p.k.ptr + (((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) >> SH);
  const char* vhead = (const char*)p.v.ptr + (((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) >> SH);
  const int kbytes = (int)((int64_t)(p.C - 1) * ssb + (p.D >> SH));
  const int vbytes = (int)((int64_t)(p.C - 1) * (p.v.ss >> SH) + (p.D >> SH));
  // K row offsets of the lane's 16-key blocks (bytes past D: out of range, read as 0).
  const int kcol = g * KLB < (p.D >> SH) ? g * KLB : 0x40000000;
  int koff[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) koff[kb] = (16 * kb + l16) * ssb + kcol;
  // V chunk swizzle: the 16 (INT4) / 8 + 8 (INT8) rows one transposed read gathers into a
  // 32-lane half spread over the banks (INT4: 2-way at most; INT8: conflict-free).
  auto vsw = [](int r) {
    if constexpr (I4 && CPR == 8) return ((r >> 1) & 1) | (((r >> 4) & 3) << 1);
    else if constexpr (I4) return (r >> 4) & (CPR - 1);
    else if constexpr (CPR == 16) return (r & 3) | (((r >> 2) & 1) << 2) | (((r >> 4) & 1) << 3);
    else if constexpr (CPR == 8) return ((r >> 1) & 1) | (((r >> 2) & 1) << 1) | (((r >> 4) & 1) << 2);
    else return ((r >> 2) & 1) | (((r >> 4) & 1) << 1);
  };
  // V DMA: piece n holds rows n·RP .. n·RP + RP - 1; lane l lands at physical chunk l % CPR of
  // row n·RP + l / CPR and fetches logical chunk (l % CPR) ^ vsw(row).
  int voff[NPV];
#pragma unroll
  for (int n = 0; n < NPV; ++n) {
    const int r = n * RP + lane / CPR;
    const int ch = (lane % CPR) ^ vsw(r);
    voff[n] = ch * 16 < (p.D >> SH) ? r * ssb + ch * 16 : 0x40000000;
  }
  // Transposed V reads: the row this lane supplies, and its swizzle.
  int vtrow, vtsw;
  {
    constexpr int PINV[8] = {0, 4, 1, 5, 2, 6, 3, 7};  // kI4Perm^-1
    int key;
    if constexpr (I4) {
      const int j = E::prec == P_FP16 ? PINV[l16 & 7] : (l16 & 7);
      key = 32 * (l16 >> 3) + 16 * (j >> 2) + 4 * g + (j & 3);
    } else {
      const int j = l16 >> 1;
      key = 16 * (j >> 2) + 4 * g + (j & 3);
    }
    vtrow = key * ROWBS + (I4 ? 0 : 8 * (l16 & 1));
    vtsw = vsw(key);
  }
  const float zk = (float)(p.k.zp + (I4 ? 8 : 0)), zv = (float)(p.v.zp + (I4 ? 8 : 0));

  uint32_t ka[NKB][KLB / 4], kn[NKB][KLB / 4];
#define DEC16_KLOAD(KR, TI)                                                                       \
  {                                                                                              \
    const int tb_ = (k0 + BK * (wave + 4 * (TI))) * ssb;                                         \
    const __amdgpu_buffer_rsrc_t rs_ = __builtin_amdgcn_make_buffer_rsrc(                        \
        (void*)(khead + tb_), (short)0, max(kbytes - tb_, 0), 0x00020000);                       \
    _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb) {                                         \
      if constexpr (KLB >= 16) {                                                                 \
        _Pragma("unroll") for (int x = 0; x < NKL; ++x) {                                        \
          const auto a_ = __builtin_amdgcn_raw_buffer_load_b128(rs_, koff[kb] + 16 * x, 0, 0);   \
          KR[kb][4 * x] = a_[0]; KR[kb][4 * x + 1] = a_[1];                                      \
          KR[kb][4 * x + 2] = a_[2]; KR[kb][4 * x + 3] = a_[3];                                  \
        }                                                                                        \
      } else {                                                                                   \
        const auto a_ = __builtin_amdgcn_raw_buffer_load_b64(rs_, koff[kb], 0, 0);               \
        KR[kb][0] = a_[0]; KR[kb][1] = a_[1];                                                    \
      }                                                                                          \
    }                                                                                            \
  }
  auto vissue = [&](int i) {
    const int rv = (k0 + BK * (wave + 4 * i)) * ssb;
    char* dst = ring + (i % NV) * TILEBS;
#pragma unroll
    for (int n = 0; n < NPV; ++n) lds_dma16(vhead + rv, max(vbytes - rv, 0), voff[n], dst + n * 1024);
  };

  f32x4 o[NDB];
#pragma unroll
  for (int db = 0; db < NDB; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -kFltMax, lh = 0.f;

  // Issue order V(0) K(0) V(1), then per tile i: K(i + 1) V(i + 2): V(i) always precedes K(i),
  // so one counted vmcnt wait for K(i) covers both.  Two slots (D = 256): K(0) V(0), then per
  // tile K(i + 1) V(i + 1), and the wait is for V(i).
#define DEC16_STEP(KC, KN, I)                                                                     \
  {                                                                                              \
    const int ii = (I);                                                                          \
    if (ii + 1 < mine) DEC16_KLOAD(KN, ii + 1);                                                  \
    if constexpr (NV == 2) {                                                                     \
      if (ii + 1 < mine) {                                                                       \
        vissue(ii + 1);                                                                          \
        __builtin_amdgcn_s_waitcnt(vm_wait(NI));                                                 \
      } else {                                                                                   \
        __builtin_amdgcn_s_waitcnt(vm_wait(0));                                                  \
      }                                                                                          \
    } else if (ii + 2 < mine) {                                                                  \
      vissue(ii + 2);                                                                            \
      __builtin_amdgcn_s_waitcnt(vm_wait(NI + NPV));                                             \
    } else if (ii + 1 < mine) {                                                                  \
      __builtin_amdgcn_s_waitcnt(vm_wait(NI));                                                   \
    } else {                                                                                     \
      __builtin_amdgcn_s_waitcnt(vm_wait(0));                                                    \
    }                                                                                            \
    const char* vs = ring + (ii % NV) * TILEBS;                                                  \
    const int t = k0 + BK * (wave + 4 * ii);                                                     \
    f32x4 sc[NKB];                                                                               \
    _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb) {                                         \
      sc[kb] = f32x4{0.f, 0.f, 0.f, 0.f};                                                        \
      _Pragma("unroll") for (int dt = 0; dt < NDT; ++dt) {                                       \
        if constexpr (I4)                                                                        \
          sc[kb] = mma16<E>(nib_widen<E>(KC[kb][dt], zk), qf[dt], sc[kb]);                       \
        else                                                                                     \
          sc[kb] = mma16<E>(widen_i8<E>(KC[kb][2 * dt], KC[kb][2 * dt + 1], zk), qf[dt], sc[kb]); \
      }                                                                                          \
    }                                                                                            \
    if (t + BK > k1 || (p.mask.causal && t + BK - 1 > qcol) || t < wlo) {                       \
      const int last = (p.mask.causal ? min(k1 - 1, qcol) : k1 - 1) - t, first = wlo - t;        \
      _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                         \
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                          \
          const int kk = 16 * kb + 4 * g + e;                                                    \
          sc[kb][e] = kk > last || kk < first ? -__builtin_inff() : sc[kb][e];                   \
        }                                                                                        \
    }                                                                                            \
    float mx = fmaxf(fmaxf(sc[0][0], sc[0][1]), fmaxf(sc[0][2], sc[0][3]));                      \
    _Pragma("unroll") for (int kb = 1; kb < NKB; ++kb)                                           \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) mx = fmaxf(mx, sc[kb][e]);                   \
    mx = xgroup_max(mx) * c;                                                                     \
    if (__any(mx > m)) {                                                                         \
      const float m_new = fmaxf(m, mx);                                                          \
      const float corr = __builtin_amdgcn_exp2f(m - m_new);                                      \
      m = m_new;                                                                                 \
      lh *= corr;                                                                                \
      _Pragma("unroll") for (int db = 0; db < NDB; ++db) o[db] *= corr;                          \
    }                                                                                            \
    float rs = 0.f;                                                                              \
    _Pragma("unroll") for (int kb = 0; kb < NKB; ++kb)                                           \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                            \
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[kb][e], c, -m));               \
        sc[kb][e] = pv;                                                                          \
        rs += pv;                                                                                \
      }                                                                                          \
    lh += rs;                                                                                    \
    i16x8 pb[NKB / 2];                                                                           \
    _Pragma("unroll") for (int cc = 0; cc < NKB / 2; ++cc)                                       \
      _Pragma("unroll") for (int e = 0; e < 4; ++e) {                                            \
        pb[cc][e] = (short)E::from_f32(sc[2 * cc][e]);                                           \
        pb[cc][4 + e] = (short)E::from_f32(sc[2 * cc + 1][e]);                                   \
      }                                                                                          \
    _Pragma("unroll") for (int db = 0; db < NDB; ++db) {                                         \
      if constexpr (I4) {                                                                        \
        const i32x2d w = __builtin_amdgcn_ds_read_tr4_b64_v2i32(                                 \
            (__attribute__((address_space(3))) i32x2d*)(vs + vtrow + 16 * ((db >> 1) ^ vtsw) +   \
                                                        8 * (db & 1)));                          \
        o[db] = mma16<E>(nib_widen<E>((uint32_t)w[0], zv), pb[0], o[db]);                        \
        o[db] = mma16<E>(nib_widen<E>((uint32_t)w[1], zv), pb[NKB / 2 - 1], o[db]);              \
      } else {                                                                                   \
        const i32x2d w = __builtin_amdgcn_ds_read_tr8_b64_v2i32(                                 \
            (__attribute__((address_space(3))) i32x2d*)(vs + vtrow + 16 * (db ^ vtsw)));         \
        o[db] = mma16<E>(widen_i8<E>((uint32_t)w[0], (uint32_t)w[1], zv), pb[0], o[db]);         \
      }                                                                                          \
    }                                                                                            \
  }

  if (mine > 0) {
    if constexpr (NV == 2) {
      DEC16_KLOAD(ka, 0);
      vissue(0);
    } else {
      vissue(0);
      DEC16_KLOAD(ka, 0);
    }
  }
  if (NV == 3 && mine > 1) vissue(1);
  for (int i = 0; i < mine; i += 2) {
    DEC16_STEP(ka, kn, i);
    if (i + 1 < mine) DEC16_STEP(kn, ka, i + 1);
  }
#undef DEC16_STEP
#undef DEC16_KLOAD

  const float l = xgroup_sum(lh);
  // The 4 waves' partials meet in LDS ([4][16][DP] O, then [4][16] (m, l)) over the ring; one
  // split: 256 threads merge them; several: the workgroup's one partial per row (as above).
  __syncthreads();
  float* po = reinterpret_cast<float*>(smem);
  float2* pml = reinterpret_cast<float2*>(smem + 4 * 16 * DP * 4);
  float* prow = po + (wave * 16 + l16) * DP;
#pragma unroll
  for (int db = 0; db < NDB; ++db)
    *reinterpret_cast<float4*>(prow + 16 * db + 4 * g) =
        make_float4(o[db][0], o[db][1], o[db][2], o[db][3]);
  if (g == 0) pml[wave * 16 + l16] = make_float2(m, l);
  __syncthreads();
  constexpr int CH = DP / 4, RPI = 256 / CH;  // 16-byte chunks per row, rows per pass
  const int ch = tid % CH;
#pragma unroll
  for (int k = 0; k < 16 / RPI; ++k) {
    const int r = tid / CH + k * RPI;
    if (r < dp.rows) {
      if (dp.fused) {
        const int gq = r / p.R, q = r % p.R;
        merge_partials(p, pml + r, 16, po + r * DP, 16 * DP, 4, b, kvh + gq * p.Hkv, q, 4 * ch,
                       ch == 0);
      } else {
        store_split_partial(p, dp, pml + r, 16, po + r * DP, 16 * DP, u, split, r, 4 * ch);
      }
    }
  }
}

// One query row per wave: combines the row's nsplit partials.  O is written with the
// caller's strides, L = m + log2 l in the descriptor's memory precision.
__global__ void __launch_bounds__(256) mfa_decode_merge_kernel(DecodeParams dp) {
  const FwdParams& p = dp.f;
  const int lane = threadIdx.x & 63;
  const int64_t rid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // (b·H + h)·R + q
  if (rid >= (int64_t)p.B * p.H * p.R) return;
  const int q = (int)(rid % p.R);
  const int bh = (int)(rid / p.R);
  const int h = bh % p.H, b = bh / p.H;
  const int kvh = h % p.Hkv, g = h / p.Hkv;
  const int row = g * p.R + q;
  const int u = (b * p.Hkv + kvh) * dp.nrt + row / 32;
  const int np = dp.nsplit;  // one partial per split (the workgroup's)
  const int64_t base = (int64_t)u * np * 32 + (row % 32);
  merge_partials(p, dp.mlpart + base, 32, dp.opart + base * p.D, (int64_t)32 * p.D, np, b, h, q,
                 4 * lane, lane == 0);
}

// Rows with many partials (more than 32: few units, long caches): one row per workgroup, the
// 4 waves take a quarter of the partials each (the same weights w_s), and their sums meet in
// LDS.
__global__ void __launch_bounds__(256) mfa_decode_merge4_kernel(DecodeParams dp) {
  const FwdParams& p = dp.f;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t rid = blockIdx.x;  // (b·H + h)·R + q
  const int q = (int)(rid % p.R);
  const int bh = (int)(rid / p.R);
  const int h = bh % p.H, b = bh / p.H;
  const int kvh = h % p.Hkv, g = h / p.Hkv;
  const int row = g * p.R + q;
  const int u = (b * p.Hkv + kvh) * dp.nrt + row / 32;
  const int np = dp.nsplit, s0 = w * np / 4, nq = (w + 1) * np / 4 - s0;
  const int64_t base = ((int64_t)u * np + s0) * 32 + (row % 32);
  const float2* ml = dp.mlpart + base;
  const float* op = dp.opart + base * p.D;
  __shared__ float smx[4], sl[4];
  __shared__ float4 sacc[4][64];
  const float mw = merge_max(ml, 32, nq);
  if (lane == 0) smx[w] = mw;
  __syncthreads();
  const float mx = fmaxf(fmaxf(smx[0], smx[1]), fmaxf(smx[2], smx[3]));
  float l = 0.f;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  merge_sum(p, ml, 32, op, (int64_t)32 * p.D, nq, mx, 4 * lane, l, acc);
  sacc[w][lane] = acc;
  if (lane == 0) sl[w] = l;
  __syncthreads();
  if (w == 0) {
    float4 a = sacc[0][lane];
#pragma unroll
    for (int v = 1; v < 4; ++v) {
      const float4 x = sacc[v][lane];
      a.x += x.x; a.y += x.y; a.z += x.z; a.w += x.w;
    }
    merge_store(p, a, ((sl[0] + sl[1]) + sl[2]) + sl[3], mx, b, h, q, 4 * lane, lane == 0);
  }
}

// Keys a decode call reads: all C, or under a causal mask only those some query row sees.
int decode_keys(int R, int C, bool causal) { return causal ? (C < R ? C : R) : C; }

// Split of the key range: enough workgroups for two per CU (512) when the units alone do not
// provide them, each wave at least 4 tiles (128 keys).
void decode_layout(int B, int Hkv, int rows, int C, int* nrt, int* nsplit, int* chunk) {
  *nrt = (rows + 31) / 32;
  const int units = B * Hkv * *nrt;
  const int tiles = (C + 31) / 32;
  int ns = (512 + units - 1) / units;
  if (ns > tiles / 16) ns = tiles / 16;
  if (ns < 1) ns = 1;
  const int per = (tiles + ns - 1) / ns;  // tiles per split, rounded to whole 4-wave rounds
  *chunk = ((per + 3) / 4) * 4 * 32;
  *nsplit = (C + *chunk - 1) / *chunk;
}

// Partials workspace of the split path; 0 when a unit's keys fit one split and the workgroup
// merges its waves' partials in LDS (the kernel then never touches the workspace).
static bool decode_fused(int nsplit) {
  const char* mv = mfa::dev_env("MFA_DECODE_MERGE");  // =1: the separate merge pass for one split too
  return nsplit == 1 && !(mv && mv[0] == '1');
}

size_t decode_workspace_bytes(int B, int Hkv, int rows, int C, int D) {
  int nrt, ns, chunk;
  decode_layout(B, Hkv, rows, C, &nrt, &ns, &chunk);
  if (decode_fused(ns)) return 0;
  const size_t parts = (size_t)B * Hkv * nrt * ns * 32;  // one partial per split and row
  return parts * D * 4 + parts * 8 + 256;
}

// The merge pass: one row per wave, or with more than 32 partials (splits) per row one row per
// workgroup (4 waves).
static hipError_t launch_merge(const DecodeParams& dp, hipStream_t stream) {
  const int64_t nrows = (int64_t)dp.f.B * dp.f.H * dp.f.R;
  if (dp.nsplit > 32)
    return launch(mfa_decode_merge4_kernel, dim3((unsigned)nrows), dim3(256), 0, stream, dp);
  return launch(mfa_decode_merge_kernel, dim3((unsigned)((nrows + 3) / 4)), dim3(256), 0, stream, dp);
}

hipError_t fwd_decode_dispatch(const FwdParams& p, int elem, void* workspace, hipStream_t stream) {
  const bool i4 = p.k.prec == P_INT4;
  if (p.k.prec != p.v.prec || (p.k.prec != P_INT8 && !i4) || p.k.ss != p.v.ss)
    return hipErrorNotSupported;
  DecodeParams dp;
  dp.f = p;
  // Causal (key <= query index): no row sees a key past R - 1.
  if (p.mask.causal) dp.f.C = decode_keys(p.R, p.C, true);
  dp.rows = (p.H / p.Hkv) * p.R;
  decode_layout(p.B, p.Hkv, dp.rows, dp.f.C, &dp.nrt, &dp.nsplit, &dp.chunk);
  const size_t parts = (size_t)p.B * p.Hkv * dp.nrt * dp.nsplit * 32;
  dp.opart = (float*)workspace;
  dp.mlpart = workspace ? (float2*)((char*)workspace + ((parts * p.D * 4 + 255) & ~(size_t)255))
                        : nullptr;
  const int units = p.B * p.Hkv * dp.nrt;
  if (units >= 65536) return hipErrorNotSupported;
  const dim3 grid(dp.nsplit, units, 1);
  const int DP = p.D <= 64 ? 64 : p.D <= 128 ? 128 : 256;
  dp.fused = decode_fused(dp.nsplit);
  if (!dp.fused && !workspace) return hipErrorInvalidValue;
  hipError_t e = hipErrorNotSupported;
  // At most 16 rows per kv head: the 16x16x32 kernel (MFA_DECODE16=0: the 32-row one; =4: INT4
  // only; =2: not at D = 256, A/B switches).
  const char* d16 = dev_env("MFA_DECODE16");
  if (dp.rows <= 16 && !(d16 && d16[0] == '0') && (i4 || !(d16 && d16[0] == '4')) &&
      !(DP == 256 && d16 && d16[0] == '2')) {
#define MFA_DEC16(ELEM, EE, DPV)                                                               \
    if (elem == ELEM && DP == DPV)                                                             \
      e = i4 ? launch(mfa_fwd_decode16_kernel<EE, DPV, SRC_I4>, grid, dim3(256),               \
                      decode16_lds<DPV, SRC_I4>(), stream, dp)                                 \
             : launch(mfa_fwd_decode16_kernel<EE, DPV, SRC_I8>, grid, dim3(256),               \
                      decode16_lds<DPV, SRC_I8>(), stream, dp);
    MFA_DEC16(P_FP16, F16, 64)
    MFA_DEC16(P_FP16, F16, 128)
    MFA_DEC16(P_BF16, BF16, 64)
    MFA_DEC16(P_BF16, BF16, 128)
    MFA_DEC16(P_FP16, F16, 256)
    MFA_DEC16(P_BF16, BF16, 256)
#undef MFA_DEC16
    if (e != hipSuccess || dp.fused) return e;
    return launch_merge(dp, stream);
  }
#define MFA_DEC(ELEM, EE, DPV)                                                                 \
  if (elem == ELEM && DP == DPV)                                                               \
    e = i4 ? launch(mfa_fwd_decode_kernel<EE, DPV, SRC_I4>, grid, dim3(256),                   \
                    4 * 2 * 2 * 32 * DPV + 1024, stream, dp)                                   \
           : launch(mfa_fwd_decode_kernel<EE, DPV, SRC_I8>, grid, dim3(256),                   \
                    4 * 2 * 2 * 32 * DPV + 1024, stream, dp);
  MFA_DEC(P_FP16, F16, 64)
  MFA_DEC(P_FP16, F16, 128)
  MFA_DEC(P_FP16, F16, 256)
  MFA_DEC(P_BF16, BF16, 64)
  MFA_DEC(P_BF16, BF16, 128)
  MFA_DEC(P_BF16, BF16, 256)
#undef MFA_DEC
  if (e != hipSuccess || dp.fused) return e;
  return launch_merge(dp, stream);
}

}  // namespace mfa
