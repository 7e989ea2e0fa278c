// attention_fwd_kv8.hip — QuantizedAttention forward with per-tensor INT8 / INT4 K/V
// dequantised on load inside the tuned 16-bit loop (GEMMHeaders.swift:679-808: the reference widens K/V
// tiles as it loads them; QuantizedAttention.swift:135-263 dispatches it).
//
// Schedule: the adjacent-pair form of the shared-tile forward (attention_fwd_v2.hip,
// mfa_fwd2_share_kernel with MIRROR = false): 512 threads own query blocks 2·pi and 2·pi + 1
// (one 4-wave group each) and every K/V tile feeds both, 256 query rows per staged tile.
// Per step s, each thread:
//   - widens its 16-byte chunk of tile s + 1's K and V bytes (in registers since step s − 1)
//     to the exact integers q − zp in FP16 (magic-number v_perm + packed subtract,
//     mfa_stage.h dequant_fast) and writes it into the 16-bit TileA image slots of tile s + 1,
//     in four pieces placed between the MFMAs of tile s's QKᵀ and PV chains;
//   - right after each widening, loads the same chunk of tile s + 2 into the freed registers
//     (global loads, about one step of latency cover; no LDS staging, so the LDS traffic is
//     the 16-bit kernel's);
//   - runs tile s from its 16-bit image exactly as the 16-bit kernel does.
// Instantiated for FP16 and BF16 at D = 64, 128 (BK = 64) and 256 (BK = 32, the 16-bit
// kernel's tile depth there; one 16-byte chunk per thread per tile at every width but 64,
// where each thread widens one 8-element chunk).
// Per-tensor scales stay folded in the softmax multiplier (K) and the output multiplier (V),
// so the MFMA operands, and hence O and L, are bit-identical to the dequantise pass +
// 16-bit kernel path — with 1 byte (INT4: half a byte) per K/V element read from HBM, no
// pass, no scratch.
// LDS: 16-bit ring of 4 tiles, reused at the end for the two O row images
// (2 x 128 rows x (4·D + 16) bytes) up to D = 128; at D = 256 rows leave from registers.
#include "attention_fwd2.h"
#include "kv_bytes.h"

namespace mfa {

// BW (round 6): block-wise K/V scales (and zero points) applied on load, at D <= 128 with the
// block size a multiple of the chunk width and untransposed K/V: a thread's chunk lies in one
// scale block, so its widening takes one scale and one zero point, loaded with the chunk's bytes
// a tile ahead, and writes (q - zp) * s rounded to E — the values the dequantisation pass
// writes (kv_dequant.hip), so the MFMA operands, O and L are bit-identical to that path
// (AttentionKernel+OuterProduct.swift:301-316 and AttentionKernel+Accumulate.swift:461-476
// apply the block scales inside the reference kernel the same way).
template <class E, int DP, int BK, int SRC, bool BW = false>
__global__ void __launch_bounds__(512, 1) mfa_fwd2_kv8_kernel(FwdParams p) {
  constexpr int NT = 512, BQ = 128, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int ORS = DP * 4 + 16;          // O row image stride
  constexpr bool OIMG = 2 * 128 * ORS <= 160 * 1024;  // O leaves through row images (D <= 128)
  using G = Kv8Geo<DP, BK>;
  constexpr int CE = G::CE;
  // Widening pieces: after QKᵀ MFMAs 1 and 3 (K) and 4 / 2 before the end of the PV chain (V);
  // one TileA chunk each (CE = 16), or the single chunk at the second slot (CE = 8).
  constexpr int NMK = (BK / 32) * (DP / 16), NMV = (BK / 32) * 2 * ND;
  constexpr int KP0 = 1, KP1 = 3, VP0 = NMV - 4, VP1 = NMV - 2;
  static_assert(KP1 < NMK && VP0 >= 0, "hook slots");
  // D = 256: the Q fragments and O accumulators leave no registers for the next tile's bytes
  // (the register-staged form spills), so the bytes go through an LDS ring by LDS-DMA instead:
  // each lane's own chunk (one 16-byte piece, or two 4-byte pieces for INT4), read back by the
  // same lane just before its widening — a counted vmcnt wait, no barrier.
  constexpr bool RAWLDS = DP == 256;
  static_assert(!(BW && RAWLDS), "block-wise scales on load: D <= 128");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / 256);
  const int gt = tid % 256;
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  char* const sk = smem;                  // 16-bit K slots 0, 1
  char* const sv = smem + 2 * TILEB;      // 16-bit V slots 0, 1

  const int BH = p.B * p.H;
  // Causal: the heaviest pairs first (balance over the grid).
  const int pi = p.mask.causal ? (p.nblk + 1) / 2 - 1 - (int)(blockIdx.x / BH) : blockIdx.x / BH;
  const int bh = blockIdx.x % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const float zk = (float)p.k.zp, zv = (float)p.v.zp;

  constexpr int ESH = SRC == SRC_I8 ? 0 : 1;
  const char* khead = (const char*)p.k.ptr + (((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) >> ESH);
  const char* vhead = (const char*)p.v.ptr + (((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) >> ESH);
  // Key tiles [kbeg, kend) of the pair's 256 rows (causal / window: the tiles some row of the
  // pair sees; the host routes these masks here only when skipping is exact, skip_ok).
  int kbeg, kend;
  key_range(p, 2 * pi * BQ, 2 * BQ, BK, &kbeg, &kend);
  const int n = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  const G geo(tid);
  const int cr = geo.r, ch0 = geo.ch0;
  const bool cvalid = geo.col < p.D;
  // Range-checked buffer loads: rows past C and chunks past D read as zeros.
  // Byte geometry: INT8 one byte per element, INT4 half a byte.
  constexpr int SH = ESH, CB = CE >> SH;
  const int kss = (int)(p.k.ss >> SH), vss = (int)(p.v.ss >> SH);
  const int kbytes = (int)((int64_t)(p.C - 1) * kss + (p.D >> SH));
  const int vbytes = (int)((int64_t)(p.C - 1) * vss + (p.D >> SH));
  const int kro = cvalid ? cr * kss + (geo.col >> SH) : 0x40000000;
  const int vro = cvalid ? cr * vss + (geo.col >> SH) : 0x40000000;
  // rk / rv: the bytes of the next tile to widen.  Each is reloaded (tile s + 2) as soon as
  // its widening into tile s + 1's slot has been issued, one step ahead of its use.
  uint4 rk = make_uint4(0u, 0u, 0u, 0u), rv = rk;
  // This thread's chunk of tile t's K (V) bytes.
  auto load1 = [&](const char* head, int ss, int bytes, int ro, int t) -> uint4 {
    const int tb = t * ss;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(head + tb), (short)0, max(bytes - tb, 0), 0x00020000);
    if constexpr (CB == 16) {
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, ro, 0, 0);
      return make_uint4(a[0], a[1], a[2], a[3]);
    } else if constexpr (CB == 8) {
      const auto a = __builtin_amdgcn_raw_buffer_load_b64(rs, ro, 0, 0);
      return make_uint4(a[0], a[1], 0u, 0u);
    } else {
      return make_uint4(__builtin_amdgcn_raw_buffer_load_b32(rs, ro, 0, 0), 0u, 0u, 0u);
    }
  };
  auto loadk = [&](int t) { return load1(khead, kss, kbytes, kro, t); };
  auto loadv = [&](int t) { return load1(vhead, vss, vbytes, vro, t); };
  // BW: the scale-block row of this thread's chunk for the next load (loads run in tile order),
  // and the pending chunk's raw scale and zero-point bits and validity.  The scale loads are
  // unconditional (an invalid chunk reads block 0; a missing zero-point table reads the scale
  // table) and their values are used only at the next step's widening: a load under a branch,
  // or used right away, made hipcc wait with vmcnt(0) after it, which also waited for the
  // chunk's byte load issued just before (every step, in the first build).
  BlockRow kbr, vbr;
  int kcb = 0, vcb = 0;
  uint32_t ksr = 0u, kzr = 0u, vsr = 0u, vzr = 0u;
  bool kok = false, vok = false;
  if constexpr (BW) {
    kbr.init(quant_row(p.k, b, kvh) + cr + kbeg, p.k.bsize);
    vbr.init(quant_row(p.v, b, kvh) + cr + kbeg, p.v.bsize);
    kcb = geo.col / p.k.bsize;
    vcb = geo.col / p.v.bsize;
  }
  auto scale_of = [&](const Operand& op, BlockRow& br, int cb, int t, uint32_t& sr, uint32_t& zr,
                      bool& ok) {
    ok = cvalid && t + cr < p.C;
    const int i = ok ? br.q * op.bcols + cb : 0;
    const uint32_t* sp = reinterpret_cast<const uint32_t*>(op.bscale);
    const uint32_t* zq = op.bzp ? reinterpret_cast<const uint32_t*>(op.bzp) : sp;
    sr = sp[i];
    zr = zq[i];
    br.advance(BK, op.bsize);
  };
  auto zp_of = [&](const Operand& op, uint32_t zr) { return op.bzp ? (float)(int)zr : 0.f; };
  // The next tile's chunk bytes (and BW: its scale) into the staging registers.
  auto nextk = [&](int t) {
    rk = loadk(t);
    if constexpr (BW) scale_of(p.k, kbr, kcb, t, ksr, kzr, kok);
  };
  auto nextv = [&](int t) {
    rv = loadv(t);
    if constexpr (BW) scale_of(p.v, vbr, vcb, t, vsr, vzr, vok);
  };
  // LDS byte ring (RAWLDS): K slots 0, 1, then V slots 0, 1, of 512 chunks each.
  constexpr int NPC = CB == 16 ? 1 : CB / 4;  // DMA instructions per operand per tile
  constexpr int RSLOT = NT * CB;
  char* const rawb = smem + 4 * TILEB;
  const int wv = tid >> 6;
  auto raw_dma = [&](const char* head, int ss, int bytes, int ro, int t, char* slot) {
    const int tb = t * ss;
    if constexpr (CB == 16) {
      lds_dma16(head + tb, max(bytes - tb, 0), ro, slot + wv * 1024);
    } else {
#pragma unroll
      for (int j = 0; j < NPC; ++j)
        lds_dma4(head + tb, max(bytes - tb, 0), ro + 4 * j, slot + j * (NT * 4) + wv * 256);
    }
  };
  // Half hf of this lane's chunk, in the registers half 0 of widen_store reads.
  auto raw_read = [&](const char* slot, int hf) -> uint4 {
    if constexpr (CB == 16) {
      const uint2 a = *reinterpret_cast<const uint2*>(slot + wv * 1024 + lane * 16 + 8 * hf);
      return make_uint4(a.x, a.y, 0u, 0u);
    } else {
      return make_uint4(*reinterpret_cast<const uint32_t*>(slot + hf * (NT * 4) + wv * 256 + lane * 4),
                        0u, 0u, 0u);
    }
  };
  // Widening of half hf read by raw_read (RAWLDS).
  auto widen_half = [&](char* img, const uint4& raw, float zp, int hf) {
    widen_store<E, DP, SRC, 0>(img, cr, ch0 + hf, raw, zp);
  };
  auto dmak = [&](int t, int sl) { raw_dma(khead, kss, kbytes, kro, t, rawb + sl * RSLOT); };
  auto dmav = [&](int t, int sl) { raw_dma(vhead, vss, vbytes, vro, t, rawb + (2 + sl) * RSLOT); };
  // The staged K (V) chunk's half HF widened into image img.
  auto widen_k = [&](char* img, auto half_c) {
    constexpr int HF = decltype(half_c)::value;
    if constexpr (BW)
      *reinterpret_cast<uint4*>(img + TileA<DP>::off(cr, ch0 + HF)) =
          widen_block<E, SRC, HF>(rk, __builtin_bit_cast(float, ksr), zp_of(p.k, kzr), kok);
    else
      widen_store<E, DP, SRC, HF>(img, cr, ch0 + HF, rk, zk);
  };
  auto widen_v = [&](char* img, auto half_c) {
    constexpr int HF = decltype(half_c)::value;
    if constexpr (BW)
      *reinterpret_cast<uint4*>(img + TileA<DP>::off(cr, ch0 + HF)) =
          widen_block<E, SRC, HF>(rv, __builtin_bit_cast(float, vsr), zp_of(p.v, vzr), vok);
    else
      widen_store<E, DP, SRC, HF>(img, cr, ch0 + HF, rv, zv);
  };
  using H0 = std::integral_constant<int, 0>;
  using H1 = std::integral_constant<int, 1>;

  const int q0 = (2 * pi + g) * BQ;
  const int qi = q0 + wg * 32 + l32;
  i16x8 qf[DP / 16];
  if constexpr (RAWLDS) {
    dmak(kbeg, 0);
    dmav(kbeg, 0);
    dmak(kbeg + BK, 1);
    dmav(kbeg + BK, 1);
    load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
    wait_vm();
    __asm__ __volatile__("" ::: "memory");
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      widen_half(sk, raw_read(rawb, hf), zk, hf);
      widen_half(sv, raw_read(rawb + 2 * RSLOT, hf), zv, hf);
    }
  } else {
    nextk(kbeg);
    nextv(kbeg);
    load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
  }
  prescale_q2<E, DP>(qf, c);
  if constexpr (!RAWLDS) {
    widen_k(sk, H0());
    widen_v(sv, H0());
    if constexpr (CE == 16) {
      widen_k(sk, H1());
      widen_v(sv, H1());
    }
    nextk(kbeg + BK);
    nextv(kbeg + BK);
  }
  __syncthreads();

  RowState<DP> st;
  st.init();
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;
  // Step s widens tile s + 1 into its 16-bit slots between the MFMAs of tile s.  On the last
  // steps the widening writes stale bytes into the slot of a tile already consumed: harmless,
  // and the MFMA chains stay branch-free.
  for (int s = 0; s < n; ++s) {
    const int cur = s & 1, nx = cur ^ 1;
    const int t = kbeg + s * BK;
    const bool mask_tile = (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) || p.mask.window;
    f32x16 sc[BK / 32];
    i16x8 pb[BK / 16];
    char* const knext = sk + nx * TILEB;
    char* const vnext = sv + nx * TILEB;
    // The widening in pieces (5 VALU + one 16-byte LDS write each), one per MFMA gap.
    auto khook = [&](int i) {
      if constexpr (RAWLDS) {
        // Tile s + 1's bytes (DMA issued at step s − 1; V(s + 1)'s pieces may still fly).
        if (i == KP0) {
          __builtin_amdgcn_s_waitcnt(0x0F70 | NPC);
          __asm__ __volatile__("" ::: "memory");
          widen_half(knext, raw_read(rawb + nx * RSLOT, 0), zk, 0);
        }
        if (i == KP1) {
          widen_half(knext, raw_read(rawb + nx * RSLOT, 1), zk, 1);
          dmak(t + 2 * BK, cur);
        }
      } else {
        if constexpr (CE == 16)
          if (i == KP0) widen_k(knext, H0());
        if (i == KP1) {
          widen_k(knext, std::integral_constant<int, CE == 16 ? 1 : 0>());
          nextk(t + 2 * BK);
        }
      }
    };
    auto vhook = [&](int i) {
      if constexpr (RAWLDS) {
        // (K(s + 2)'s pieces, issued above, may still fly.)
        if (i == VP0) {
          __builtin_amdgcn_s_waitcnt(0x0F70 | NPC);
          __asm__ __volatile__("" ::: "memory");
          widen_half(vnext, raw_read(rawb + (2 + nx) * RSLOT, 0), zv, 0);
        }
        if (i == VP1) {
          widen_half(vnext, raw_read(rawb + (2 + nx) * RSLOT, 1), zv, 1);
          dmav(t + 2 * BK, cur);
        }
      } else {
        if constexpr (CE == 16)
          if (i == VP0) widen_v(vnext, H0());
        if (i == VP1) {
          widen_v(vnext, std::integral_constant<int, CE == 16 ? 1 : 0>());
          nextv(t + 2 * BK);
        }
      }
    };
    fwd2_qk<E, DP, BK>(sk + cur * TILEB, rbase, qf, st, sc, khook);
    fwd2_softmax<E, DP, BK>(st, sc, pb, t, mask_tile, qi, p, c, wsz, hh);
    fwd2_pv<E, DP, BK>(sv + cur * TILEB, trb, pb, st, vhook);
    __syncthreads();
  }

  float l = cross_half_sum(st.lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if constexpr (!OIMG) {
    // D = 256: two 128-row images do not fit; rows leave from registers, as the 16-bit
    // shared-tile kernel's do at this width.
    if (qi < p.R) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
    return;
  } else {
    // Both blocks leave through O row images (one per group) as whole rows from all 8 waves.
    const float inv = p.o_mul / l;
    char* orow = smem + (g * 128 + wg * 32 + l32) * ORS;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
            make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                        st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
    if (hh == 0 && qi < p.R) store_l(p, st.m + __log2f(l), b, h, qi);
    __syncthreads();
    float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
    for (int blk = 0; blk < 2; ++blk) {
      const int qb = (2 * pi + blk) * BQ;
      store_o_image<DP, 128, NT, true>(p, obase, smem + blk * 128 * ORS, ORS, qb, tid,
                                       qb + BQ <= p.R && p.D == DP);
    }
  }
}

// (DP, BK) per padded head width: the 16-bit shared-tile kernel's tile depths.
template <int DP>
constexpr int kv8_bk() { return DP == 256 ? 32 : 64; }

template <int DP>
constexpr size_t kv8_lds() {
  constexpr int BK = kv8_bk<DP>();
  constexpr int RING = 4 * BK * DP * 2;
  constexpr int OIMG = 2 * 128 * (DP * 4 + 16);
  // D = 256: the ring plus the byte ring (4 slots x 512 chunks of at most 16 bytes).
  return OIMG > 160 * 1024 ? RING + 4 * 512 * 16 : (RING > OIMG ? RING : OIMG);
}

size_t fwd_kv8_lds_bytes(int DP) {
  return DP == 64 ? kv8_lds<64>() : DP == 128 ? kv8_lds<128>() : kv8_lds<256>();
}

template <class E, int DP>
static hipError_t launch_kv8(const FwdParams& q, int src, dim3 grid, hipStream_t stream) {
  constexpr int BK = kv8_bk<DP>();
  if constexpr (DP <= 128) {
    if (q.k.bscale) {
      if (src == SRC_I8)
        return launch(mfa_fwd2_kv8_kernel<E, DP, BK, SRC_I8, true>, grid, dim3(512), kv8_lds<DP>(),
                      stream, q);
      if (src == SRC_I4)
        return launch(mfa_fwd2_kv8_kernel<E, DP, BK, SRC_I4, true>, grid, dim3(512), kv8_lds<DP>(),
                      stream, q);
      return hipErrorNotSupported;
    }
  } else {
    if (q.k.bscale) return hipErrorNotSupported;
  }
  if (src == SRC_I8)
    return launch(mfa_fwd2_kv8_kernel<E, DP, BK, SRC_I8>, grid, dim3(512), kv8_lds<DP>(), stream, q);
  if (src == SRC_I4)
    return launch(mfa_fwd2_kv8_kernel<E, DP, BK, SRC_I4>, grid, dim3(512), kv8_lds<DP>(), stream, q);
  return hipErrorNotSupported;
}

hipError_t fwd_kv8_dispatch(const FwdParams& p, int elem, int DP, int src, hipStream_t stream) {
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  const dim3 grid(npairs * p.B * p.H);
#define MFA_KV8(ELEM, EE, DPV) \
  if (elem == ELEM && DP == DPV) return launch_kv8<EE, DPV>(q, src, grid, stream);
  MFA_KV8(P_FP16, F16, 64)
  MFA_KV8(P_FP16, F16, 128)
  MFA_KV8(P_FP16, F16, 256)
  MFA_KV8(P_BF16, BF16, 64)
  MFA_KV8(P_BF16, BF16, 128)
  MFA_KV8(P_BF16, BF16, 256)
#undef MFA_KV8
  return hipErrorNotSupported;
}

}  // namespace mfa
