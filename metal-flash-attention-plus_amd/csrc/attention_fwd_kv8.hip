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
// Per-tensor scales stay folded in the softmax multiplier (K) and the output multiplier (V),
// so the MFMA operands, and hence O and L, are bit-identical to the dequantise pass +
// 16-bit kernel path — with 1 byte (INT4: half a byte) per K/V element read from HBM, no
// pass, no scratch.
// LDS: 16-bit ring 4 x 16 KiB, reused at the end for the two O row images
// (2 x 128 rows x (4·D + 16) bytes).
#include "attention_fwd2.h"

namespace mfa {

// 8 quantised elements (row r, columns 16c + 8·HALF ..+7) -> one 16-byte chunk of the TileA
// image.
// INT8: raw holds 16 bytes (half h: dwords 2h, 2h+1); INT4: 16 nibbles in raw.x, raw.y
// (half h: dword h, element 2i in the low nibble).
template <class E, int DP, int SRC, int HALF>
__device__ __forceinline__ void widen_store(char* img, int r, int c, const uint4 raw, float zp) {
  uint4 q;
  if constexpr (SRC == SRC_I8)
    q = HALF ? make_uint4(raw.z, raw.w, 0u, 0u) : make_uint4(raw.x, raw.y, 0u, 0u);
  else
    q = make_uint4(HALF ? raw.y : raw.x, 0u, 0u, 0u);
  *reinterpret_cast<uint4*>(img + TileA<DP>::off(r, 2 * c + HALF)) = dequant_fast<E, SRC>(q, zp);
}

template <class E, int DP, int BK, int SRC, int KP0 = 1, int KP1 = 3, int VP0 = 12, int VP1 = 14>
__global__ void __launch_bounds__(512, 1) mfa_fwd2_kv8_kernel(FwdParams p) {
  constexpr int NT = 512, BQ = 128, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int CPR = DP / 4;               // 16-byte O chunks per row
  constexpr int OST = BQ * CPR / NT;        // O stores per thread per block
  constexpr int ORS = DP * 4 + 16;          // O row image stride
  constexpr int C8 = DP / 16;               // 16-byte INT8 chunks per row
  static_assert(BK * C8 == NT, "one INT8 chunk of K and of V per thread per tile");
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
  const int pi = blockIdx.x / BH;
  const int bh = blockIdx.x % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const float zk = (float)p.k.zp, zv = (float)p.v.zp;

  constexpr int ESH = SRC == SRC_I8 ? 0 : 1;
  const char* khead = (const char*)p.k.ptr + (((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) >> ESH);
  const char* vhead = (const char*)p.v.ptr + (((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) >> ESH);
  const int n = (p.C + BK - 1) / BK;
  // This thread's 16-byte INT8 chunk of a tile: wave w covers rows 8w..8w+7; 16 consecutive
  // lanes take the 8 rows x 2 chunk parities, so each 16-byte write into the TileA image
  // (bank group 4·(r & 3) + ((chunk & 3) ^ ((r >> 2) & 3))) hits 16 distinct bank groups.
  static_assert(C8 == 8, "8 chunks per row");
  const int cr = (tid >> 6) * 8 + (lane & 7);
  const int cc = ((lane >> 3) & 1) | ((lane >> 4) << 1);
  const bool cvalid = cc * 16 < p.D;
  // Range-checked buffer loads: rows past C and chunks past D read as zeros.
  // Byte geometry: INT8 one byte per element, INT4 half a byte (16-element chunk: 16 / 8 B).
  constexpr int SH = SRC == SRC_I8 ? 0 : 1, CB = 16 >> SH;
  const int kss = (int)(p.k.ss >> SH), vss = (int)(p.v.ss >> SH);
  const int kbytes = (int)((int64_t)(p.C - 1) * kss + (p.D >> SH));
  const int vbytes = (int)((int64_t)(p.C - 1) * vss + (p.D >> SH));
  const int kro = cvalid ? cr * kss + cc * CB : 0x40000000;
  const int vro = cvalid ? cr * vss + cc * CB : 0x40000000;
  // This thread's chunk of tile t's K (V) bytes.
  auto load1 = [&](const char* head, int ss, int bytes, int ro, int t) -> uint4 {
    const int tb = t * ss;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(head + tb), (short)0, max(bytes - tb, 0), 0x00020000);
    if constexpr (SRC == SRC_I8) {
      const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, ro, 0, 0);
      return make_uint4(a[0], a[1], a[2], a[3]);
    } else {
      const auto a = __builtin_amdgcn_raw_buffer_load_b64(rs, ro, 0, 0);
      return make_uint4(a[0], a[1], 0u, 0u);
    }
  };
  auto loadk = [&](int t) { return load1(khead, kss, kbytes, kro, t); };
  auto loadv = [&](int t) { return load1(vhead, vss, vbytes, vro, t); };

  const int q0 = (2 * pi + g) * BQ;
  const int qi = q0 + wg * 32 + l32;
  i16x8 qf[DP / 16];
  // rk / rv: the bytes of the next tile to widen.  Each is reloaded (tile s + 2) as soon as
  // its widening into tile s + 1's slot has been issued, one step ahead of its use.
  uint4 rk = loadk(0), rv = loadv(0);
  load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
  prescale_q2<E, DP>(qf, c);
  widen_store<E, DP, SRC, 0>(sk, cr, cc, rk, zk);
  widen_store<E, DP, SRC, 1>(sk, cr, cc, rk, zk);
  widen_store<E, DP, SRC, 0>(sv, cr, cc, rv, zv);
  widen_store<E, DP, SRC, 1>(sv, cr, cc, rv, zv);
  rk = loadk(BK);
  rv = loadv(BK);
  __syncthreads();

  RowState<DP> st;
  st.init();
  const int wsz = 0x3fffffff;
  // Step s widens tile s + 1 into its 16-bit slots between the MFMAs of tile s.  On the last
  // steps the widening writes stale bytes into the slot of a tile already consumed: harmless,
  // and the MFMA chains stay branch-free.
  for (int s = 0; s < n; ++s) {
    const int cur = s & 1, nx = cur ^ 1;
    const int t = s * BK;
    const bool mask_tile = t + BK > p.C;
    f32x16 sc[BK / 32];
    i16x8 pb[BK / 16];
    char* const knext = sk + nx * TILEB;
    char* const vnext = sv + nx * TILEB;
    // The widening in four pieces (5 VALU + one 16-byte LDS write each), one per MFMA gap.
    auto khook = [&](int i) {
      if (i == KP0) widen_store<E, DP, SRC, 0>(knext, cr, cc, rk, zk);
      if (i == KP1) {
        widen_store<E, DP, SRC, 1>(knext, cr, cc, rk, zk);
        rk = loadk(t + 2 * BK);
      }
    };
    auto vhook = [&](int i) {
      if (i == VP0) widen_store<E, DP, SRC, 0>(vnext, cr, cc, rv, zv);
      if (i == VP1) {
        widen_store<E, DP, SRC, 1>(vnext, cr, cc, rv, zv);
        rv = loadv(t + 2 * BK);
      }
    };
    fwd2_qk<E, DP, BK>(sk + cur * TILEB, rbase, qf, st, sc, khook);
    fwd2_softmax<E, DP, BK>(st, sc, pb, t, mask_tile, qi, p, c, wsz, hh);
    fwd2_pv<E, DP, BK>(sv + cur * TILEB, trb, pb, st, vhook);
    __syncthreads();
  }

  // Both blocks leave through O row images (one per group) as whole rows from all 8 waves.
  float l = cross_half_sum(st.lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
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

size_t fwd_kv8_lds_bytes() {
  constexpr int DP = 128, BK = 64;
  constexpr int RING = 4 * BK * DP * 2;
  constexpr int OIMG = 2 * 128 * (DP * 4 + 16);
  return RING > OIMG ? RING : OIMG;
}

hipError_t fwd_kv8_dispatch(const FwdParams& p, int elem, int src, hipStream_t stream) {
  if (elem != P_FP16) return hipErrorNotSupported;
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  const dim3 grid(npairs * p.B * p.H);
  const size_t lds = fwd_kv8_lds_bytes();
  // MFA_KV8_SLOTS=1 (development A/B): the widening pieces at QK^T MFMAs 4 / 10 and PV 4 / 10.
  const char* sl = mfa::dev_env("MFA_KV8_SLOTS");
  const bool alt = sl && sl[0] == '1';
  if (src == SRC_I8)
    return alt ? launch(mfa_fwd2_kv8_kernel<F16, 128, 64, SRC_I8, 4, 10, 4, 10>, grid, dim3(512), lds, stream, q)
               : launch(mfa_fwd2_kv8_kernel<F16, 128, 64, SRC_I8>, grid, dim3(512), lds, stream, q);
  if (src == SRC_I4)
    return alt ? launch(mfa_fwd2_kv8_kernel<F16, 128, 64, SRC_I4, 4, 10, 4, 10>, grid, dim3(512), lds, stream, q)
               : launch(mfa_fwd2_kv8_kernel<F16, 128, 64, SRC_I4>, grid, dim3(512), lds, stream, q);
  return hipErrorNotSupported;
}

}  // namespace mfa
