// attention_fwd_v2.hip — second-generation forward for 16-bit operands on gfx950.
//
// Same algorithm and numerics contract as attention_fwd.hip (the reference forward,
// AttentionKernel+Source.swift:372-416: S = QK^T, base-2 online softmax, O = PV / l,
// L = m + log2 l), restricted to fp16/bf16 Q/K/V with contiguous 16-byte aligned rows,
// D % 8 == 0, D <= DP ∈ {64, 128, 256}, a positive softmax scale, and at most causal /
// sliding-window masks whose fully masked tiles may be skipped (so no row is masked
// everywhere).  The host routes everything else to the other kernels.
//
// What is different from the first-generation forward (attention_fwd_fast.hip, removed in round
// 5), all aimed at the VALU work per MFMA (the binding limit of that kernel):
//   * K/V tiles land by LDS-DMA in the sub-tiled TileA image, so every fragment read is a base
//     register plus an immediate (no per-read address arithmetic);
//   * fp16: Q is pre-scaled by c = scale·log2(e) in registers and the first QK^T MFMA of each
//     chain accumulates onto a register tile holding −m (the running row max), so the MFMA
//     output already is S·c − m and P = exp2(S') needs no subtract or multiply per element.
//     (bf16 keeps the fused multiply-add: pre-scaling would round Q·c to 8 bits.);
//   * built with MFMA accumulators in VGPRs (Makefile): the in-loop O rescale would otherwise
//     make hipcc copy all of O between AGPRs and VGPRs every iteration; D=256 then fits in
//     244 registers and runs two waves per SIMD;
//   * masked scores are −inf: with no fully masked row the reference's finite mask value and
//     −inf give the same P (exactly 0) and the same O and L.
// Lazy rescaling (threshold 8 in log2 units, cdna_hip_programming.md T13) is kept: the running
// max and the −m tile change only when a tile's max exceeds m + 8.
#include "attention_fwd2.h"
#include "kv_bytes.h"

namespace mfa {

// ---------------------------------------------------------------------------------------
// Rows with no unmasked key (empty sparse range, or a range the causal / window predicates
// empty).  The reference masks with a finite value (AttentionKernel+Softmax.swift:257), so
// such a row sees the same score for every key: P = 1, O = Σ_k V_k / C, and L = m + log2 C
// with m = (mask value)·c as the forward computes it.  The tuned forward masks with -inf and
// skips tiles, so the wave owning such a row writes it afterwards: lanes across the head
// dimension, keys summed in order.
__device__ __forceinline__ bool masked_everywhere(const FwdParams& p, uint32_t x, uint32_t y,
                                                  int q) {
  int64_t lo = x, hi = min((int64_t)y, (int64_t)p.C);
  if (p.mask.causal) hi = min(hi, (int64_t)q + 1);
  if (p.mask.window) lo = max(lo, (int64_t)q - (int64_t)p.mask.window_size);
  return lo >= hi;
}

// The wave's empty rows (bit r of `rows`: row q0w + r) all get the same mean of V, so it is
// summed once per wave (keys in order, lanes across the head dimension) and written to each;
// a per-row sum made block-sparse patterns with many empty rows cost O(rows·C·D/64).
template <class E, int DP>
__device__ __forceinline__ void fill_masked_rows(const FwdParams& p, int b, int h, int kvh, int q0w,
                                                 uint64_t rows, int lane) {
  constexpr int NDV = (DP + 63) / 64;
  const uint16_t* vbase = (const uint16_t*)p.v.ptr + (int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh;
  const float l = (float)p.C;
  float acc[NDV];
#pragma unroll
  for (int j = 0; j < NDV; ++j) {
    const int d = lane + 64 * j;
    acc[j] = 0.f;
    if (d < p.D)
      for (int k = 0; k < p.C; ++k) acc[j] += E::to_f32(vbase[(int64_t)k * p.v.ss + (int64_t)d * p.v.sd]);
    acc[j] *= p.o_mul / l;
  }
  const float L = mul_rn(kMaskValue, p.c_log2) + __log2f(l);
  while (rows) {
    const int q = q0w + __builtin_ctzll(rows);
    rows &= rows - 1;
    float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)q * p.o_ss;
#pragma unroll
    for (int j = 0; j < NDV; ++j)
      if (lane + 64 * j < p.D) orow[(int64_t)(lane + 64 * j) * p.o_sd] = acc[j];
    if (lane == 0) store_l(p, L, b, h, q);
  }
}

// ---------------------------------------------------------------------------------------
// One 128-row query block per workgroup (4 waves x 32 rows); WPS workgroups' waves per SIMD.
template <class E, int DP, int BK, int WPS, class TU = TuneDefault>
__global__ void __launch_bounds__(256, WPS) mfa_fwd2_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128;
  constexpr int TILEB = BK * DP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  // Causal: heaviest blocks first over the whole grid (balance); otherwise each head's blocks
  // together on one XCD (L2 reuse of its K/V).
  int bh, blk;
  if (p.mask.causal) {
    bh = blockIdx.x % (p.B * p.H);
    blk = blockIdx.x / (p.B * p.H);
  } else {
    xcd_unit_block(blockIdx.x, p.B * p.H, p.nblk, &bh, &blk);
  }
  const int rb = p.nblk - 1 - blk;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  MFA_STAMP(0);
  MFA_CYC(0);
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  int kbeg, kend;
  key_range(p, q0, BQ, BK, &kbeg, &kend);
  // Sparse ranges (SparseMQABuilder, AttentionKernel+Softmax.swift:278-304): the row's keys
  // [x, y); tiles outside the union of the block's non-empty ranges are skipped.  Rows left
  // with no unmasked key are written by their wave after the loop (fill_masked_rows: the
  // reference's finite mask value makes them a uniform average over every key).
  int rlo = -0x40000000, rhi = 0x3fffffff;
  int in_lo = 0, in_hi = 0x3fffffff;  // keys inside every non-empty range of the block
  bool row_empty = false;
  if (p.mask.ranges) {
    uint32_t x = 0u, y = 0u;
    if (qvalid) {
      const uint32_t* rp = p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + qi);
      x = rp[0];
      y = rp[1];
      row_empty = masked_everywhere(p, x, y, qi);
    }
    rlo = (int)min(x, 0x3fffffffu);
    rhi = (int)min(y, 0x3fffffffu) - 1;
    // Empty rows are rewritten afterwards, so they constrain neither the union nor the
    // range-free interior.
    const bool ne = x < y;
    int mn = ne ? rlo : 0x3fffffff, mx = ne ? rhi + 1 : 0;
    in_lo = ne ? rlo : 0;
    in_hi = ne ? rhi + 1 : 0x3fffffff;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o));
      mx = max(mx, __shfl_xor(mx, o));
      in_lo = max(in_lo, __shfl_xor(in_lo, o));
      in_hi = min(in_hi, __shfl_xor(in_hi, o));
    }
    int* red = reinterpret_cast<int*>(smem);
    if (lane == 0) {
      red[4 * wave] = mn;
      red[4 * wave + 1] = mx;
      red[4 * wave + 2] = in_lo;
      red[4 * wave + 3] = in_hi;
    }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      mn = min(mn, red[4 * w]);
      mx = max(mx, red[4 * w + 1]);
      in_lo = max(in_lo, red[4 * w + 2]);
      in_hi = min(in_hi, red[4 * w + 3]);
    }
    __syncthreads();  // the reduction slots are the first K slot's bytes
    kbeg = max(kbeg, (mn / BK) * BK);
    kend = min(kend, mx);
  }
  DmaA<DP, BK, NT> kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;
  if (kbeg < kend) {
    kd.issue(khead, kbeg, kb0);
    vd.issue(vhead, kbeg, vb0);
  }
  i16x8 qf[DP / 16];
  load_q2<E, DP>(qf, p, b, h, qi, qvalid, hh, c);
  RowState<DP> st;
  st.init();
  wait_vm();
  __syncthreads();
  MFA_STAMP(1);
  MFA_ACC_DECL();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool nxt = t + BK < kend;
    if (!TU::SPREAD && nxt) {
      kd.issue(khead, t + BK, kb0 + (cur ^ 1) * TILEB);
      vd.issue(vhead, t + BK, vb0 + (cur ^ 1) * TILEB);
    }
    MFA_ACC(0);
    auto hook = [&](int i) {
      if constexpr (TU::SPREAD) {
        constexpr int PPW = DmaA<DP, BK, NT>::PPW;
        if ((i & 1) == 0 && i / 2 < 2 * PPW && nxt) {
          const int k = i / 2;
          if (k < PPW)
            kd.issue_piece(khead, t + BK, kb0 + (cur ^ 1) * TILEB, k);
          else
            vd.issue_piece(vhead, t + BK, vb0 + (cur ^ 1) * TILEB, k - PPW);
        }
      }
    };
    const bool mask_tile = (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) ||
                           p.mask.window || t < in_lo || t + BK > in_hi;
    fwd2_tile<E, DP, BK, TU>(kb0 + cur * TILEB, vb0 + cur * TILEB, rbase, trb, qf, st, t, mask_tile,
                         qi, p, c, wsz, hh, hook, rlo, rhi);
    MFA_ACC(1);
    wait_vm();
    __syncthreads();
    MFA_ACC(2);
    cur ^= 1;
  }
  MFA_ACC_END();

  MFA_STAMP(2);
  float l = cross_half_sum(st.lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if (qvalid && !row_empty) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
  if (p.mask.ranges) {
    // The wave writes its rows with no unmasked key itself (rare).
    const uint64_t todo = __ballot(row_empty && hh == 0);
    if (todo) fill_masked_rows<E, DP>(p, b, h, kvh, q0 + wave * 32, todo, lane);
  }
  MFA_STAMP(3);
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(4);
}

// ---------------------------------------------------------------------------------------
// Causal balance: two groups of NWG waves.  A workgroup owns the mirrored pair of query
// blocks (i, nblk-1-i) of NWG*32 rows (equal causal work per workgroup); inside each block
// group 0 takes the first half of the key tiles and group 1 the second half, and the two
// partial softmax states (O, m, l) merge through LDS before group 0 stores the block.
// NWG = 4: one 512-thread workgroup per CU; NWG = 2 (64-row blocks, BK = 32): two
// independent 256-thread workgroups per CU, whose waves are not tied by a shared barrier.

// OVL: the seam between the two blocks overlaps.  The staging ring is laid out slot-major
// (slot 0 of both groups in [0, 4*TILEB), slot 1 in [4*TILEB, 8*TILEB)), so once the first
// block's loop ends, the second block's first K/V tiles and its Q fragments are issued into
// slot 0 and registers before the merge, which runs over slot 1 and beyond; block two then
// waits with a counted vmcnt that leaves block one's O stores in flight.
template <class E, int DP, int BK, int NWG, bool OVL>
__global__ void __launch_bounds__(NWG * 128, 2) mfa_fwd2_pair_kernel(FwdParams p) {
  constexpr int NT = NWG * 64, BQ = NWG * 32, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int CPR = DP / 4;                        // 16-byte O chunks per row
  constexpr int OST = BQ * CPR / (2 * NT);           // O stores per thread per block
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / NT);
  const int gt = tid % NT;
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  // K of ring slot s at kb0 + s * SLOT, V at vb0 + s * SLOT.
  constexpr int SLOT = OVL ? 4 * TILEB : TILEB;
  char* const kb0 = smem + (OVL ? g * 2 * TILEB : g * 4 * TILEB);
  char* const vb0 = kb0 + (OVL ? TILEB : 2 * TILEB);
  char* const mbase = smem + (OVL ? 4 * TILEB : 0);  // merge area / O row image

  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int pi = bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;
  MFA_STAMP(0);
  MFA_CYC(0);

  DmaA<DP, BK, NT> kd, vd;
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, gt);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, gt);
  const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
  const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;

  // This group's key range [t0, t1) of query block rb and the shared step count nA.
  auto range = [&](int rb, int& t0, int& t1, int& nA) {
    int kbeg, kend;
    key_range(p, rb * BQ, BQ, BK, &kbeg, &kend);
    const int ntile = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    nA = (ntile + 1) / 2;
    t0 = g == 0 ? kbeg : kbeg + nA * BK;
    t1 = g == 0 ? min(kend, kbeg + nA * BK) : kend;
  };

  const int rbA = pi, rbB = p.nblk - 1 - pi;
  i16x8 qf[DP / 16];
  int t0, t1, nA;
  range(rbB, t0, t1, nA);
  if (t0 < t1) {
    kd.issue(khead, t0, kb0);
    vd.issue(vhead, t0, vb0);
  }
  load_q2_raw<DP>(qf, p, b, h, rbB * BQ + wg * 32 + l32, rbB * BQ + wg * 32 + l32 < p.R, hh);
  bool counted = false;  // this block's loads were issued before the previous block's stores
  for (int which = 0; which < 2; ++which) {
    const int rb = which == 0 ? rbB : rbA;
    if (which == 1 && rbA >= rbB) break;  // odd middle block handled once
    const int q0 = rb * BQ;
    const int qi = q0 + wg * 32 + l32;
    const bool qvalid = qi < p.R;
    if (!OVL && which == 1) {
      if (t0 < t1) {
        kd.issue(khead, t0, kb0);
        vd.issue(vhead, t0, vb0);
      }
      load_q2_raw<DP>(qf, p, b, h, qi, qvalid, hh);
    }
    // Older than the (at most OST + 1) stores the previous block left in flight.
    if (OVL && counted)
      __builtin_amdgcn_s_waitcnt(0x0F70 | (OST & 15) | ((OST >> 4) << 14));
    else
      wait_vm();
    prescale_q2<E, DP>(qf, c);
    RowState<DP> st;
    st.init();
    __syncthreads();
    MFA_STAMP(1 + 3 * which);
    int cur = 0;
    for (int step = 0; step < nA; ++step) {
      const int t = t0 + step * BK;
      if (t < t1) {
        if (t + BK < t1) {
          kd.issue(khead, t + BK, kb0 + (cur ^ 1) * SLOT);
          vd.issue(vhead, t + BK, vb0 + (cur ^ 1) * SLOT);
        }
        const bool mask_tile =
            (t + BK > p.C) || (p.mask.causal && t + BK - 1 > q0) || p.mask.window;
        fwd2_tile<E, DP, BK>(kb0 + cur * SLOT, vb0 + cur * SLOT, rbase, trb, qf, st, t,
                             mask_tile, qi, p, c, wsz, hh);
        wait_vm();
      }
      __syncthreads();
      cur ^= 1;
    }

    MFA_STAMP(2 + 3 * which);
    if (which == 0) {
      range(rbA, t0, t1, nA);
      if (OVL && rbA < rbB) {
        // Every wave passed the loop's last barrier: slot 0 is free for the next block.
        if (t0 < t1) {
          kd.issue(khead, t0, kb0);
          vd.issue(vhead, t0, vb0);
        }
        const int nqi = rbA * BQ + wg * 32 + l32;
        load_q2_raw<DP>(qf, p, b, h, nqi, nqi < p.R, hh);
        // Full block: every wave issues exactly OST O stores after these loads (and group 0
        // one L store before them), so a counted wait covers the loads.
        counted = q0 + BQ <= p.R && p.D == DP;
        __asm__ __volatile__("" ::: "memory");  // keep the loads ahead of the stores
      }
    }
    // Merge group 1's partial state into group 0 through LDS.
    float* mrg = reinterpret_cast<float*>(mbase);       // [NWG waves][ND*16][64]
    float* mml = mrg + NWG * ND * 16 * 64;              // [NWG waves][2][64]
    if (g == 1) {
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mrg[((wg * ND + dt) * 16 + i) * 64 + lane] = st.o[dt][i];
      mml[(wg * 2 + 0) * 64 + lane] = st.m;
      mml[(wg * 2 + 1) * 64 + lane] = st.lh;
    }
    __syncthreads();
    float inv = 0.f;
    if (g == 0) {
      const float mb = mml[(wg * 2 + 0) * 64 + lane];
      const float lb = mml[(wg * 2 + 1) * 64 + lane];
      const float mf = fmaxf(st.m, mb);
      const float ca = __builtin_amdgcn_exp2f(st.m - mf);
      const float cb = __builtin_amdgcn_exp2f(mb - mf);
      float l = cross_half_sum(st.lh * ca + lb * cb) + kFltMin;
      if (!(l > 0.f)) l = kFltMin;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i)
          st.o[dt][i] = st.o[dt][i] * ca + mrg[((wg * ND + dt) * 16 + i) * 64 + lane] * cb;
      inv = p.o_mul / l;
      if (hh == 0 && qvalid) store_l(p, mf + __log2f(l), b, h, qi);
    }
    __syncthreads();
    // O leaves through LDS as whole rows (T21): group 0 writes its lanes' rows into a padded
    // [BQ][DP] fp32 image over the (now free) merge area, then all 2·NT threads store 16-byte
    // chunks along the rows, one wave instruction covering 1 KiB of consecutive O bytes
    // instead of 64 rows x 16 B.
    constexpr int ORS = DP * 4 + 16;  // padded row stride (bytes): conflict-free b128 writes
    if (g == 0) {
      char* orow = mbase + (wg * 32 + l32) * ORS;
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
          *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
              make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                          st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
    }
    __syncthreads();
    {
      float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
      for (int k = 0; k < OST; ++k) {
        const int idx = k * 2 * NT + tid;
        const int r = idx / CPR, d = (idx % CPR) * 4;
        if (q0 + r < p.R && d < p.D)
          *reinterpret_cast<float4*>(obase + (int64_t)(q0 + r) * p.o_ss + d) =
              *reinterpret_cast<const float4*>(mbase + r * ORS + d * 4);
      }
    }
    __syncthreads();
    MFA_STAMP(3 + 3 * which);
  }
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(7);
}

// ---------------------------------------------------------------------------------------
// Causal balance with shared K/V tiles ("share" schedule, no window).  The workgroup owns the
// mirrored pair of 128-row blocks A (light, pi: nA key tiles) and B (heavy, nblk-1-pi: nB
// tiles).  A's keys are the first nA of B's, so:
//   phase 1 (steps 0..nA-1): one tile per step, staged by all 8 waves and read by both
//     groups — group 0 (waves 0-3) with A's rows, group 1 (waves 4-7) with B's rows.  Half
//     the K/V bytes and DMA instructions of the pair kernel for these steps;
//   phase 2: B's remaining nB - nA tiles, split between the groups (each with its own ring,
//     one tile each per step, as in the pair kernel).  Group 0 enters it with B's rows: it
//     stores A's O and L from registers at the switch and takes B's Q from LDS, where it
//     staged them by DMA during the last shared step.
// Steps: nA + ceil((nB - nA) / 2) — 33 for every workgroup at C2, as in the pair kernel.  B's
// two partial states merge through LDS at the end.  LDS: ring 0 (shared, then group 0's),
// ring 1 (group 1's), group 0's Q staging: 160 KiB at D = 128.
// MIRROR = false (no mask): the pair is two adjacent blocks (2·pi, 2·pi + 1) with the same key
// range, so every step is a shared one (256 query rows per K/V tile).
// IMG: adjacent pairs — both blocks' O through LDS row images; mirrored pairs — A's O at the
// switch through the wave's Q staging region.
// DV (mirrored pairs with nA >= 2): the prologue waits for K0 and Q only — Q arrives by
// LDS-DMA like the tiles (group 0 into the Q staging, group 1 into ring 1, unused before
// phase 2) so that every prologue load is counted by hand — and step 0 waits for V0 between
// its softmax and its PV.
// Quantised K/V staging of the shared-tile kernel (KVS != SRC_SAME): a thread's byte offset of
// its chunk in a tile (out of range past D), one chunk's bytes of the tile at row t (rows past
// the end read as zeros), and one chunk's widening into the 16-bit TileA image.
template <int DP, int BK>
__device__ __forceinline__ int share_byte_off(const Kv8Geo<DP, BK>& geo, int ss, int D, int sh) {
  return geo.col < D ? geo.r * ss + (geo.col >> sh) : 0x40000000;
}
template <int CB>
__device__ __forceinline__ uint4 share_ld_bytes(const char* head, int ss, int bytes, int t, int off) {
  const int tb = t * ss;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(head + tb), (short)0, max(bytes - tb, 0), 0x00020000);
  if constexpr (CB == 16) {
    const auto a = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    return make_uint4(a[0], a[1], a[2], a[3]);
  } else {
    const auto a = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
    return make_uint4(a[0], a[1], 0u, 0u);
  }
}
template <class E, int DP, int KVS, int BK>
__device__ __forceinline__ void share_widen2(char* img, const Kv8Geo<DP, BK>& geo, const uint4 raw,
                                             float zp) {
  widen_store<E, DP, KVS, 0>(img, geo.r, geo.ch0, raw, zp);
  widen_store<E, DP, KVS, 1>(img, geo.r, geo.ch0 + 1, raw, zp);
}

// KVS: K/V storage — SRC_SAME (16-bit, LDS-DMA into the rings) or SRC_I8 / SRC_I4 per-tensor
// quantised (mfa_fwd2_share_kv8_kernel): each step widens the next step's tile(s) from
// registers into their 16-bit slots (the shared tile by all 512 threads, a group's own tile by
// its 256) and loads the bytes of the step after it (attention_fwd_kv8.hip's scheme, in this
// schedule), so the MFMA operands are those of the dequantisation pass + 16-bit kernel path.
template <class E, int DP, int BK, bool MIRROR, bool NTS, bool IMG, bool DV, int KVS>
__device__ __forceinline__ void fwd2_share_body(const FwdParams& p) {
  constexpr bool QKV = KVS != SRC_SAME;
  static_assert(!(QKV && DV), "quantised K/V: no deferred-V prologue");
  constexpr int NT = 256, BQ = 128, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int QW = 32 * DP * 2;                    // one wave's 32 Q rows
  constexpr int CPR = DP / 4;                        // 16-byte O chunks per row
  constexpr int OST = BQ * CPR / (2 * NT);           // O stores per thread (final block)
  constexpr int NSW = 4 * ND + 1;                    // stores per wave at the switch (O + L)
  static_assert(NSW < 64, "counted vmcnt");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / NT);
  const int gt = tid % NT;
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  char* const sk = smem;                  // ring 0: K slots 0, 1, then V slots 0, 1
  char* const sv = smem + 2 * TILEB;
  char* const kb0 = smem + g * 4 * TILEB; // this group's ring in phase 2
  char* const vb0 = kb0 + 2 * TILEB;
  char* const qstg = smem + 8 * TILEB + wg * QW;

  const int BH = p.B * p.H;
  int pi = blockIdx.x / BH;
  int bh = blockIdx.x % BH;
  // Adjacent (unmasked) pairs: each XCD walks one head's pairs at a time (xcd_unit_block), so
  // the K/V of the heads in flight on an XCD stay in its 4 MiB L2 (a head's K/V is 4 MiB at
  // S 8192 D 128 and at S 4096 D 256); dealt round-robin, an XCD held 2-8 heads at once.
  if (!MIRROR && p.xcd_heads) xcd_unit_block(blockIdx.x, BH, (p.nblk + 1) / 2, &bh, &pi);
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = 0x3fffffff;
  MFA_STAMP(0);
  MFA_CYC(0);
  if (MIRROR && pi >= p.pro_split) {
    // Light pairs: the heavy pairs' prologue (Q of both blocks, the first tiles: every CU at
    // once, HBM-bound) goes first.
    for (int i = 0; i < p.pro_delay; ++i) __builtin_amdgcn_s_sleep(8);
  }

  DmaA<DP, BK, NT> kd, vd;         // a group's own tiles
  DmaA<DP, BK, 2 * NT> ksh, vsh;   // shared tiles, staged by all 8 waves
  constexpr int KSH = KVS == SRC_I4 ? 1 : 0;  // INT4: element -> byte offsets
  auto head_of = [&](const Operand& op) {
    const int64_t e = (int64_t)b * op.sb + (int64_t)kvh * op.sh;
    return (const char*)op.ptr + (QKV ? e >> KSH : e * 2);
  };
  const char* khead = head_of(p.k);
  const char* vhead = head_of(p.v);
  if constexpr (!QKV) {
    kd.init((int)p.k.ss * 2, p.C, p.D * 2, gt);
    vd.init((int)p.v.ss * 2, p.C, p.D * 2, gt);
    ksh.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
    vsh.init((int)p.v.ss * 2, p.C, p.D * 2, tid);
  }

  // Adjacent pairs: an odd last block leaves group 1 without rows (it still stages tiles).
  const int rbA = MIRROR ? pi : 2 * pi;
  const int rbB = MIRROR ? p.nblk - 1 - pi : 2 * pi + 1;
  int a0, a1, b0, b1;
  key_range(p, rbA * BQ, BQ, BK, &a0, &a1);
  key_range(p, MIRROR ? rbB * BQ : rbA * BQ, BQ, BK, &b0, &b1);
  // Sparse ranges (adjacent pairs; SparseMQABuilder.swift:30-62, AttentionKernel+Softmax.swift:
  // 278-304): each row's keys [x, y).  The pair stages the tiles between the first and last key
  // any of its 256 rows keeps; a group computes only the tiles that meet its own block's union,
  // masks with its rows' ranges (no mask on tiles inside every range of the block), and rows
  // left with no unmasked key are written after the loop (fill_masked_rows).
  int rlo = -0x40000000, rhi = 0x3fffffff, in_lo = 0, in_hi = 0x3fffffff;
  int g_lo = 0, g_hi = 0x3fffffff;  // this group's block union
  bool row_empty = false;
  if (!MIRROR && p.mask.ranges) {
    const int qr = (g == 0 ? rbA : rbB) * BQ + wg * 32 + l32;
    uint32_t x = 0u, y = 0u;
    if (qr < p.R) {
      const uint32_t* rp = p.mask.ranges + 2 * ((int64_t)(b * p.Hkv + kvh) * p.R + qr);
      x = rp[0];
      y = rp[1];
      row_empty = masked_everywhere(p, x, y, qr);
    }
    rlo = (int)min(x, 0x3fffffffu);
    rhi = (int)min(y, 0x3fffffffu) - 1;
    const bool ne = x < y;
    int mn = ne ? rlo : 0x3fffffff, mx = ne ? rhi + 1 : 0;
    in_lo = ne ? rlo : 0;
    in_hi = ne ? rhi + 1 : 0x3fffffff;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      mn = min(mn, __shfl_xor(mn, o));
      mx = max(mx, __shfl_xor(mx, o));
      in_lo = max(in_lo, __shfl_xor(in_lo, o));
      in_hi = min(in_hi, __shfl_xor(in_hi, o));
    }
    int* red = reinterpret_cast<int*>(smem);
    if (lane == 0) {
      const int wv = tid >> 6;
      red[4 * wv] = mn;
      red[4 * wv + 1] = mx;
      red[4 * wv + 2] = in_lo;
      red[4 * wv + 3] = in_hi;
    }
    __syncthreads();
    int umn = 0x3fffffff, umx = 0;
    g_lo = 0x3fffffff;
    g_hi = 0;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) {
      umn = min(umn, red[4 * w8]);
      umx = max(umx, red[4 * w8 + 1]);
      if (w8 / 4 == g) {
        g_lo = min(g_lo, red[4 * w8]);
        g_hi = max(g_hi, red[4 * w8 + 1]);
        in_lo = max(in_lo, red[4 * w8 + 2]);
        in_hi = min(in_hi, red[4 * w8 + 3]);
      }
    }
    __syncthreads();  // the reduction slots are the first K slot's bytes
    b0 = max(b0, (umn / BK) * BK);
    b1 = min(b1, umx);
  }
  const int nB = b1 > b0 ? (b1 - b0 + BK - 1) / BK : 0;
  // Mirrored: the odd middle block is B only.
  const int nA = !MIRROR ? nB : rbA < rbB && a1 > a0 ? (a1 - a0 + BK - 1) / BK : 0;
  const int n2 = nB - nA;            // phase-2 tiles
  const int h0 = (n2 + 1) / 2;       // group 0's share of them
  const int S = nA + h0;
  // Tile index of this group at step s (group 0: s; group 1: s, then s + h0); false past its
  // range.
  auto tile = [&](int s, int& t) -> bool {
    const int i = (g == 1 && s >= nA) ? s + h0 : s;
    t = b0 + i * BK;
    return s < S && i < nB;
  };

  // QKV: the bytes of one step's tile(s) in registers — the shared tile's chunk of this thread
  // (Kv8Geo over 512 threads), or two chunks of the group's own tile (over its 256 threads).
  // Range-checked buffer loads: rows past C and chunks past D read as zeros (their widened
  // values -zp meet masked keys, or Q / output columns past D).
  using Geo = Kv8Geo<DP, BK>;
  constexpr int CB = 16 >> KSH;  // stored bytes per 16-element chunk
  uint4 rk0 = make_uint4(0u, 0u, 0u, 0u), rk1 = rk0, rv0 = rk0, rv1 = rk0;  // shared chunk in rk0 / rv0
  // (a group tile: two chunks, 0 and 1)
  const float zk = (float)p.k.zp, zv = (float)p.v.zp;
  const int kss = QKV ? (int)(p.k.ss >> KSH) : 0, vss = QKV ? (int)(p.v.ss >> KSH) : 0;
  const int kbytes = QKV ? (int)((int64_t)(p.C - 1) * kss + (p.D >> KSH)) : 0;
  const int vbytes = QKV ? (int)((int64_t)(p.C - 1) * vss + (p.D >> KSH)) : 0;
  const Geo gs(tid), g0(gt), g1(gt + 256);  // shared chunk; the group tile's two chunks
  const int kos = share_byte_off(gs, kss, p.D, KSH), vos = share_byte_off(gs, vss, p.D, KSH);
  const int ko0 = share_byte_off(g0, kss, p.D, KSH), vo0 = share_byte_off(g0, vss, p.D, KSH);
  const int ko1 = share_byte_off(g1, kss, p.D, KSH), vo1 = share_byte_off(g1, vss, p.D, KSH);
  // Staging, written out in place (closures holding references to these registers, or
  // assignments to them under data-dependent branches, kept them in scratch).  Step s2's bytes:
  // the shared tile's chunk (rk0 / rv0; the second loads read nothing) or the group tile's two
  // chunks; a step without a tile for this group reads nothing (zero bytes in range).
#define QKV_LOAD(S2)                                                                         \
  do {                                                                                       \
    int t_;                                                                                  \
    const bool sh_ = (S2) < nA;                                                              \
    const bool has_ = tile((S2), t_) || sh_;                                                 \
    if (sh_) t_ = b0 + (S2) * BK;                                                            \
    const int kb_ = has_ ? kbytes : 0, vb_ = has_ ? vbytes : 0;                              \
    rk0 = share_ld_bytes<CB>(khead, kss, kb_, t_, sh_ ? kos : ko0);                          \
    rv0 = share_ld_bytes<CB>(vhead, vss, vb_, t_, sh_ ? vos : vo0);                          \
    rk1 = share_ld_bytes<CB>(khead, kss, sh_ ? 0 : kb_, t_, ko1);                            \
    rv1 = share_ld_bytes<CB>(vhead, vss, sh_ ? 0 : vb_, t_, vo1);                            \
  } while (0)
  // Step s1's tile(s) from the registers into 16-bit slot SL of the shared or the group's ring.
#define QKV_WIDEN(S1, SL)                                                                    \
  do {                                                                                       \
    int t_;                                                                                  \
    const bool sh_ = (S1) < nA;                                                              \
    if (sh_ || tile((S1), t_)) {                                                             \
      char* const kd_ = (sh_ ? sk : kb0) + (SL) * TILEB;                                     \
      char* const vd_ = (sh_ ? sv : vb0) + (SL) * TILEB;                                     \
      const int r_ = sh_ ? gs.r : g0.r, c_ = sh_ ? gs.ch0 : g0.ch0;                          \
      widen_store<E, DP, KVS, 0>(kd_, r_, c_, rk0, zk);                                      \
      widen_store<E, DP, KVS, 1>(kd_, r_, c_ + 1, rk0, zk);                                  \
      widen_store<E, DP, KVS, 0>(vd_, r_, c_, rv0, zv);                                      \
      widen_store<E, DP, KVS, 1>(vd_, r_, c_ + 1, rv0, zv);                                  \
      if (!sh_) {                                                                            \
        widen_store<E, DP, KVS, 0>(kd_, g1.r, g1.ch0, rk1, zk);                              \
        widen_store<E, DP, KVS, 1>(kd_, g1.r, g1.ch0 + 1, rk1, zk);                          \
        widen_store<E, DP, KVS, 0>(vd_, g1.r, g1.ch0, rv1, zv);                              \
        widen_store<E, DP, KVS, 1>(vd_, g1.r, g1.ch0 + 1, rv1, zv);                          \
      }                                                                                      \
    }                                                                                        \
  } while (0)

  int q0 = (g == 0 && (nA > 0 || !MIRROR) ? rbA : rbB) * BQ;
  int qi = q0 + wg * 32 + l32;
  i16x8 qf[DP / 16];
  DmaA<DP, 32, 64> qd;  // this wave's 32 Q rows (group 0: B's, staged for the switch)
  qd.init((int)p.q.ss * 2, p.R, p.D * 2, lane);
  const char* qhead = (const char*)p.q.ptr + ((int64_t)b * p.q.sb + (int64_t)h * p.q.sh) * 2;
  RowState<DP> st;
  st.init();
  const bool dv = DV && nA >= 2;
  if (dv) {
    char* const qdst = g == 0 ? qstg : smem + 4 * TILEB + wg * QW;
    ksh.issue(khead, b0, sk);
    qd.issue(qhead, q0 + wg * 32, qdst);
    vsh.issue(vhead, b0, sv);
    constexpr int PV0 = DmaA<DP, BK, 2 * NT>::PPW;  // V0 pieces per wave (the youngest)
    __builtin_amdgcn_s_waitcnt(0x0F70 | PV0);
    __syncthreads();
    using A = Arith16<E, DP>;
#pragma unroll
    for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(qdst, rbase, 0, ds);
    prescale_q2<E, DP>(qf, c);
  } else if constexpr (QKV) {
    // Bytes of step 0's tile(s), widened into slot 0; then step 1's bytes.
    QKV_LOAD(0);
    load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
    QKV_WIDEN(0, 0);
    QKV_LOAD(1);
    prescale_q2<E, DP>(qf, c);
    __syncthreads();
  } else {
    if (nA > 0) {
      ksh.issue(khead, b0, sk);
      vsh.issue(vhead, b0, sv);
    } else {
      int t;
      if (tile(0, t)) {
        kd.issue(khead, t, kb0);
        vd.issue(vhead, t, vb0);
      }
    }
    load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
    wait_vm();
    prescale_q2<E, DP>(qf, c);
    __syncthreads();
  }

  const bool full_sw = rbA * BQ + BQ <= p.R && p.D == DP;  // every switch store is issued
  auto step = [&](int s, bool sw, auto first_c) {
    constexpr bool FIRST = decltype(first_c)::value;  // step 0 of the deferred-V prologue
    // Stage the next step's tile(s) into the slot read two steps ago.
    const int nx = (s + 1) & 1;
    if constexpr (QKV) {
      // The next step's tile(s) widened from the bytes loaded a step ago; then the bytes of the
      // step after it.
      QKV_WIDEN(s + 1, nx);
      QKV_LOAD(s + 2);
    } else if (s + 1 < nA) {
      ksh.issue(khead, b0 + (s + 1) * BK, sk + nx * TILEB);
      vsh.issue(vhead, b0 + (s + 1) * BK, sv + nx * TILEB);
    } else {
      int tn;
#ifdef MFA_ABLATE_P2_DMA
      // Diagnostic builds only (tools/diag/fwd_stamps_p2): phase 2 computes on whatever its
      // ring holds, to price its own-tile staging.  Results are wrong.
      if (s + 1 == nA && tile(s + 1, tn)) {
#else
      if (tile(s + 1, tn)) {
#endif
        kd.issue(khead, tn, kb0 + nx * TILEB);
        vd.issue(vhead, tn, vb0 + nx * TILEB);
      }
    }
    if (sw) {
      // A is complete: its O and L leave from registers (the next tiles' DMA is older than
      // these stores, so the step's counted wait below leaves them in flight).
      float l = cross_half_sum(st.lh) + kFltMin;
      if (!(l > 0.f)) l = kFltMin;
      using A = Arith16<E, DP>;
      if constexpr (MIRROR && IMG) {
        // B's Q rows first (this wave's staging region is then free), then A's O leaves
        // through that region in two column halves: the wave writes its 32 rows (row per
        // lane, 16-byte chunks XOR-swizzled by row) and reads them back as whole half-rows,
        // so each store instruction covers 4 rows x DP*2 contiguous bytes (row-per-lane stores
        // touched 32 rows x 32 B); wave-private, so no barrier.  Same store count (NSW).
        char* const wreg = qstg;  // this wave's staging region
        MFA_STAMP(4);
#pragma unroll
        for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(wreg, rbase, 0, ds);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): Q is in registers
        MFA_STAMP(5);
        constexpr int HB = DP * 2, NCH = DP / 8;  // bytes and 16-byte chunks per half-row
        const float inv = p.o_mul / l;
        const int qa0 = q0 + wg * 32;
        float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
#pragma unroll
        for (int half = 0; half < 2; ++half) {
#pragma unroll
          for (int dt = 0; dt < ND / 2; ++dt)
#pragma unroll
            for (int gq = 0; gq < 4; ++gq) {
              const int cch = dt * 8 + 2 * gq + hh;
              const f32x16& o = st.o[half * (ND / 2) + dt];
              *reinterpret_cast<float4*>(wreg + l32 * HB + ((cch ^ (l32 & (NCH - 1))) * 16)) =
                  make_float4(o[4 * gq] * inv, o[4 * gq + 1] * inv, o[4 * gq + 2] * inv,
                              o[4 * gq + 3] * inv);
            }
          __builtin_amdgcn_s_waitcnt(0xC07F);
          constexpr int RPI = 64 / NCH;  // rows per read instruction
          constexpr int NK = 32 / RPI;
          const int rl = lane / NCH, j = lane % NCH;
          float4 v[NK];
#pragma unroll
          for (int k = 0; k < NK; ++k) {
            const int r = k * RPI + rl;
            v[k] = *reinterpret_cast<const float4*>(wreg + r * HB + ((j ^ (r & (NCH - 1))) * 16));
          }
          const int col = half * (DP / 2) + 4 * j;
          if (full_sw) {
            // Whole block: unguarded stores, the row address advanced by a constant.
            float* dst = obase + (int64_t)(qa0 + rl) * p.o_ss + col;
            const int64_t rstep = (int64_t)RPI * p.o_ss;
#pragma unroll
            for (int k = 0; k < NK; ++k) st_o4<NTS>(dst + k * rstep, v[k].x, v[k].y, v[k].z, v[k].w);
          } else {
#pragma unroll
            for (int k = 0; k < NK; ++k) {
              const int r = k * RPI + rl;
              if (qa0 + r < p.R && col < p.D)
                st_o4<NTS>(obase + (int64_t)(qa0 + r) * p.o_ss + col, v[k].x, v[k].y, v[k].z, v[k].w);
            }
          }
          __builtin_amdgcn_s_waitcnt(0xC07F);  // reads done before the next half's writes
        }
        if (hh == 0 && qi < p.R) store_l(p, st.m + __log2f(l), b, h, qi);
        MFA_STAMP(6);
        __asm__ __volatile__("" ::: "memory");
        q0 = rbB * BQ;
        qi = q0 + wg * 32 + l32;
      } else {
        if (qi < p.R) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
        __asm__ __volatile__("" ::: "memory");
        q0 = rbB * BQ;
        qi = q0 + wg * 32 + l32;
#pragma unroll
        for (int ds = 0; ds < DP / 16; ++ds) qf[ds] = A::read_row_a(qstg, rbase, 0, ds);
      }
      prescale_q2<E, DP>(qf, c);
      st.init();
    }
    int tc;
    // (Sparse ranges: a group skips the tiles outside its block's union.)
    if (tile(s, tc) && tc + BK > g_lo && tc < g_hi) {
      const bool shared = s < nA;
      const char* kt = (shared ? sk : kb0) + (s & 1) * TILEB;
      const char* vt = (shared ? sv : vb0) + (s & 1) * TILEB;
      const bool mask_tile = (tc + BK > p.C) || (p.mask.causal && tc + BK - 1 > q0) ||
                             tc < in_lo || tc + BK > in_hi;
      if constexpr (FIRST) {
        // V0 is older than the next shared tile's pieces issued above.
        constexpr int NPN = 2 * DmaA<DP, BK, 2 * NT>::PPW;
        f32x16 sc[BK / 32];
        i16x8 pb[BK / 16];
        fwd2_qk<E, DP, BK>(kt, rbase, qf, st, sc);
        fwd2_softmax<E, DP, BK>(st, sc, pb, tc, mask_tile, qi, p, c, wsz, hh);
        __builtin_amdgcn_s_waitcnt(0x0F70 | NPN);
        __syncthreads();
        fwd2_pv<E, DP, BK>(vt, trb, pb, st);
      } else {
        fwd2_tile<E, DP, BK>(kt, vt, rbase, trb, qf, st, tc, mask_tile, qi, p, c, wsz, hh,
                             NoHook(), rlo, rhi);
      }
    }
    if constexpr (QKV) {
      // Only the staging of B's Q rows (LDS-DMA, issued before step nA - 1) must land here;
      // the byte loads stay in flight.
      if (s == nA - 1) wait_vm();
    } else if (sw && full_sw) {
      __builtin_amdgcn_s_waitcnt(0x0F70 | (NSW & 15) | ((NSW >> 4) << 14));
    } else {
      wait_vm();
    }
    __syncthreads();
  };
  MFA_STAMP(1);
  // Phase 1 up to its last step, which also stages B's Q rows; group 0 switches at step nA.
  int s = 0;
  using F0 = std::false_type;
  if (dv) step(s++, false, std::true_type());
  for (; s < nA - 1; ++s) step(s, false, F0());
  if (nA > 0 && n2 > 0) {
    if (g == 0) qd.issue(qhead, rbB * BQ + wg * 32, qstg);
    step(s++, false, F0());
    MFA_STAMP(2);
    step(s++, g == 0, F0());
  }
  for (; s < S; ++s) step(s, false, F0());
  MFA_STAMP(3);

  char* const mbase = smem;  // the rings are free: merge area, then the O row image
  if (n2 == 0) {
    // Group 0 holds all of A (if any), group 1 all of B: no merge.
    float l = cross_half_sum(st.lh) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    if constexpr (!MIRROR && IMG) {
      // Adjacent pairs: both blocks leave through O row images (one per group, over the free
      // ring) as whole rows from all 8 waves.
      constexpr int ORS = DP * 4 + 16;
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
        const int qb = (blk ? rbB : rbA) * BQ;
        store_o_image<DP, 128, 2 * NT, NTS>(p, obase, smem + blk * 128 * ORS, ORS, qb, tid,
                                            qb + BQ <= p.R && p.D == DP);
      }
      if (p.mask.ranges) {
        // Rows with no unmasked key: the image wrote them from an empty state; the owning wave
        // rewrites them once every store of the workgroup has completed.
        const uint64_t todo = __ballot(row_empty && hh == 0);
        wait_vm();
        __syncthreads();
        if (todo) fill_masked_rows<E, DP>(p, b, h, kvh, q0 + wg * 32, todo, lane);
      }
      return;
    }
    if (qi < p.R && (g == 1 || nA > 0) && !row_empty) store_o_l<DP>(p, st.o, st.m, l, b, h, qi, hh);
    if (p.mask.ranges) {
      const uint64_t todo = __ballot(row_empty && hh == 0);
      if (todo) fill_masked_rows<E, DP>(p, b, h, kvh, q0 + wg * 32, todo, lane);
    }
    return;
  }
  // Merge group 1's partial state of B into group 0 through LDS.
  float* mrg = reinterpret_cast<float*>(mbase);       // [4 waves][ND*16][64]
  float* mml = mrg + 4 * ND * 16 * 64;                // [4 waves][2][64]
  if (g == 1) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) mrg[((wg * ND + dt) * 16 + i) * 64 + lane] = st.o[dt][i];
    mml[(wg * 2 + 0) * 64 + lane] = st.m;
    mml[(wg * 2 + 1) * 64 + lane] = st.lh;
  }
  __syncthreads();
  float inv = 0.f;
  if (g == 0) {
    const float mb = mml[(wg * 2 + 0) * 64 + lane];
    const float lb = mml[(wg * 2 + 1) * 64 + lane];
    const float mf = fmaxf(st.m, mb);
    const float ca = __builtin_amdgcn_exp2f(st.m - mf);
    const float cb = __builtin_amdgcn_exp2f(mb - mf);
    float l = cross_half_sum(st.lh * ca + lb * cb) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        st.o[dt][i] = st.o[dt][i] * ca + mrg[((wg * ND + dt) * 16 + i) * 64 + lane] * cb;
    inv = p.o_mul / l;
    if (hh == 0 && qi < p.R) store_l(p, mf + __log2f(l), b, h, qi);
  }
  __syncthreads();
  // O leaves through LDS as whole rows (T21), as in the pair kernel.
  constexpr int ORS = DP * 4 + 16;
  if (g == 0) {
    char* orow = mbase + (wg * 32 + l32) * ORS;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq)
        *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
            make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                        st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
  }
  __syncthreads();
  float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
  store_o_image<DP, 128, 2 * NT, NTS>(p, obase, mbase, ORS, q0, tid, q0 + BQ <= p.R && p.D == DP);
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(7);
}

#undef QKV_LOAD
#undef QKV_WIDEN

template <class E, int DP, int BK, bool MIRROR, bool NTS = false, bool IMG = false, bool DV = false>
__global__ void __launch_bounds__(512, 2) mfa_fwd2_share_kernel(FwdParams p) {
  fwd2_share_body<E, DP, BK, MIRROR, NTS, IMG, DV, SRC_SAME>(p);
}

constexpr int DP_KV8 = 128;

// Causal pairs with per-tensor INT8 / INT4 K/V widened on load (mirrored schedule, non-temporal
// O image stores, A's O through the Q staging region at the switch; no deferred V).
template <class E, int DP, int BK, int KVS>
__global__ void __launch_bounds__(512, 2) mfa_fwd2_share_kv8_kernel(FwdParams p) {
  fwd2_share_body<E, DP, BK, true, true, true, false, KVS>(p);
}

// Mirrored pairs: the light half of the pairs waits 8 x 512 cycles (~2 us) before its
// prologue loads, so the heavy pairs (the critical path: ~7 us more loop than the lightest) get
// the prologue's HBM burst first.  C2, one-process A/B over delays 0/4/8/12 and splits 4/8/12
// (profiles/r06d_ab_prologue_delay.txt): 0.0733 -> 0.0721 ms at split 8 (+1.7 %), +0.4..0.7 %
// in the other two runs.  A/B knobs: MFA_FWD_DELAY (rounds), MFA_FWD_DELAY_SPLIT (first
// delayed pair index).
static void set_prologue_delay(FwdParams& q, int npairs) {
  const char* dl = mfa::dev_env("MFA_FWD_DELAY");
  const char* ds = mfa::dev_env("MFA_FWD_DELAY_SPLIT");
  q.pro_delay = dl ? atoi(dl) : 8;
  q.pro_split = ds ? atoi(ds) : npairs / 2;
}

template <class E, int DP, int BK, bool MIRROR = true>
static hipError_t launch_fwd2_share(const FwdParams& p, hipStream_t stream) {
  // Adjacent pairs use ring 0 only (every step is shared, no merge).
  constexpr int RING = MIRROR ? 8 * BK * DP * 2 + 4 * 32 * DP * 2 : 4 * BK * DP * 2;
  constexpr int MERGE = 4 * (DP / 32) * 16 * 64 * 4 + 4 * 2 * 64 * 4;
  constexpr int OIMG = 128 * (DP * 4 + 16);
  constexpr int LDS = !MIRROR ? RING
                      : RING > MERGE ? (RING > OIMG ? RING : OIMG) : (MERGE > OIMG ? MERGE : OIMG);
  constexpr int LDS_IMG = 2 * OIMG > RING ? 2 * OIMG : RING;  // adjacent pairs, two O images
  static_assert(LDS <= 160 * 1024, "LDS");
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int npairs = (q.nblk + 1) / 2;
  {
    const char* xh = mfa::dev_env("MFA_SHARE_XCD");  // A/B: 0 deals pairs round-robin over heads
    q.xcd_heads = !(xh && xh[0] == '0');
  }
  set_prologue_delay(q, npairs);
  // Mirrored pairs store the final O image non-temporally; MFA_SHARE_NT=0 keeps plain stores
  // (A/B).
  // Mirrored pairs: deferred V0 (+1.2 % at C2 in one-process A/B) and non-temporal O image
  // stores by default; MFA_SHARE_DV=0 / MFA_SHARE_NT=0 turn them off (A/B).
  const char* dvv = mfa::dev_env("MFA_SHARE_DV");
  const char* nt = mfa::dev_env("MFA_SHARE_NT");
  // ... and A's O at the switch leaves through the wave's Q staging region as whole
  // half-rows (+0.8 % at C2; MFA_SHARE_SWI=0 keeps row-per-lane stores there).
  const char* swi = mfa::dev_env("MFA_SHARE_SWI");
  if (MIRROR && !(dvv && dvv[0] == '0') && !(nt && nt[0] == '0')) {
    if (swi && swi[0] == '0')
      return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, false, true>,
                    dim3(npairs * p.B * p.H), dim3(512), LDS, stream, q);
    return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, true, true>,
                  dim3(npairs * p.B * p.H), dim3(512), LDS, stream, q);
  }
  if constexpr (!MIRROR && LDS_IMG <= 160 * 1024) {
    // Adjacent pairs (D <= 128): both blocks leave through O row images by non-temporal
    // whole-row stores (C3 +0.8 %, C4's attention +1.9 % in one-process A/B; plain stores
    // from the images: +0.5 / +0.9 %).  MFA_SHARE_IMG=0 keeps row-per-lane stores (A/B).
    const char* im = mfa::dev_env("MFA_SHARE_IMG");
    if (!(im && im[0] == '0'))
      return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true, true>,
                    dim3(npairs * p.B * p.H), dim3(512), LDS_IMG, stream, q);
  }
  if (MIRROR && !(nt && nt[0] == '0'))
    return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR, true>, dim3(npairs * p.B * p.H),
                  dim3(512), LDS, stream, q);
  return launch(mfa_fwd2_share_kernel<E, DP, BK, MIRROR>, dim3(npairs * p.B * p.H), dim3(512),
                LDS, stream, q);
}

template <class E, int DP, int BK, int WPS, class TU = TuneDefault>
static hipError_t launch_fwd2(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = 4 * BK * DP * 2;
  auto kern = mfa_fwd2_kernel<E, DP, BK, WPS, TU>;
  return launch(kern, dim3(p.nblk * p.B * p.H), dim3(256), LDS, stream, p);
}

template <class E, int DP, int BK, int NWG, bool OVL = true>
static hipError_t launch_fwd2_pair(const FwdParams& p, hipStream_t stream) {
  constexpr int MERGE = NWG * (DP / 32) * 16 * 64 * 4 + NWG * 2 * 64 * 4;
  constexpr int OIMG = NWG * 32 * (DP * 4 + 16);
  constexpr int MB = OVL ? 4 * BK * DP * 2 : 0;  // merge area / O image base
  constexpr int RING = 8 * BK * DP * 2;
  constexpr int LDS = RING > MB + MERGE && RING > MB + OIMG ? RING
                      : (MERGE > OIMG ? MB + MERGE : MB + OIMG);
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(NWG * 32 * (DP / 4) % (NWG * 128) == 0 && NWG * 32 * (DP / 4) / (NWG * 128) < 64,
                "O stores per thread (counted vmcnt)");
  auto kern = mfa_fwd2_pair_kernel<E, DP, BK, NWG, OVL>;
  FwdParams q = p;
  q.nblk = (p.R + NWG * 32 - 1) / (NWG * 32);
  const int npairs = (q.nblk + 1) / 2;
  return launch(kern, dim3(npairs * p.B * p.H), dim3(NWG * 128), LDS, stream, q);
}

// Causal per-tensor INT8 / INT4 K/V widened on load, in the mirrored shared-tile schedule
// where fwd2_dispatch would run it for 16-bit operands (D = 128, causal only, at most ~1.5
// rounds of the chip of blocks, or up to 3 for long rows); hipErrorNotSupported elsewhere
// (the caller then takes the dequantisation pass).
hipError_t fwd_share_kv8_dispatch(const FwdParams& p, int elem, int DP, int src,
                                  hipStream_t stream) {
  // (Block-wise K/V scales: the adjacent-pair on-load kernel, attention_fwd_kv8.hip.)
  if (DP != 128 || !p.mask.causal || p.mask.window || p.mask.ranges || p.mask.amask ||
      p.k.bscale || p.v.bscale)
    return hipErrorNotSupported;
  FwdParams q = p;
  q.nblk = (p.R + 127) / 128;
  const int blocks = q.nblk * p.B * p.H;
  if (blocks > 768 && !(q.nblk >= 64 && blocks <= 1536)) return hipErrorNotSupported;
  set_prologue_delay(q, (q.nblk + 1) / 2);
  constexpr int BK = 64;
  constexpr int RING = 8 * BK * DP_KV8 * 2 + 4 * 32 * DP_KV8 * 2;
  constexpr int MERGE = 4 * (DP_KV8 / 32) * 16 * 64 * 4 + 4 * 2 * 64 * 4;
  constexpr int OIMG = 128 * (DP_KV8 * 4 + 16);
  constexpr int LDS = RING > MERGE ? (RING > OIMG ? RING : OIMG) : (MERGE > OIMG ? MERGE : OIMG);
  static_assert(LDS <= 160 * 1024, "LDS");
  const dim3 grid(((q.nblk + 1) / 2) * p.B * p.H);
#define MFA_SKV8(ELEM, EE, SRC)                                                                   \
  if (elem == ELEM && src == SRC)                                                                \
    return launch(mfa_fwd2_share_kv8_kernel<EE, DP_KV8, BK, SRC>, grid, dim3(512), LDS, stream, q);
  MFA_SKV8(P_FP16, F16, SRC_I8)
  MFA_SKV8(P_FP16, F16, SRC_I4)
  MFA_SKV8(P_BF16, BF16, SRC_I8)
  MFA_SKV8(P_BF16, BF16, SRC_I4)
#undef MFA_SKV8
  return hipErrorNotSupported;
}

// hipErrorNotSupported when the configuration is not covered (the caller falls back).
hipError_t fwd2_dispatch(const FwdParams& p, int elem, int DP, hipStream_t stream) {
  const char* var = mfa::dev_env("MFA_FWD_VARIANT");
  const int blocks = p.nblk * p.B * p.H;
  // Causal: mirrored pairs while they fill at most ~1.5 rounds of the chip, or up to 3 rounds
  // for long rows (S >= 8192: 64 blocks; one-process A/B: H16 S8192 1057 vs 987 TF single,
  // B2 H16 S8192 1027 vs 1043, B2 H16 S4096 881 vs 889).
  bool single = !p.mask.causal || DP > 128 || (blocks > 768 && !(p.nblk >= 64 && blocks <= 1536)) ||
                p.mask.ranges;
  if (var && var[0] == 's') single = true;
  if (var && var[0] == 'p' && !p.mask.ranges) single = false;
  // Development A/B of the scheduling knobs on the fp16 D=128 single-block kernel.
  if (const char* tv = mfa::dev_env("MFA_FWD2_TUNE")) {
    if (elem == P_FP16 && DP == 128 && single) {
      switch (tv[0]) {
        case '1': return launch_fwd2<F16, 128, 64, 2, Tune<8, 4>>(p, stream);
        case '2': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, false, false>>(p, stream);
        case '3': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, true, true>>(p, stream);
        case '4': return launch_fwd2<F16, 128, 128, 2>(p, stream);
        case '5': return launch_fwd2<F16, 128, 64, 2, Tune<2, 2>>(p, stream);
        case '6': return launch_fwd2<F16, 128, 64, 2, Tune<4, 3, false, true, true>>(p, stream);
        default: break;
      }
    }
  }
  const char* pv = mfa::dev_env("MFA_FWD_PAIR");
  const bool pair64 = pv && pv[0] == '2';
  // Causal pairs run the shared-tile schedule; MFA_FWD_PAIR=o keeps the pair kernel (A/B).
  const bool share = !(pv && (pv[0] == 'o' || pv[0] == '2' || pv[0] == 'n')) && !p.mask.window;
  if (pv && pv[0] == 'n' && elem == P_FP16 && DP == 128 && !single)  // A/B: serial seam
    return launch_fwd2_pair<F16, 128, 64, 4, false>(p, stream);
  // Unmasked forwards with at least a full wave of pairs: adjacent block pairs share every
  // K/V tile (256 query rows per staged tile; +6.5 % at C3 over the single-block kernel).
  // MFA_FWD_SHARE=0 keeps the single-block kernel (A/B), =1 takes the shared-tile kernel at
  // any size (tests).
  const char* sv = mfa::dev_env("MFA_FWD_SHARE");
  // (An odd block count leaves group 1 of the last pair without rows: not for nblk < 8 odd.)
  // Sparse ranges take the adjacent pairs too (D <= 128): the pair stages the union of its
  // blocks' key ranges and each group computes its own (MFA_FWD_SHARE=0 keeps the single-block
  // kernel with tile skipping).
  const bool adj = !p.mask.causal && !p.mask.window && (!p.mask.ranges || DP <= 128) && !var &&
                   (sv ? sv[0] == '1'
                       : (p.nblk % 2 == 0 || p.nblk >= 8) &&
                             (int64_t)((p.nblk + 1) / 2) * p.B * p.H >= 256);
  // Adjacent fp16 D = 128 pairs: the software-pipelined kernel with hand-placed blocks
  // (attention_fwd_pipe.hip; bit-identical, +1.1 % at C3 in one-process A/B).  MFA_FWD_PIPE=0
  // keeps the compiler-scheduled shared-tile kernel (A/B).
  if (adj && elem == P_FP16 && DP == 128) {
    const char* pp = mfa::dev_env("MFA_FWD_PIPE");
    if (!(pp && pp[0] == '0')) {
      const hipError_t e = fwd_pipe_dispatch(p, elem, DP, stream);
      if (e != hipErrorNotSupported) return e;
    }
  }
#define MFA_F2(ELEM, EE, DPV, BKV, WPS)                                          \
  if (elem == ELEM && DP == DPV && adj)                                         \
    return launch_fwd2_share<EE, DPV, BKV, false>(p, stream);                   \
  if (elem == ELEM && DP == DPV)                                                \
    return single  ? launch_fwd2<EE, DPV, BKV, WPS>(p, stream)                  \
           : share ? launch_fwd2_share<EE, DPV, BKV>(p, stream)                  \
                   : (pair64 ? launch_fwd2_pair<EE, DPV, 32, 2>(p, stream)       \
                             : launch_fwd2_pair<EE, DPV, BKV, 4>(p, stream));
  MFA_F2(P_FP16, F16, 64, 64, 2)
  MFA_F2(P_FP16, F16, 128, 64, 2)
  MFA_F2(P_BF16, BF16, 64, 64, 2)
  MFA_F2(P_BF16, BF16, 128, 64, 2)
#undef MFA_F2
  if (elem == P_FP16 && DP == 256)
    return adj ? launch_fwd2_share<F16, 256, 32, false>(p, stream) : launch_fwd2<F16, 256, 32, 2>(p, stream);
  if (elem == P_BF16 && DP == 256)
    return adj ? launch_fwd2_share<BF16, 256, 32, false>(p, stream) : launch_fwd2<BF16, 256, 32, 2>(p, stream);
  return hipErrorNotSupported;
}

#define MFA_F2_INST(EE, DPV, BKV, WPS)                                        \
  template __global__ void mfa_fwd2_kernel<EE, DPV, BKV, WPS>(FwdParams);     \
  template __global__ void mfa_fwd2_pair_kernel<EE, DPV, BKV, 4, true>(FwdParams);  \
  template __global__ void mfa_fwd2_pair_kernel<EE, DPV, 32, 2, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, true, true>(FwdParams);  \
  template __global__ void mfa_fwd2_share_kernel<EE, DPV, BKV, false>(FwdParams);
MFA_F2_INST(F16, 64, 64, 2)
MFA_F2_INST(F16, 128, 64, 2)
MFA_F2_INST(BF16, 64, 64, 2)
MFA_F2_INST(BF16, 128, 64, 2)
#undef MFA_F2_INST
template __global__ void mfa_fwd2_pair_kernel<F16, 128, 64, 4, false>(FwdParams);
template __global__ void mfa_fwd2_kernel<F16, 256, 32, 2>(FwdParams);
template __global__ void mfa_fwd2_share_kernel<F16, 256, 32, false>(FwdParams);
template __global__ void mfa_fwd2_share_kernel<BF16, 256, 32, false>(FwdParams);
template __global__ void mfa_fwd2_kernel<BF16, 256, 32, 2>(FwdParams);

}  // namespace mfa
