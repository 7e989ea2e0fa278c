// attention_fwd_fast.hip — the forward kernel for the common case, tuned for gfx950.
//
// Same algorithm and numerics contract as attention_fwd.hip (the reference forward,
// AttentionKernel+Source.swift:372-416), restricted to what the hot configurations need so
// the loop carries no generic-path code: fp16/bf16 operands whose rows are 16-byte aligned
// (D % 8 == 0, last dimension contiguous), causal / sliding-window masks only (no additive
// mask, no sparse ranges), per-tensor INT8 K/V optional.  The host routes everything else to
// the generic kernel.
//
// Differences from the generic kernel, all exact up to fp32 rounding:
//   * two workgroups per CU (__launch_bounds__(256, 2): <= 256 VGPR+AGPR per lane), so each
//     SIMD interleaves one wave's MFMA chain with the other wave's softmax VALU work;
//   * lazy rescaling (cdna_hip_programming.md T13): the running max m is raised only when a
//     tile's max exceeds it by more than THR (P is then bounded by 2^THR instead of 1); O / l
//     and L = m + log2(l) are the same quantities whichever m the row ends with;
//   * the cross-half row max uses v_permlane32_swap instead of an LDS round trip, and the row
//     sum is kept per half-wave until the epilogue;
//   * staging issues all global loads of tile t+1 before the MFMA work on tile t and writes
//     them to the other LDS buffer after it (one barrier per tile).
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {

// K/V tile staging through range-checked buffer loads.  The descriptor is rebuilt per tile
// from wave-uniform values (base advanced to the tile's first row, num_records = the bytes
// left in the head), so rows past the end and chunks past D (offset forced out of range)
// load as zeros without per-lane branches; the per-thread offsets are loop invariant.
template <int DP, int BK, int NT, int KVSRC>
struct KVStage {
  // INT8 K/V (dequantised on the way into LDS): register staging through buffer loads.
  using T = Tile16<DP>;
  static constexpr int CPR = DP / 8;           // 8-element chunks per row
  static constexpr int PER = BK * CPR / NT;    // chunks per thread per tile
  static constexpr int RPI = NT / CPR;         // tile rows between a thread's chunks
  static constexpr int ESZ = 1;
  static_assert(PER >= 1 && BK * CPR % NT == 0 && NT % CPR == 0, "tile/thread mismatch");
  const char* kg;
  const char* vg;
  int kstep, vstep, kbytes, vbytes;
  int koff, voff, loff;  // chunk 0's offsets; chunk i is RPI rows further (same swizzle)
  uint4 rk[PER], rv[PER];

  __device__ __forceinline__ void init(const FwdParams& p, int b, int kvh, int gt) {
    kg = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * ESZ;
    vg = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * ESZ;
    kstep = (int)p.k.ss * ESZ;
    vstep = (int)p.v.ss * ESZ;
    kbytes = (int)(((int64_t)(p.C - 1) * p.k.ss + p.D) * ESZ);
    vbytes = (int)(((int64_t)(p.C - 1) * p.v.ss + p.D) * ESZ);
    const int row = gt / CPR, ch = gt % CPR;
    const bool in = ch * 8 < p.D;
    koff = in ? row * kstep + ch * 8 * ESZ : 0x40000000;
    voff = in ? row * vstep + ch * 8 * ESZ : 0x40000000;
    loff = T::off(row, ch);
  }
  __device__ __forceinline__ void load(int t) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int kb = (t + i * RPI) * kstep, vb = (t + i * RPI) * vstep;
      const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(kg + kb), (short)0, max(kbytes - kb, 0), 0x00020000);
      const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(vg + vb), (short)0, max(vbytes - vb, 0), 0x00020000);
      const auto a = __builtin_amdgcn_raw_buffer_load_b64(krs, koff, 0, 0);
      const auto v = __builtin_amdgcn_raw_buffer_load_b64(vrs, voff, 0, 0);
      rk[i] = make_uint4(a[0], a[1], 0u, 0u);
      rv[i] = make_uint4(v[0], v[1], 0u, 0u);
    }
  }
  template <class E>
  __device__ __forceinline__ void store(char* kt, char* vt, float kzp, float vzp) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      *reinterpret_cast<uint4*>(kt + loff + i * RPI * T::ROWB) = dequant_fast<E, KVSRC>(rk[i], kzp);
      *reinterpret_cast<uint4*>(vt + loff + i * RPI * T::ROWB) = dequant_fast<E, KVSRC>(rv[i], vzp);
    }
  }
};

// 16-bit K/V: LDS-DMA straight into the swizzled tile (mfa_stage.h TileDMA).
template <int DP, int BK, int NT>
struct KVStage<DP, BK, NT, SRC_SAME> {
  TileDMA<DP * 2, BK, NT> kd, vd;
  __device__ __forceinline__ void init(const FwdParams& p, int b, int kvh, int gt) {
    kd.init((const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2,
            (int)p.k.ss * 2, p.C, p.D * 2, gt);
    vd.init((const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2,
            (int)p.v.ss * 2, p.C, p.D * 2, gt);
  }
  __device__ __forceinline__ void issue(int t, char* kt, char* vt) const {
    kd.issue(t, kt);
    vd.issue(t, vt);
  }
};

// One 64-key tile of the forward for one wave (32 query rows): S^T = K·Q^T, masks, online
// softmax (lazy rescale), O^T += V^T·P^T.  Shared by the single-block and pair kernels.
template <class E, int DP, int BK>
__device__ __forceinline__ void fwd_tile(const char* kt, const char* vt,
                                         const i16x8 (&qf)[DP / 16], f32x16 (&o)[DP / 32],
                                         float& m, float& lh, int t, int q0, int qi,
                                         const FwdParams& p, float c, int wsz, int lane) {
  using A = Arith16<E, DP>;
  constexpr int NJ = BK / 32;
  constexpr float THR = 8.0f;  // lazy-rescale threshold (log2 units)
  const int l32 = lane & 31, hh = lane >> 5;
  f32x16 s[NJ];
#pragma unroll
  for (int j = 0; j < NJ; ++j) s[j] = zero16();
  {
    // K fragments are read QK_AHEAD MFMAs ahead of their use; sched_barrier(0) pins the
    // order (left alone, hipcc issues each read right before its MFMA and waits on it).
    constexpr int NM = A::DSTEPS * NJ;
    constexpr int AH = 4;
    i16x8 kf[AH];
#pragma unroll
    for (int i = 0; i < AH; ++i) kf[i] = A::read_row(kt, (i % NJ) * 32 + l32, i / NJ, hh);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int ds = i / NJ, j = i % NJ;
      s[j] = A::mma(kf[i % AH], qf[ds], s[j]);
      if (i + AH < NM)
        kf[i % AH] = A::read_row(kt, ((i + AH) % NJ) * 32 + l32, (i + AH) / NJ, hh);
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  // Masks: only tiles that reach past the diagonal / edge / window.
  const bool edge = t + BK > p.C;
  const bool diag = p.mask.causal && t + BK - 1 > q0;
  if (edge || diag || p.mask.window) {
    MFA_KEEP_BRANCH();
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = t + j * 32 + acc_row(i, hh);
        float x = s[j][i];
        if ((p.mask.causal && key > qi) || (p.mask.window && qi - key > wsz)) x = kMaskValue;
        if (key >= p.C) x = -__builtin_inff();
        s[j][i] = x;
      }
  }

  float mx = s[0][0];
#pragma unroll
  for (int j = 0; j < NJ; ++j)
#pragma unroll
    for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[j][i]);
  const float m_tile = cross_half_max(mx) * c;
  if (__any(m_tile > m + THR)) {
    const float m_new = fmaxf(m, m_tile);
    const float corr = __builtin_amdgcn_exp2f(m - m_new);
    m = m_new;
    lh *= corr;
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
      for (int i = 0; i < 16; ++i) o[dt][i] *= corr;
  }
  // P = exp2(s·c − m); four independent partial row sums keep the adds off one serial chain.
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  if (__any(m < kMaskLevel)) {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = __builtin_amdgcn_exp2f(mul_rn(s[j][i], c) - m);
        s[j][i] = pv;
        rs[i & 3] += pv;
      }
  } else {
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[j][i], c, -m));
        s[j][i] = pv;
        rs[i & 3] += pv;
      }
  }
  lh += (rs[0] + rs[1]) + (rs[2] + rs[3]);

  {
    // V^T fragments (two tr-reads each) PV_AHEAD MFMAs ahead, order pinned as above.
    constexpr int ND = DP / 32;
    constexpr int NM = NJ * 2 * ND;
    constexpr int AH = 3;
    i16x8 pb[NJ * 2];
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) pb[j * 2 + ks] = A::pack(s[j], ks);
    i16x8 vf[AH];
#pragma unroll
    for (int i = 0; i < AH; ++i) {
      const int jk = i / ND, dt = i % ND;
      vf[i] = A::read_tr(vt, (jk >> 1) * 32, jk & 1, dt * 32, lane);
    }
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const int jk = i / ND, dt = i % ND;
      o[dt] = A::mma(vf[i % AH], pb[jk], o[dt]);
      if (i + AH < NM) {
        const int jn = (i + AH) / ND, dn = (i + AH) % ND;
        vf[i % AH] = A::read_tr(vt, (jn >> 1) * 32, jn & 1, dn * 32, lane);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

template <class E, int DP, int BK, int KVSRC>
__global__ void __launch_bounds__(256, 2) mfa_fwd_fast_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128;
  constexpr int TILEB = BK * DP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const kb0 = smem;
  char* const vb0 = smem + 2 * TILEB;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int rb = p.nblk - 1 - bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const int q0 = rb * BQ;
  const int qi = q0 + wave * 32 + l32;
  const bool qvalid = qi < p.R;

  i16x8 qf[DP / 16];
#pragma unroll
  for (int s = 0; s < DP / 16; ++s) qf[s] = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
  {
    const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb +
                           (int64_t)h * p.q.sh + (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) {
      const int d0 = 16 * s + 8 * hh;
      if (qvalid && d0 < p.D) qf[s] = *reinterpret_cast<const i16x8*>(qrow + d0);
    }
  }

  int kend = p.C;
  if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
  int kbeg = 0;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
    kbeg = lo > 0 ? (int)(lo / BK) * BK : 0;
  }

  KVStage<DP, BK, NT, KVSRC> st;
  st.init(p, b, kvh, tid);
  const float kzp = (float)p.k.zp, vzp = (float)p.v.zp;

  f32x16 o[DP / 32];
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt) o[dt] = zero16();
  float m = -kFltMax, lh = 0.f;  // l per half-wave; l0 = FLT_MIN added at the end
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  if (kbeg < kend) {
    if constexpr (KVSRC == SRC_SAME) {
      st.issue(kbeg, kb0, vb0);
      wait_vm();
    } else {
      st.load(kbeg);
      st.template store<E>(kb0, vb0, kzp, vzp);
    }
  }
  __syncthreads();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool has_next = t + BK < kend;
    if constexpr (KVSRC == SRC_SAME) {
      // The other buffer was last read in the previous iteration (barrier since).
      if (has_next) st.issue(t + BK, kb0 + (cur ^ 1) * TILEB, vb0 + (cur ^ 1) * TILEB);
    } else {
      if (has_next) st.load(t + BK);
    }
    fwd_tile<E, DP, BK>(kb0 + cur * TILEB, vb0 + cur * TILEB, qf, o, m, lh, t, q0, qi, p, c,
                        wsz, lane);
    if constexpr (KVSRC == SRC_SAME) {
      wait_vm();
    } else {
      if (has_next)
        st.template store<E>(kb0 + (cur ^ 1) * TILEB, vb0 + (cur ^ 1) * TILEB, kzp, vzp);
    }
    __syncthreads();
    cur ^= 1;
  }

  float l = cross_half_sum(lh) + kFltMin;
  if (!(l > 0.f)) l = kFltMin;
  if (qvalid) {
    const float inv = p.o_mul / l;
    float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int d = dt * 32 + 8 * g + 4 * hh;
        if (d < p.D)
          *reinterpret_cast<float4*>(orow + d) =
              make_float4(o[dt][4 * g] * inv, o[dt][4 * g + 1] * inv, o[dt][4 * g + 2] * inv,
                          o[dt][4 * g + 3] * inv);
      }
    if (hh == 0) {
      const float L = m + __log2f(l);
      const int64_t li = (int64_t)(b * p.H + h) * p.R + qi;
      if (p.l_f16)
        reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
      else
        reinterpret_cast<float*>(p.l)[li] = L;
    }
  }
}


// ---------------------------------------------------------------------------------------
// Balanced variant: 8 waves = two groups of 4.  A workgroup owns the mirrored pair of query
// blocks (i, nblk-1-i) (equal causal work for every workgroup) and, inside each block, group 0
// takes the first half of the key tiles and group 1 the second half; the two partial softmax
// states (O, m, l) are merged through LDS before group 0 stores the block.  Each group stages
// its own K/V tiles; both groups run the same number of lock-step iterations (one barrier
// each), group 1 idling through the odd step.
template <class E, int DP, int BK, int KVSRC>
__global__ void __launch_bounds__(512, 2) mfa_fwd_pair_kernel(FwdParams p) {
  constexpr int NT = 256, BQ = 128;
  constexpr int TILEB = BK * DP * 2;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  // Group index, wave-uniform; readfirstlane makes that provable, so the per-tile buffer
  // descriptors (built from t, which depends on g) stay in SGPRs without waterfall loops.
  const int g = __builtin_amdgcn_readfirstlane(tid >> 8);
  const int gt = tid & 255;           // thread within group
  const int lane = tid & 63, wg = gt >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  char* const kb0 = smem + g * 4 * TILEB;
  char* const vb0 = kb0 + 2 * TILEB;

  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int pi = bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  KVStage<DP, BK, NT, KVSRC> st;
  st.init(p, b, kvh, gt);
  const float kzp = (float)p.k.zp, vzp = (float)p.v.zp;

  const int rbA = pi, rbB = p.nblk - 1 - pi;
  for (int which = 0; which < 2; ++which) {
    const int rb = which == 0 ? rbB : rbA;
    if (which == 1 && rbA >= rbB) break;  // odd middle block handled once
    const int q0 = rb * BQ;
    const int qi = q0 + wg * 32 + l32;
    const bool qvalid = qi < p.R;

    i16x8 qf[DP / 16];
#pragma unroll
    for (int s = 0; s < DP / 16; ++s) qf[s] = i16x8{0, 0, 0, 0, 0, 0, 0, 0};
    {
      const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb +
                             (int64_t)h * p.q.sh + (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
      for (int s = 0; s < DP / 16; ++s) {
        const int d0 = 16 * s + 8 * hh;
        if (qvalid && d0 < p.D) qf[s] = *reinterpret_cast<const i16x8*>(qrow + d0);
      }
    }
    int kend = p.C;
    if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
    int kbeg = 0;
    if (p.mask.window && p.mask.skip_ok) {
      const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
      kbeg = lo > 0 ? (int)(lo / BK) * BK : 0;
    }
    const int ntile = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
    const int nA = (ntile + 1) / 2;
    const int t0 = g == 0 ? kbeg : kbeg + nA * BK;
    const int t1 = g == 0 ? min(kend, kbeg + nA * BK) : kend;

    f32x16 o[DP / 32];
#pragma unroll
    for (int dt = 0; dt < DP / 32; ++dt) o[dt] = zero16();
    float m = -kFltMax, lh = 0.f;

    if (t0 < t1) {
      if constexpr (KVSRC == SRC_SAME) {
        st.issue(t0, kb0, vb0);
        wait_vm();
      } else {
        st.load(t0);
        st.template store<E>(kb0, vb0, kzp, vzp);
      }
    }
    __syncthreads();
    int cur = 0;
    for (int step = 0; step < nA; ++step) {
      const int t = t0 + step * BK;
      if (t < t1) {
        const bool has_next = t + BK < t1;
        if constexpr (KVSRC == SRC_SAME) {
          if (has_next) st.issue(t + BK, kb0 + (cur ^ 1) * TILEB, vb0 + (cur ^ 1) * TILEB);
        } else {
          if (has_next) st.load(t + BK);
        }
        fwd_tile<E, DP, BK>(kb0 + cur * TILEB, vb0 + cur * TILEB, qf, o, m, lh, t, q0, qi, p,
                            c, wsz, lane);
        if constexpr (KVSRC == SRC_SAME) {
          wait_vm();
        } else {
          if (has_next)
            st.template store<E>(kb0 + (cur ^ 1) * TILEB, vb0 + (cur ^ 1) * TILEB, kzp, vzp);
        }
      }
      __syncthreads();
      cur ^= 1;
    }

    // Merge group 1's partial state into group 0 through LDS (staging buffers are free).
    float* mrg = reinterpret_cast<float*>(smem);                 // [4 waves][DP/32*16][64]
    float* mml = mrg + 4 * (DP / 32) * 16 * 64;                   // [4 waves][2][64]
    if (g == 1) {
#pragma unroll
      for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) mrg[((wg * (DP / 32) + dt) * 16 + i) * 64 + lane] = o[dt][i];
      mml[(wg * 2 + 0) * 64 + lane] = m;
      mml[(wg * 2 + 1) * 64 + lane] = lh;
    }
    __syncthreads();
    if (g == 0) {
      const float mb = mml[(wg * 2 + 0) * 64 + lane];
      const float lb = mml[(wg * 2 + 1) * 64 + lane];
      const float mf = fmaxf(m, mb);
      const float ca = __builtin_amdgcn_exp2f(m - mf);
      const float cb = __builtin_amdgcn_exp2f(mb - mf);
      lh = lh * ca + lb * cb;
      float l = cross_half_sum(lh);
      if (!(l > 0.f)) l = kFltMin;
      if (qvalid) {
        const float inv = p.o_mul / l;
        float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi * p.o_ss;
#pragma unroll
        for (int dt = 0; dt < DP / 32; ++dt)
#pragma unroll
          for (int gg = 0; gg < 4; ++gg) {
            const int d = dt * 32 + 8 * gg + 4 * hh;
            float4 val;
            float* vp = &val.x;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * gg + e;
              const float ob = mrg[((wg * (DP / 32) + dt) * 16 + i) * 64 + lane];
              vp[e] = (o[dt][i] * ca + ob * cb) * inv;
            }
            if (d < p.D) *reinterpret_cast<float4*>(orow + d) = val;
          }
        if (hh == 0) {
          const float L = mf + __log2f(l);
          const int64_t li = (int64_t)(b * p.H + h) * p.R + qi;
          if (p.l_f16)
            reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
          else
            reinterpret_cast<float*>(p.l)[li] = L;
        }
      }
    }
    __syncthreads();
  }
}

template <class E, int DP, int BK, int KVSRC>
static hipError_t launch_pair(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = 8 * BK * DP * 2;  // two groups x (K, V) x double buffer
  static_assert(LDS >= 4 * (DP / 32) * 16 * 64 * 4 + 4 * 2 * 64 * 4, "merge area");
  auto kern = mfa_fwd_pair_kernel<E, DP, BK, KVSRC>;
  const int npairs = (p.nblk + 1) / 2;
  return launch(kern, dim3(npairs * p.B * p.H), dim3(512), LDS, stream, p);
}

template <class E, int DP, int BK, int KVSRC>
static hipError_t launch_fast(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = 4 * BK * DP * 2;
  auto kern = mfa_fwd_fast_kernel<E, DP, BK, KVSRC>;
  return launch(kern, dim3(p.nblk * p.B * p.H), dim3(256), LDS, stream, p);
}

// Returns hipErrorNotSupported when the configuration is not covered (caller falls back).
hipError_t fwd_fast_dispatch(const FwdParams& p, int elem, int DP, int kvsrc, hipStream_t stream) {
  // Variant choice: with causal skipping, query blocks carry 1..nblk tiles; when the grid is
  // about one round of workgroup slots (2 per CU) the heaviest block sets the makespan, so the
  // mirrored-pair kernel (equal work per workgroup) wins; with several rounds the single-block
  // kernel's heavy-first order balances on its own and its two independent workgroups per CU
  // overlap better.  MFA_FWD_VARIANT=single|pair overrides.
  const char* var = getenv("MFA_FWD_VARIANT");
  const int blocks = p.nblk * p.B * p.H;
  bool single = !(p.mask.causal && p.mask.skip_ok) || blocks > 768;
  if (var && var[0] == 's') single = true;
  if (var && var[0] == 'p') single = false;
#define MFA_FAST(ELEM, EE, DPV, BKV, KS)                                  \
  if (elem == ELEM && DP == DPV && kvsrc == KS)                           \
    return single ? launch_fast<EE, DPV, BKV, KS>(p, stream)              \
                  : launch_pair<EE, DPV, BKV, KS>(p, stream);
  MFA_FAST(P_FP16, F16, 64, 64, SRC_SAME)
  MFA_FAST(P_FP16, F16, 128, 64, SRC_SAME)
  MFA_FAST(P_BF16, BF16, 64, 64, SRC_SAME)
  MFA_FAST(P_BF16, BF16, 128, 64, SRC_SAME)
  MFA_FAST(P_FP16, F16, 128, 64, SRC_I8)
  MFA_FAST(P_BF16, BF16, 128, 64, SRC_I8)
#undef MFA_FAST
  return hipErrorNotSupported;
}

}  // namespace mfa
