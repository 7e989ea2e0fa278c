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

__device__ __forceinline__ float cross_half_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float cross_half_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

template <class E, int DP, int BK, int KVSRC>
__global__ void __launch_bounds__(256, 2) mfa_fwd_fast_kernel(FwdParams p) {
  using A = Arith16<E, DP>;
  using T = Tile16<DP>;
  constexpr int NW = 4, NT = 256, BQ = 128;
  constexpr int NJ = BK / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int CPR = DP / 8;                 // 16-byte chunks per row
  constexpr int PER = BK * CPR / NT;          // chunks per thread per tile
  static_assert(PER >= 1 && BK * CPR % NT == 0, "tile/thread mismatch");
  constexpr float THR = 8.0f;                 // lazy-rescale threshold (log2 units)
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

  typename A::frag qf[A::DSTEPS];
  {
    const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb + (int64_t)h * p.q.sh +
                           (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
    for (int s = 0; s < A::DSTEPS; ++s) {
      const int d0 = 16 * s + 8 * hh;
      i16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
      qf[s] = v;
    }
  }

  int kend = p.C;
  if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
  int kbeg = 0;
  if (p.mask.window && p.mask.skip_ok) {
    const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
    kbeg = lo > 0 ? (int)(lo / BK) * BK : 0;
  }

  // Staging geometry: chunk id = tid + i*NT -> (row, chunk) of the tile; loop invariant.
  const int esz = KVSRC == SRC_SAME ? 2 : 1;  // bytes per stored element
  const int64_t kbase = (int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh;
  const int64_t vbase = (int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh;
  const char* kg = (const char*)p.k.ptr + kbase * esz;
  const char* vg = (const char*)p.v.ptr + vbase * esz;
  int srow[PER], soff[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int id = tid + i * NT;
    srow[i] = id / CPR;
    soff[i] = T::off(id / CPR, id % CPR);
  }
  uint4 rk[PER], rv[PER];
  auto load = [&](int t) {
    const bool full = t + BK <= p.C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = tid + i * NT;
      const int64_t row = t + srow[i];
      const int c = id % CPR;
      uint4 a = make_uint4(0u, 0u, 0u, 0u), v = a;
      if (full || row < p.C) {
        if constexpr (KVSRC == SRC_SAME) {
          if (c * 8 < p.D) {
            a = *reinterpret_cast<const uint4*>(kg + (row * p.k.ss + c * 8) * 2);
            v = *reinterpret_cast<const uint4*>(vg + (row * p.v.ss + c * 8) * 2);
          }
        } else {  // INT8: 8 bytes per chunk
          if (c * 8 < p.D) {
            const uint2 ka = *reinterpret_cast<const uint2*>(kg + row * p.k.ss + c * 8);
            const uint2 va = *reinterpret_cast<const uint2*>(vg + row * p.v.ss + c * 8);
            a.x = ka.x; a.y = ka.y; v.x = va.x; v.y = va.y;
          }
        }
      }
      rk[i] = a;
      rv[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      uint4 a = rk[i], v = rv[i];
      if constexpr (KVSRC != SRC_SAME) {
        a = dequant_fast<E, KVSRC>(a, (float)p.k.zp);
        v = dequant_fast<E, KVSRC>(v, (float)p.v.zp);
      }
      *reinterpret_cast<uint4*>(kb0 + buf * TILEB + soff[i]) = a;
      *reinterpret_cast<uint4*>(vb0 + buf * TILEB + soff[i]) = v;
    }
  };

  f32x16 o[DP / 32];
#pragma unroll
  for (int dt = 0; dt < DP / 32; ++dt) o[dt] = zero16();
  float m = -kFltMax, lh = 0.f;  // l per half-wave; l0 = FLT_MIN added at the end
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  if (kbeg < kend) {
    load(kbeg);
    store(0);
  }
  __syncthreads();

  int cur = 0;
  for (int t = kbeg; t < kend; t += BK) {
    const bool has_next = t + BK < kend;
    if (has_next) load(t + BK);
    const char* kt = kb0 + cur * TILEB;
    const char* vt = vb0 + cur * TILEB;

    f32x16 s[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) s[j] = zero16();
#pragma unroll
    for (int ds = 0; ds < A::DSTEPS; ++ds)
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        s[j] = A::mma(A::read_row(kt, j * 32 + l32, ds, hh), qf[ds], s[j]);

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
    float rs = 0.f;
    if (__any(m < kMaskLevel)) {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(mul_rn(s[j][i], c) - m);
          s[j][i] = pv;
          rs += pv;
        }
    } else {
#pragma unroll
      for (int j = 0; j < NJ; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(s[j][i] * c - m);
          s[j][i] = pv;
          rs += pv;
        }
    }
    lh += rs;

#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const i16x8 pb = A::pack(s[j], ks);
#pragma unroll
        for (int dt = 0; dt < DP / 32; ++dt)
          o[dt] = A::mma(A::read_tr(vt, j * 32, ks, dt * 32, lane), pb, o[dt]);
      }

    if (has_next) store(cur ^ 1);
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
  using A = Arith16<E, DP>;
  using T = Tile16<DP>;
  constexpr int NT = 256, BQ = 128;
  constexpr int NJ = BK / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int CPR = DP / 8;
  constexpr int PER = BK * CPR / NT;
  static_assert(PER >= 1 && BK * CPR % NT == 0, "tile/thread mismatch");
  constexpr float THR = 8.0f;
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = tid >> 8;             // group
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

  const int esz = KVSRC == SRC_SAME ? 2 : 1;
  const char* kg = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * esz;
  const char* vg = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * esz;
  int srow[PER], soff[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int id = gt + i * NT;
    srow[i] = id / CPR;
    soff[i] = T::off(id / CPR, id % CPR);
  }
  uint4 rk[PER], rv[PER];
  auto load = [&](int t) {
    const bool full = t + BK <= p.C;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int id = gt + i * NT;
      const int64_t row = t + srow[i];
      const int cc = id % CPR;
      uint4 a = make_uint4(0u, 0u, 0u, 0u), v = a;
      if ((full || row < p.C) && cc * 8 < p.D) {
        if constexpr (KVSRC == SRC_SAME) {
          a = *reinterpret_cast<const uint4*>(kg + (row * p.k.ss + cc * 8) * 2);
          v = *reinterpret_cast<const uint4*>(vg + (row * p.v.ss + cc * 8) * 2);
        } else {
          const uint2 ka = *reinterpret_cast<const uint2*>(kg + row * p.k.ss + cc * 8);
          const uint2 va = *reinterpret_cast<const uint2*>(vg + row * p.v.ss + cc * 8);
          a.x = ka.x; a.y = ka.y; v.x = va.x; v.y = va.y;
        }
      }
      rk[i] = a;
      rv[i] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      uint4 a = rk[i], v = rv[i];
      if constexpr (KVSRC != SRC_SAME) {
        a = dequant_fast<E, KVSRC>(a, (float)p.k.zp);
        v = dequant_fast<E, KVSRC>(v, (float)p.v.zp);
      }
      *reinterpret_cast<uint4*>(kb0 + buf * TILEB + soff[i]) = a;
      *reinterpret_cast<uint4*>(vb0 + buf * TILEB + soff[i]) = v;
    }
  };

  const int rbA = pi, rbB = p.nblk - 1 - pi;
  for (int which = 0; which < 2; ++which) {
    const int rb = which == 0 ? rbB : rbA;
    if (which == 1 && rbA >= rbB) break;  // odd middle block handled once
    const int q0 = rb * BQ;
    const int qi = q0 + wg * 32 + l32;
    const bool qvalid = qi < p.R;

    i16x8 qf[A::DSTEPS];
    {
      const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb +
                             (int64_t)h * p.q.sh + (int64_t)(qvalid ? qi : 0) * p.q.ss;
#pragma unroll
      for (int s = 0; s < A::DSTEPS; ++s) {
        const int d0 = 16 * s + 8 * hh;
        i16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (qvalid && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
        qf[s] = v;
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
      load(t0);
      store(0);
    }
    __syncthreads();
    int cur = 0;
    for (int step = 0; step < nA; ++step) {
      const int t = t0 + step * BK;
      if (t < t1) {
        const bool has_next = t + BK < t1;
        if (has_next) load(t + BK);
        const char* kt = kb0 + cur * TILEB;
        const char* vt = vb0 + cur * TILEB;
        f32x16 s[NJ];
#pragma unroll
        for (int j = 0; j < NJ; ++j) s[j] = zero16();
#pragma unroll
        for (int ds = 0; ds < A::DSTEPS; ++ds)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            s[j] = A::mma(A::read_row(kt, j * 32 + l32, ds, hh), qf[ds], s[j]);
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
        float rs = 0.f;
        if (__any(m < kMaskLevel)) {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float pv = __builtin_amdgcn_exp2f(mul_rn(s[j][i], c) - m);
              s[j][i] = pv;
              rs += pv;
            }
        } else {
#pragma unroll
          for (int j = 0; j < NJ; ++j)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const float pv = __builtin_amdgcn_exp2f(s[j][i] * c - m);
              s[j][i] = pv;
              rs += pv;
            }
        }
        lh += rs;
#pragma unroll
        for (int j = 0; j < NJ; ++j)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const i16x8 pb = A::pack(s[j], ks);
#pragma unroll
            for (int dt = 0; dt < DP / 32; ++dt)
              o[dt] = A::mma(A::read_tr(vt, j * 32, ks, dt * 32, lane), pb, o[dt]);
          }
        if (has_next) store(cur ^ 1);
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
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int npairs = (p.nblk + 1) / 2;
  hipLaunchKernelGGL(kern, dim3(npairs * p.B * p.H), dim3(512), LDS, stream, p);
  return hipGetLastError();
}

template <class E, int DP, int BK, int KVSRC>
static hipError_t launch_fast(const FwdParams& p, hipStream_t stream) {
  constexpr int LDS = 4 * BK * DP * 2;
  auto kern = mfa_fwd_fast_kernel<E, DP, BK, KVSRC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.nblk * p.B * p.H), dim3(256), LDS, stream, p);
  return hipGetLastError();
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
