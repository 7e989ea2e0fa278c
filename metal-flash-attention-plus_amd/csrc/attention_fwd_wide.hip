// attention_fwd_wide.hip — forward kernel with one wave per SIMD and two query blocks per
// wave, for fp16/bf16 operands with D <= 128 (the C2/C3 configurations).
//
// Same algorithm and numerics contract as attention_fwd_fast.hip (reference forward,
// AttentionKernel+Source.swift:372-416).  What changes is the shape of the work, following the
// CDNA4 guide's one-wave-per-SIMD attention structure (cdna_hip_programming.md, "4-wave,
// one-wave-per-SIMD"):
//   * a workgroup is 4 waves (one per SIMD, up to 512 registers each); each wave owns 64
//     query rows as two 32-row MFMA blocks A and B, so every K/V fragment read from LDS feeds
//     two MFMAs (half the LDS traffic per FLOP of the 32-row design) and block B's QK^T MFMAs
//     can issue while block A's softmax runs on the VALU;
//   * K/V tiles arrive by LDS-DMA (buffer_load ... lds, 1 KiB per wave-instruction) straight
//     into the XOR-swizzled layout: each lane fetches the global chunk that belongs at its
//     LDS slot, so no staging registers and no ds_write;
//   * waves {0,1} and {2,3} form two groups; a workgroup owns a 128-row block (or, for causal
//     skipping, the mirrored pair of blocks r and n-1-r, equal work for every workgroup); the
//     two groups split each block's key range and merge (m, l, O) through LDS.
#include "mfa_stage.h"
#include "mfa_dispatch.h"

namespace mfa {
namespace {

__device__ __forceinline__ float wx_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return fmaxf(__builtin_bit_cast(float, (unsigned)r[0]), __builtin_bit_cast(float, (unsigned)r[1]));
}
__device__ __forceinline__ float wx_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, x),
                                                  __builtin_bit_cast(unsigned, x), false, false);
  return __builtin_bit_cast(float, (unsigned)r[0]) + __builtin_bit_cast(float, (unsigned)r[1]);
}

constexpr int WDP = 128;                 // head-dimension padding
constexpr int WBK = 64;                  // keys per tile
constexpr int WTILE = WBK * WDP * 2;     // bytes per K (or V) tile
constexpr int WGROUP_LDS = 4 * WTILE;    // K, V double-buffered per group
constexpr int WLDS = 2 * WGROUP_LDS;     // 128 KiB

// LDS-DMA of one 64x128 16-bit tile by the 2 waves of a group: 16 wave-instructions of 1 KiB
// (4 rows each); wave wq issues rows 4n..4n+3 for n = wq + 2i.  Lane l lands at byte 16*l of
// the piece, i.e. row 4n + (l>>4), physical chunk l&15, so it fetches logical chunk
// (l&15) ^ swz(row) — the Tile16<128> swizzle, which depends on row&3 = (l>>4)&3 and
// (row>>2)&3 = n&3 only.
struct WideDMA {
  const char* base;  // head base (bytes)
  int step;          // bytes per key row
  int bytes;         // bytes in the head (range limit)
  int off[2];        // per-lane offset for n&3 == wq and n&3 == wq^2

  __device__ __forceinline__ void init(const char* b, int ss, int C, int D, int wq, int lane) {
    base = b;
    step = ss * 2;
    bytes = (int)(((int64_t)(C - 1) * ss + D) * 2);
    const int rl = lane >> 4, pc = lane & 15;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int n3 = (wq + 2 * v) & 3;
      const int ch = pc ^ (((rl & 3) << 2) | n3);
      off[v] = ch * 8 < D ? rl * step + ch * 16 : 0x40000000;
    }
  }
  // Issue the 8 pieces of this wave for the tile starting at key t into LDS tile `dst`.
  __device__ __forceinline__ void issue(int t, char* dst, int wq) const {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int n = wq + 2 * i;
      const int rb = (t + 4 * n) * step;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(base + rb), (short)0, max(bytes - rb, 0), 0x00020000);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rs, (__attribute__((address_space(3))) void*)(dst + n * 1024), 16, off[i & 1], 0, 0, 0);
    }
  }
};

__device__ __forceinline__ void wait_dma() {
  // vmcnt(0), expcnt/lgkmcnt untouched (gfx9 s_waitcnt encoding).
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

// One 64-key tile for the wave's two 32-row query blocks.
template <class E>
__device__ __forceinline__ void wide_tile(const char* kt, const char* vt,
                                          const i16x8 (&qf)[2][WDP / 16],
                                          f32x16 (&o)[2][WDP / 32], float (&m)[2],
                                          float (&lh)[2], int t, const int (&qb0)[2],
                                          const int (&qi)[2], const FwdParams& p, float c,
                                          int wsz, int lane) {
  using A = Arith16<E, WDP>;
  constexpr float THR = 8.0f;
  const int l32 = lane & 31, hh = lane >> 5;
  f32x16 s[2][2];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int j = 0; j < 2; ++j) s[x][j] = zero16();
#pragma unroll
  for (int ds = 0; ds < A::DSTEPS; ++ds)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const i16x8 kf = A::read_row(kt, j * 32 + l32, ds, hh);
#pragma unroll
      for (int x = 0; x < 2; ++x) s[x][j] = A::mma(kf, qf[x][ds], s[x][j]);
    }

  const bool edge = t + WBK > p.C;
  const bool diag = p.mask.causal && t + WBK - 1 > qb0[0];
  if (edge || diag || p.mask.window) {
    MFA_KEEP_BRANCH();
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = t + j * 32 + acc_row(i, hh);
          float v = s[x][j][i];
          if ((p.mask.causal && key > qi[x]) || (p.mask.window && qi[x] - key > wsz))
            v = kMaskValue;
          if (key >= p.C) v = -__builtin_inff();
          s[x][j][i] = v;
        }
  }

  float mt[2];
#pragma unroll
  for (int x = 0; x < 2; ++x) {
    float mx = s[x][0][0];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i) mx = fmaxf(mx, s[x][j][i]);
    mt[x] = wx_max(mx) * c;
  }
  if (__any(mt[0] > m[0] + THR || mt[1] > m[1] + THR)) {
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const float m_new = mt[x] > m[x] + THR ? fmaxf(m[x], mt[x]) : m[x];
      const float corr = __builtin_amdgcn_exp2f(m[x] - m_new);
      m[x] = m_new;
      lh[x] *= corr;
#pragma unroll
      for (int dt = 0; dt < WDP / 32; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[x][dt][i] *= corr;
    }
  }
  float rs[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  if (__any(m[0] < kMaskLevel || m[1] < kMaskLevel)) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = __builtin_amdgcn_exp2f(mul_rn(s[x][j][i], c) - m[x]);
          s[x][j][i] = pv;
          rs[x][i & 3] += pv;
        }
  } else {
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 16; ++i)
#pragma unroll
        for (int x = 0; x < 2; ++x) {
          const float pv = __builtin_amdgcn_exp2f(__builtin_fmaf(s[x][j][i], c, -m[x]));
          s[x][j][i] = pv;
          rs[x][i & 3] += pv;
        }
  }
#pragma unroll
  for (int x = 0; x < 2; ++x) lh[x] += (rs[x][0] + rs[x][1]) + (rs[x][2] + rs[x][3]);

#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const i16x8 pa = A::pack(s[0][j], ks);
      const i16x8 pb = A::pack(s[1][j], ks);
#pragma unroll
      for (int dt = 0; dt < WDP / 32; ++dt) {
        const i16x8 vf = A::read_tr(vt, j * 32, ks, dt * 32, lane);
        o[0][dt] = A::mma(vf, pa, o[0][dt]);
        o[1][dt] = A::mma(vf, pb, o[1][dt]);
      }
    }
}

template <class E, bool PAIR>
__global__ void __launch_bounds__(256, 1) mfa_fwd_wide_kernel(FwdParams p) {
  constexpr int BQ = 128;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = wave >> 1;   // group: half of each block's key range
  const int wq = wave & 1;   // 64-row half of the 128-row block
  const int l32 = lane & 31, hh = lane >> 5;
  char* const kb0 = smem + g * WGROUP_LDS;
  char* const vb0 = kb0 + 2 * WTILE;

  const int BH = p.B * p.H;
  const int bid = blockIdx.x;
  const int pi = bid / BH;
  const int bh = bid % BH;
  const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
  const float c = p.c_log2;
  const int wsz = p.mask.window_size > 0x3fffffffu ? 0x3fffffff : (int)p.mask.window_size;

  WideDMA kd, vd;
  kd.init((const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2,
          (int)p.k.ss, p.C, p.D, wq, lane);
  vd.init((const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2,
          (int)p.v.ss, p.C, p.D, wq, lane);

  const int nrounds = PAIR ? 2 : 1;
  for (int which = 0; which < nrounds; ++which) {
    const int rb = PAIR ? (which == 0 ? p.nblk - 1 - pi : pi) : p.nblk - 1 - pi;
    if (PAIR && which == 1 && pi >= p.nblk - 1 - pi) break;  // odd middle block once
    const int q0 = rb * BQ;
    int qb0[2], qi[2];
    bool qv[2];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      qb0[x] = q0 + 64 * wq + 32 * x;
      qi[x] = qb0[x] + l32;
      qv[x] = qi[x] < p.R;
    }

    i16x8 qf[2][WDP / 16];
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const uint16_t* qrow = (const uint16_t*)p.q.ptr + (int64_t)b * p.q.sb +
                             (int64_t)h * p.q.sh + (int64_t)(qv[x] ? qi[x] : 0) * p.q.ss;
#pragma unroll
      for (int s = 0; s < WDP / 16; ++s) {
        const int d0 = 16 * s + 8 * hh;
        i16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
        if (qv[x] && d0 < p.D) v = *reinterpret_cast<const i16x8*>(qrow + d0);
        qf[x][s] = v;
      }
    }

    int kend = p.C;
    if (p.mask.causal && p.mask.skip_ok) kend = min(kend, q0 + BQ);
    int kbeg = 0;
    if (p.mask.window && p.mask.skip_ok) {
      const int64_t lo = (int64_t)q0 - (int64_t)p.mask.window_size;
      kbeg = lo > 0 ? (int)(lo / WBK) * WBK : 0;
    }
    const int ntile = kend > kbeg ? (kend - kbeg + WBK - 1) / WBK : 0;
    const int nA = (ntile + 1) / 2;
    const int t0 = g == 0 ? kbeg : kbeg + nA * WBK;
    const int t1 = g == 0 ? min(kend, kbeg + nA * WBK) : kend;

    f32x16 o[2][WDP / 32];
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int dt = 0; dt < WDP / 32; ++dt) o[x][dt] = zero16();
    float m[2] = {-kFltMax, -kFltMax}, lh[2] = {0.f, 0.f};

    if (t0 < t1) {
      kd.issue(t0, kb0, wq);
      vd.issue(t0, vb0, wq);
    }
    wait_dma();
    __syncthreads();
    int cur = 0;
    for (int step = 0; step < nA; ++step) {
      const int t = t0 + step * WBK;
      if (t < t1) {
        if (t + WBK < t1) {
          kd.issue(t + WBK, kb0 + (cur ^ 1) * WTILE, wq);
          vd.issue(t + WBK, vb0 + (cur ^ 1) * WTILE, wq);
        }
        wide_tile<E>(kb0 + cur * WTILE, vb0 + cur * WTILE, qf, o, m, lh, t, qb0, qi, p, c,
                     wsz, lane);
      }
      wait_dma();
      __syncthreads();
      cur ^= 1;
    }

    // Merge group 1's partial state into group 0 through LDS (staging buffers are free).
    float* mrg = reinterpret_cast<float*>(smem);          // [2 waves][2 blocks][4][16][64]
    float* mml = mrg + 2 * 2 * (WDP / 32) * 16 * 64;       // [2 waves][2 blocks][2][64]
    if (g == 1) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
#pragma unroll
        for (int dt = 0; dt < WDP / 32; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i)
            mrg[(((wq * 2 + x) * (WDP / 32) + dt) * 16 + i) * 64 + lane] = o[x][dt][i];
        mml[((wq * 2 + x) * 2 + 0) * 64 + lane] = m[x];
        mml[((wq * 2 + x) * 2 + 1) * 64 + lane] = lh[x];
      }
    }
    __syncthreads();
    if (g == 0) {
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        const float mb = mml[((wq * 2 + x) * 2 + 0) * 64 + lane];
        const float lb = mml[((wq * 2 + x) * 2 + 1) * 64 + lane];
        const float mf = fmaxf(m[x], mb);
        const float ca = __builtin_amdgcn_exp2f(m[x] - mf);
        const float cb = __builtin_amdgcn_exp2f(mb - mf);
        float l = wx_sum(lh[x] * ca + lb * cb);
        if (!(l > 0.f)) l = kFltMin;
        if (qv[x]) {
          const float inv = p.o_mul / l;
          float* orow = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh + (int64_t)qi[x] * p.o_ss;
#pragma unroll
          for (int dt = 0; dt < WDP / 32; ++dt)
#pragma unroll
            for (int gg = 0; gg < 4; ++gg) {
              const int d = dt * 32 + 8 * gg + 4 * hh;
              float4 val;
              float* vp = &val.x;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const int i = 4 * gg + e;
                const float ob = mrg[(((wq * 2 + x) * (WDP / 32) + dt) * 16 + i) * 64 + lane];
                vp[e] = (o[x][dt][i] * ca + ob * cb) * inv;
              }
              if (d < p.D) *reinterpret_cast<float4*>(orow + d) = val;
            }
          if (hh == 0) {
            const float L = mf + __log2f(l);
            const int64_t li = (int64_t)(b * p.H + h) * p.R + qi[x];
            if (p.l_f16)
              reinterpret_cast<uint16_t*>(p.l)[li] = f32_to_f16(L);
            else
              reinterpret_cast<float*>(p.l)[li] = L;
          }
        }
      }
    }
    __syncthreads();
  }
}

template <class E, bool PAIR>
hipError_t launch_wide(const FwdParams& p, hipStream_t stream) {
  static_assert(WLDS >= 2 * 2 * (WDP / 32) * 16 * 64 * 4 + 2 * 2 * 2 * 64 * 4, "merge area");
  auto kern = mfa_fwd_wide_kernel<E, PAIR>;
  static bool attr_set = false;
  if (!attr_set) {
    hipError_t e = hipFuncSetAttribute((const void*)kern,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, WLDS);
    if (e != hipSuccess) return e;
    attr_set = true;
  }
  const int nb = PAIR ? (p.nblk + 1) / 2 : p.nblk;
  hipLaunchKernelGGL(kern, dim3(nb * p.B * p.H), dim3(256), WLDS, stream, p);
  return hipGetLastError();
}

}  // namespace

// fp16/bf16 Q/K/V with D <= 128 (16-byte aligned rows), no additive mask / sparse ranges.
hipError_t fwd_wide_dispatch(const FwdParams& p, int elem, hipStream_t stream) {
  const bool pair = p.mask.causal && p.mask.skip_ok;
  if (elem == P_FP16) return pair ? launch_wide<F16, true>(p, stream) : launch_wide<F16, false>(p, stream);
  if (elem == P_BF16) return pair ? launch_wide<BF16, true>(p, stream) : launch_wide<BF16, false>(p, stream);
  return hipErrorNotSupported;
}

}  // namespace mfa
