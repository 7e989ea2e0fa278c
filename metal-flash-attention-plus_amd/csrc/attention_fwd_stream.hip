// attention_fwd_stream.hip — causal 16-bit forward, key tiles dealt out in equal contiguous
// ranges ("stream" split) to one 512-thread workgroup per CU.
//
// Same algorithm and numerics as the shared-tile forward of attention_fwd_v2.hip (the
// reference forward, AttentionKernel+Source.swift:372-416; causal predicate
// AttentionKernel+Softmax.swift:243-304), same tile body (attention_fwd2.h).  What differs is
// who does which (query block, key tile) pair:
//
//   * a query block is 256 rows, held by the two 4-wave groups of the workgroup (128 rows
//     each), so EVERY staged K/V tile is read by 256 query rows.  The mirrored-pair kernel
//     shares a tile between its two blocks only while the light block still has keys; for the
//     rest (about half of C2's steps) one staged tile serves 128 rows and a step costs
//     ≈ 1.95 instead of ≈ 1.66 µs (DESIGN.md, round-3 stamps);
//   * the causal work of a (batch, head) is the list of its blocks' key tiles, ordered as
//     mirrored pairs (heavy block nb-1-i, then light block i) with an odd middle block last;
//     the lists of all heads are concatenated and cut into W equal ranges, one per workgroup
//     (W = the CU count).  At C2 (H16 S4096) every range is 34 tiles: the heavy block of a
//     pair is split between the pair's two workgroups, the light one is whole;
//   * a block cut between ranges leaves one partial softmax state (O, m, l) per range.  The
//     part that ends its range (the block's first part, "closer") merges at its end when
//     every other part has been published; the others ("publishers") write their state to a
//     workspace slot by write-through (sc1) stores and count themselves in on the block's
//     arrival counter after their stores have drained.  If the closer finds parts missing it
//     publishes too, and whichever part counts in last merges.  No workgroup ever waits for
//     another, so nothing depends on which workgroups are resident; the merge adds the parts
//     in part order, so the result does not depend on which part merges.
//   * hand-off (cdna_hip_programming.md Guideline 16; MI355X_MICROARCH.md § visibility, first
//     row of the sc1 table): every payload byte is stored sc1 and drained by each storing wave
//     (s_waitcnt vmcnt(0)), then a workgroup barrier, then one lane's agent-scope atomic add;
//     the merging workgroup reads the counter (add result or relaxed poll) on one lane, passes
//     the decision through LDS behind a barrier, and loads every part with sc1 loads.  The
//     last arriver resets the counter to 0, so the counters (zeroed once when the workspace
//     is allocated) are zero between launches.
#include "attention_fwd2.h"

namespace mfa {

namespace {

constexpr int kSBQ = 256;  // query rows per block (two 128-row groups)

typedef __attribute__((address_space(1))) unsigned gu32;

// Key tiles of 256-row block `blk` under the causal mask: keys [0, min(C, 256 (blk + 1))).
__host__ __device__ inline int stream_tiles(int blk, int C, int BK) {
  const int kend = C < (blk + 1) * kSBQ ? C : (blk + 1) * kSBQ;
  return (kend + BK - 1) / BK;
}

// Tile r of one (batch, head)'s work list -> (block, tile offset in it, the block's tiles).
// Order: pairs (nb-1-i heavy, then i light) for i = 0, 1, ..., then the middle block of an odd
// count.
__host__ __device__ inline void stream_locate(int r, int nb, int C, int BK, int* blk, int* toff,
                                              int* ntb) {
  for (int i = 0; i < nb; ++i) {
    const int J = nb - 1 - i, j = i;
    const int nh = stream_tiles(J, C, BK);
    if (r < nh || J <= j) {
      *blk = J;
      *toff = r;
      *ntb = nh;
      return;
    }
    r -= nh;
    const int nl = stream_tiles(j, C, BK);
    if (r < nl) {
      *blk = j;
      *toff = r;
      *ntb = nl;
      return;
    }
    r -= nl;
  }
  *blk = 0;
  *toff = 0;
  *ntb = 0;
}

__host__ __device__ inline int stream_head_tiles(int nb, int C, int BK) {
  int t = 0;
  for (int blk = 0; blk < nb; ++blk) t += stream_tiles(blk, C, BK);
  return t;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t part_rsrc(char* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
}

// 16 bytes, write-through to memory (sc1): visible to any XCD after the storing wave drains.
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t rs, int off, float a, float b, float c,
                                       float d) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = {__builtin_bit_cast(unsigned, a), __builtin_bit_cast(unsigned, b),
                   __builtin_bit_cast(unsigned, c), __builtin_bit_cast(unsigned, d)};
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);
}
// (The whole vector is bit-cast: hipcc 7.2 folds __builtin_bit_cast(float, a[i]) of an element
// of the returned vector to element 0 for every i.)
__device__ __forceinline__ float4 ld_sc1(__amdgpu_buffer_rsrc_t rs, int off) {
  const f32x4 a = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16));
  return make_float4(a[0], a[1], a[2], a[3]);
}

}  // namespace

// ---------------------------------------------------------------------------------------
template <class E, int DP, int BK>
__global__ void __launch_bounds__(512, 2) mfa_fwd2_stream_kernel(FwdParams p) {
  constexpr int NT = 256, ND = DP / 32;
  constexpr int TILEB = BK * DP * 2;
  constexpr int NCH = ND * 4 + 1;          // 16-byte chunks per thread in a partial slot
  constexpr int SLOTB = NCH * 512 * 16;    // one part: [chunk][thread] x 16 B
  constexpr int ORS = DP * 4 + 16;         // O row image: padded row (bytes)
  constexpr int OIMG = 128 * ORS;
  constexpr int IMG = 4 * TILEB;            // O row image, above the ring (see merge_store)
  constexpr int FLAG = IMG + OIMG;         // LDS decision word
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x;
  const int g = __builtin_amdgcn_readfirstlane(tid / NT);
  const int lane = tid & 63, wg = (tid % NT) >> 6;
  const int l32 = lane & 31, hh = lane >> 5;
  const int rbase[2] = {TileA<DP>::row_base(l32, hh, 0), TileA<DP>::row_base(l32, hh, 1)};
  const int trb[2] = {TileA<DP>::tr_base(lane, 0), TileA<DP>::tr_base(lane, 1)};
  char* const sk = smem;                   // K slots 0, 1
  char* const sv = smem + 2 * TILEB;       // V slots 0, 1
  int* const flag = reinterpret_cast<int*>(smem + FLAG);  // ordered by the barriers around it
  const float c = p.c_log2;
  const int wsz = 0x3fffffff;

  DmaA<DP, BK, 2 * NT> kd, vd;  // every tile is staged by all 8 waves
  kd.init((int)p.k.ss * 2, p.C, p.D * 2, tid);
  vd.init((int)p.v.ss * 2, p.C, p.D * 2, tid);

  // Virtual range index: the ranges of consecutive indices (the same heads) go to one XCD, so
  // a head's K/V stays in that XCD's L2 (workgroups are dealt round-robin over the 8 XCDs;
  // placement only changes speed).
  const int W = gridDim.x;
  const int v = (W & 7) == 0 ? (int)(blockIdx.x & 7) * (W >> 3) + (int)(blockIdx.x >> 3)
                             : (int)blockIdx.x;
  const int L = p.sk_len, T = p.sk_total, Th = p.sk_head, nb = p.nblk;
  const int g0 = v * L, g1 = min(g0 + L, T);
  gu32* const cnt = (gu32*)(p.ws);
  char* const parts = (char*)p.ws + p.sk_cnt_bytes;
  auto slot_rs = [&](int slot) { return part_rsrc(parts + (size_t)slot * SLOTB, SLOTB); };

  // A published part whose counter add is still to come (after its stores drained), and a
  // merge this workgroup owes at the end of its range because its add came last.
  int pend_x = -1;             // counter index
  unsigned pend_old = 0;       // lane 0: value its add returned
  int dm_bh = 0, dm_blk = 0, dm_vf = 0, dm_np = 0;
  bool dm_pending = false;

  // Merge the nparts parts of block (bh, blk) in part order (part 0 = the closer's, in slot
  // 2·vf + 1; part q >= 1 = range vf + q's, in slot 2·(vf + q)) and store O and L.  own = 0:
  // part 0 is the state in st (the closer); own = -1: every part comes from the workspace.
  // The sum runs over the parts in order either way (st.o is the accumulator), so the result
  // does not depend on which workgroup merges.
  auto merge_store = [&](RowState<DP>& st, int own, int bh, int blk, int vf, int nparts) {
    auto slot_of = [&](int q) { return q == 0 ? 2 * vf + 1 : 2 * (vf + q); };
    float M = own == 0 ? st.m : -kFltMax;
    for (int q = own == 0 ? 1 : 0; q < nparts; ++q)
      M = fmaxf(M, ld_sc1(slot_rs(slot_of(q)), ((NCH - 1) * 512 + tid) * 16).x);
    // Part 0 starts the sums as a product (the same instruction whether it comes from the
    // registers or the workspace), every later part is added by an fma.
    float la = 0.f;
    if (own == 0) {
      const float f = __builtin_amdgcn_exp2f(st.m - M);
#pragma unroll
      for (int dt = 0; dt < ND; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) st.o[dt][i] *= f;
      la = st.lh * f;
    }
    for (int q = own == 0 ? 1 : 0; q < nparts; ++q) {
      const __amdgpu_buffer_rsrc_t rs = slot_rs(slot_of(q));
      const float4 ml = ld_sc1(rs, ((NCH - 1) * 512 + tid) * 16);
      constexpr int HK = ND * 2;  // chunks per batch of loads (two batches: register budget)
#pragma unroll
      for (int hb = 0; hb < 2; ++hb) {
        float4 x[HK];
#pragma unroll
        for (int k = 0; k < HK; ++k) x[k] = ld_sc1(rs, ((hb * HK + k) * 512 + tid) * 16);
        const float f = __builtin_amdgcn_exp2f(ml.x - M);
        if (q == 0) {
#pragma unroll
          for (int kk = 0; kk < HK; ++kk) {
            const int k = hb * HK + kk, dt = k / 4, i0 = (k % 4) * 4;
            st.o[dt][i0] = x[kk].x * f;
            st.o[dt][i0 + 1] = x[kk].y * f;
            st.o[dt][i0 + 2] = x[kk].z * f;
            st.o[dt][i0 + 3] = x[kk].w * f;
          }
        } else {
#pragma unroll
          for (int kk = 0; kk < HK; ++kk) {
            const int k = hb * HK + kk, dt = k / 4, i0 = (k % 4) * 4;
            st.o[dt][i0] = __builtin_fmaf(x[kk].x, f, st.o[dt][i0]);
            st.o[dt][i0 + 1] = __builtin_fmaf(x[kk].y, f, st.o[dt][i0 + 1]);
            st.o[dt][i0 + 2] = __builtin_fmaf(x[kk].z, f, st.o[dt][i0 + 2]);
            st.o[dt][i0 + 3] = __builtin_fmaf(x[kk].w, f, st.o[dt][i0 + 3]);
          }
        }
      }
      const float fl = __builtin_amdgcn_exp2f(ml.x - M);
      la = q == 0 ? ml.y * fl : __builtin_fmaf(ml.y, fl, la);
    }
    float l = cross_half_sum(la) + kFltMin;
    if (!(l > 0.f)) l = kFltMin;
    const int b = bh / p.H, h = bh % p.H;
    const int qi = blk * kSBQ + g * 128 + wg * 32 + l32;
    // Both groups' rows leave through O row images as whole rows from all 8 waves.
    const float inv = p.o_mul / l;
    if (hh == 0 && qi < p.R) store_l(p, M + __log2f(l), b, h, qi);
    // Each group's rows leave through one O row image above the ring (so the next segment's
    // first tile, staged during this segment's last step, stays intact), as whole rows from
    // all 8 waves: group 0's, then group 1's.
    float* obase = p.o + (int64_t)b * p.o_sb + (int64_t)h * p.o_sh;
    char* const img = smem + IMG;
#pragma unroll
    for (int gg = 0; gg < 2; ++gg) {
      if (g == gg) {
        char* orow = img + (wg * 32 + l32) * ORS;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
          for (int gq = 0; gq < 4; ++gq)
            *reinterpret_cast<float4*>(orow + (dt * 32 + 8 * gq + 4 * hh) * 4) =
                make_float4(st.o[dt][4 * gq] * inv, st.o[dt][4 * gq + 1] * inv,
                            st.o[dt][4 * gq + 2] * inv, st.o[dt][4 * gq + 3] * inv);
      }
      __syncthreads();
      const int qb = blk * kSBQ + gg * 128;
      store_o_image<DP, 128, 2 * NT, true>(p, obase, img, ORS, qb, tid,
                                           qb + 128 <= p.R && p.D == DP);
      __syncthreads();
    }
  };

  // One counter add for this workgroup's drained stores (lane 0; the caller ran wait_vm() and
  // a barrier after the stores).
  auto count_in = [&](int x) -> unsigned {
    return __hip_atomic_fetch_add(cnt + x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };

  MFA_STAMP(0);
  MFA_CYC(0);
  // One iteration per segment of the range, plus one at the end when a published part's
  // counter add (made during a later segment) came last and its merge is still owed.  One
  // merge / store site and one publish site keep the register budget of the tile loop.
  int seg = 0;
  // The next segment's first K/V tile (ring slot `slot`) and Q fragments (qn) are issued
  // during the last step of the segment before it, so a segment seam costs no load latency.
  bool pref = false;
  int slot = 0;
  i16x8 qn[DP / 16];
  for (int gpos = g0;; ++seg) {
    const bool tiles = gpos < g1;
    if (!tiles && !dm_pending) break;
    RowState<DP> st;
    st.init();
    int m_bh, m_blk, m_vf = 0, m_np = 1, own = 0;  // the block to store / merge
    bool store = true;
    if (tiles) {
      const int bh = gpos / Th;
      int blk, toff, ntb;
      stream_locate(gpos - bh * Th, nb, p.C, BK, &blk, &toff, &ntb);
      const int t_lo = toff, t_hi = min(ntb, toff + (g1 - gpos));
      const int gs = gpos - toff;  // global start of the block's list
      gpos += t_hi - t_lo;

      const int b = bh / p.H, h = bh % p.H, kvh = h % p.Hkv;
      const int q0w = blk * kSBQ + g * 128 + wg * 32;  // this wave's first row
      const int qi = q0w + l32;
      const char* khead = (const char*)p.k.ptr + ((int64_t)b * p.k.sb + (int64_t)kvh * p.k.sh) * 2;
      const char* vhead = (const char*)p.v.ptr + ((int64_t)b * p.v.sb + (int64_t)kvh * p.v.sh) * 2;
      i16x8 qf[DP / 16];
      if (pref) {
#pragma unroll
        for (int i = 0; i < DP / 16; ++i) qf[i] = qn[i];
      } else {
        kd.issue(khead, t_lo * BK, sk + slot * TILEB);
        vd.issue(vhead, t_lo * BK, sv + slot * TILEB);
        load_q2_raw<DP>(qf, p, b, h, qi, qi < p.R, hh);
        wait_vm();
      }
      prescale_q2<E, DP>(qf, c);
      __syncthreads();
      if (seg < 2) MFA_STAMP(1 + 3 * seg);
      // The segment after this one (same range), if any.
      pref = gpos < g1;
      int nbh = 0, nblk = 0, ntoff = 0, nntb = 0;
      if (pref) {
        nbh = gpos / Th;
        stream_locate(gpos - nbh * Th, nb, p.C, BK, &nblk, &ntoff, &nntb);
      }
      const bool live = q0w < p.R;
      auto step = [&](int s, auto last_c) {
        constexpr bool LAST = decltype(last_c)::value;
        const int cur = slot ^ ((s - t_lo) & 1);
        if (!LAST) {
          kd.issue(khead, (s + 1) * BK, sk + (cur ^ 1) * TILEB);
          vd.issue(vhead, (s + 1) * BK, sv + (cur ^ 1) * TILEB);
        } else if (pref) {
          const int nb_ = nbh / p.H, nh_ = nbh % p.H, nkvh = nh_ % p.Hkv;
          const char* nk = (const char*)p.k.ptr + ((int64_t)nb_ * p.k.sb + (int64_t)nkvh * p.k.sh) * 2;
          const char* nv = (const char*)p.v.ptr + ((int64_t)nb_ * p.v.sb + (int64_t)nkvh * p.v.sh) * 2;
          kd.issue(nk, ntoff * BK, sk + (cur ^ 1) * TILEB);
          vd.issue(nv, ntoff * BK, sv + (cur ^ 1) * TILEB);
          const int nqi = nblk * kSBQ + g * 128 + wg * 32 + l32;
          load_q2_raw<DP>(qn, p, nb_, nh_, nqi, nqi < p.R, hh);
        }
        const int tc = s * BK;
        // Tiles wholly above the wave's rows (causal) are skipped; masks on the diagonal ones.
        if (live && tc <= q0w + 31) {
          const bool mask_tile = (tc + BK > p.C) || (tc + BK - 1 > q0w);
          fwd2_tile<E, DP, BK>(sk + cur * TILEB, sv + cur * TILEB, rbase, trb, qf, st, tc,
                               mask_tile, qi, p, c, wsz, hh);
        }
        wait_vm();
        __syncthreads();
        if (pend_x >= 0) {
          // The published part's stores are drained in every wave: count it in.
          if (tid == 0) pend_old = count_in(pend_x);
          pend_x = -1;
        }
      };
      for (int s = t_lo; s < t_hi - 1; ++s) step(s, std::false_type());
      step(t_hi - 1, std::true_type());
      slot ^= (t_hi - t_lo) & 1;  // the ring slot after this segment's last
      if (seg < 2) MFA_STAMP(2 + 3 * seg);
      m_bh = bh;
      m_blk = blk;
      if (t_lo != 0 || t_hi != ntb) {
        // A part of a cut block: the closer (t_lo == 0, the block's first part) merges now if
        // every other part is published; otherwise the part is published.
        const int X = bh * nb + blk;
        m_vf = gs / L;
        m_np = (gs + ntb - 1) / L - m_vf + 1;
        const bool closer = t_lo == 0;
        bool publish = true;
        if (closer) {
          if (tid == 0) {
            const unsigned n = __hip_atomic_load(cnt + X, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const bool all_in = n == (unsigned)(m_np - 1) && !(p.sk_flags & 1);
            if (all_in) __hip_atomic_store(cnt + X, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            *flag = all_in;
          }
          __syncthreads();
          publish = *flag == 0;
          __syncthreads();
        }
        own = closer ? 0 : -1;  // a publisher's merge re-reads its own (drained) part
        if (publish) {
          const __amdgpu_buffer_rsrc_t rs = slot_rs(closer ? 2 * v + 1 : 2 * v);
#pragma unroll
          for (int k = 0; k < ND * 4; ++k)
            st_sc1(rs, (k * 512 + tid) * 16, st.o[k / 4][(k % 4) * 4], st.o[k / 4][(k % 4) * 4 + 1],
                   st.o[k / 4][(k % 4) * 4 + 2], st.o[k / 4][(k % 4) * 4 + 3]);
          st_sc1(rs, ((NCH - 1) * 512 + tid) * 16, st.m, st.lh, 0.f, 0.f);
          if (!closer && gpos < g1) {
            // More work follows: count in after the next segment's first step has drained
            // the stores (every step ends with wait_vm() + a barrier); merge at the end if
            // that add comes last.
            pend_x = X;
            dm_pending = true;
            dm_bh = bh;
            dm_blk = blk;
            dm_vf = m_vf;
            dm_np = m_np;
            store = false;
          } else {
            wait_vm();
            __syncthreads();
            if (tid == 0) {
              const bool last = count_in(X) == (unsigned)(m_np - 1);
              if (last) __hip_atomic_store(cnt + X, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              *flag = last;
            }
            __syncthreads();
            store = *flag != 0;
            __syncthreads();
          }
        }
      }
    } else {
      // The owed decision for the part published earlier in this range.
      if (pend_x >= 0) {  // no step followed it
        wait_vm();
        __syncthreads();
        if (tid == 0) pend_old = count_in(pend_x);
        pend_x = -1;
      }
      if (tid == 0) {
        const bool last = pend_old == (unsigned)(dm_np - 1);
        if (last)
          __hip_atomic_store(cnt + dm_bh * nb + dm_blk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
      }
      __syncthreads();
      store = *flag != 0;
      __syncthreads();
      dm_pending = false;
      m_bh = dm_bh;
      m_blk = dm_blk;
      m_vf = dm_vf;
      m_np = dm_np;
      own = -1;
    }
    if (store) merge_store(st, own, m_bh, m_blk, m_vf, m_np);
    if (seg < 2) MFA_STAMP(3 + 3 * seg);
  }
  MFA_CYC(1);
  MFA_STAMP_DRAIN();
  MFA_STAMP(7);
}

// ---------------------------------------------------------------------------------------
// Host side.

static int stream_grid() {
  static int w = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    return n;
  }();
  if (const char* e = mfa::dev_env("MFA_FWD_STREAM_WGS")) {
    const int n = atoi(e);
    if (n > 0) return n;
  }
  return w;
}

// The split for p: W ranges of L tiles over T tiles (Th per head), 0 when p does not take the
// stream kernel.
static bool stream_split(const FwdParams& p, int elem, int DP, int* W, int* L, int* T, int* Th,
                         int* nb) {
  const char* e = mfa::dev_env("MFA_FWD_STREAM");
  if (e && e[0] == '0') return false;
  const bool force = e && e[0] == '1';
  // The other causal kernels' A/B switches keep those kernels.
  if (!force && (mfa::dev_env("MFA_FWD_VARIANT") || mfa::dev_env("MFA_FWD_PAIR"))) return false;
  if (!p.mask.causal || p.mask.window || p.mask.ranges || p.mask.amask) return false;
  if ((elem != P_FP16 && elem != P_BF16) || (DP != 64 && DP != 128)) return false;
  constexpr int BK = 64;
  *nb = (p.R + kSBQ - 1) / kSBQ;
  *Th = stream_head_tiles(*nb, p.C, BK);
  const int64_t t = (int64_t)p.B * p.H * *Th;
  if (t <= 0 || t >= ((int64_t)1 << 30)) return false;
  *T = (int)t;
  *W = stream_grid();
  if (!force) {
    if (*T < 8 * *W) return false;  // too little work per range
    // Where the mirrored shared-tile pair kernel runs (at most ~1.5 rounds of 128-row blocks,
    // or 3 rounds of long rows; attention_fwd_v2.hip fwd2_dispatch) it is faster: C2 (H16
    // S4096) 929 vs 895 TF, H16 S8192 1066 vs 1062 (one-process A/B).  Past that, the stream
    // split beats the heaviest-first single-block kernel: B4 H16 S4096 964 vs 927, H32 S8192
    // 1058 vs 1024, B8 H16 S2048 829 vs 769 TF.
    const int64_t nblk128 = (p.R + 127) / 128, blocks = nblk128 * p.B * p.H;
    const bool pair_kernel = DP <= 128 && (blocks <= 768 || (nblk128 >= 64 && blocks <= 1536));
    if (pair_kernel) return false;
  }
  if (*W > *T) *W = *T;
  *L = (*T + *W - 1) / *W;
  *W = (*T + *L - 1) / *L;
  return true;
}

size_t fwd_stream_workspace_bytes(const FwdParams& p, int elem, int DP, size_t* zero_bytes) {
  int W, L, T, Th, nb;
  *zero_bytes = 0;
  if (!stream_split(p, elem, DP, &W, &L, &T, &Th, &nb)) return 0;
  const size_t cnt = ((size_t)p.B * p.H * nb * 4 + 255) / 256 * 256;
  const size_t slot = (size_t)((DP / 32) * 4 + 1) * 512 * 16;
  *zero_bytes = cnt;
  return cnt + 2 * (size_t)W * slot;
}

hipError_t fwd_stream_dispatch(const FwdParams& p0, int elem, int DP, hipStream_t stream) {
  int W, L, T, Th, nb;
  if (!p0.ws || !stream_split(p0, elem, DP, &W, &L, &T, &Th, &nb)) return hipErrorNotSupported;
  FwdParams p = p0;
  p.nblk = nb;
  p.sk_len = L;
  p.sk_total = T;
  p.sk_head = Th;
  p.sk_cnt_bytes = (int)(((size_t)p.B * p.H * nb * 4 + 255) / 256 * 256);
  // Tests: MFA_FWD_STREAM_SLOW=1 makes every closer publish and count in (the merge then
  // runs from the workspace in whichever workgroup counts in last).
  const char* sl = mfa::dev_env("MFA_FWD_STREAM_SLOW");
  p.sk_flags = sl && sl[0] == '1' ? 1 : 0;
  auto lds = [](int dp) { return 4 * 64 * dp * 2 + 128 * (dp * 4 + 16) + 16; };  // ring, image, flag
#define MFA_FS(ELEM, EE, DPV)                                                              \
  if (elem == ELEM && DP == DPV)                                                           \
    return launch(mfa_fwd2_stream_kernel<EE, DPV, 64>, dim3(W), dim3(512), lds(DPV), stream, p);
  MFA_FS(P_FP16, F16, 64)
  MFA_FS(P_FP16, F16, 128)
  MFA_FS(P_BF16, BF16, 64)
  MFA_FS(P_BF16, BF16, 128)
#undef MFA_FS
  return hipErrorNotSupported;
}

template __global__ void mfa_fwd2_stream_kernel<F16, 64, 64>(FwdParams);
template __global__ void mfa_fwd2_stream_kernel<F16, 128, 64>(FwdParams);
template __global__ void mfa_fwd2_stream_kernel<BF16, 64, 64>(FwdParams);
template __global__ void mfa_fwd2_stream_kernel<BF16, 128, 64>(FwdParams);

}  // namespace mfa
