/*
 * mfa_oracle.c — CPU ORACLE for the MI355X attention library.  TEST INFRASTRUCTURE ONLY:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker (never as the measured or shipped path).
 *
 * A plain-C restatement of the reference's own CPU references and host arithmetic
 * (bghira/metal-flash-attention-plus; paths relative to its repository root):
 *
 *   - attention forward / backward: Tests/FlashAttentionTests/Utilities/Network.swift:137-409
 *     (row-wise S, P, L, dP, dS, D; inferenceAttention, derivativeV/K/Q), generalised to the
 *     batched BHSD + causal form of KernelRegressionTests.swift:72-147 and the general-dO
 *     flash backward of QuantizedAttentionTest.swift:822-936; converted to the GPU output
 *     conventions L_gpu = log2(e)·L_nat (SquareAttentionTest.swift:424-426) and
 *     D_gpu = scale·D_nat (SquareAttentionTest.swift:427-429);
 *   - mask predicates exactly as the generated kernel applies them
 *     (AttentionKernel+Softmax.swift:243-474): masked elements take the finite value
 *     (0.875/log2e)·(-FLT_MAX), so a fully masked row is a uniform average (the reference's
 *     behaviour); the additive mask is added to QK^T before scaling (:306-336);
 *   - quantisation: GEMMQuantization.swift:305-676 (tensor-, row-, block-wise parameters,
 *     round-half-away-from-zero, Int8(clamping:), INT4 (q+8) nibbles, blockwise indexing);
 *   - deterministic data: KernelRegressionTests.swift:41-59 (LCG + bf16 RNE) and
 *     QuantizedAttentionTest.swift:446-450 (LCG, Int32 truncation);
 *   - GEMM: C = A·B (GEMMDescriptor.swift:11-47) for the MLA decompression
 *     (MLAOptimizedGEMMMFA.swift:97-154), accumulated in double.
 *
 * Accumulations use double (the Swift oracles use Float); this only tightens the reference.
 * Parity pinning: the reference (Swift + Metal) cannot be built or run on Linux, so this
 * restatement is pinned by the reference's known-answer tests (tests/test_oracle.py) and by
 * an independent numpy float64 restatement + the finite-difference check Network.swift:14-60
 * prescribes.  See DESIGN.md §Oracle.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define ORACLE_API __attribute__((visibility("default")))

static const float kMaskValue = -(0.875f / 1.442695041f) * 3.402823466e+38f;

/* ---------------------------------------------------------------- data generators */

/* KernelRegressionTests.deterministicData (KernelRegressionTests.swift:41-50). */
ORACLE_API void mfa_oracle_lcg_fill(uint64_t seed, uint64_t count, float scale, float* out) {
  uint64_t state = seed * 6364136223846793005ULL + 1442695040888963407ULL;
  for (uint64_t i = 0; i < count; ++i) {
    state = state * 6364136223846793005ULL + 1442695040888963407ULL;
    const float unit = (float)(state >> 40) / (float)(1 << 24);
    out[i] = (unit * 2.0f - 1.0f) * scale;
  }
}

/* QuantizedAttentionTest nextRandom (QuantizedAttentionTest.swift:446-450): x = r*mul + add
 * with r = Float(Int32(truncatingIfNeeded: seed)) / Float(Int32.max).  The state advances
 * across calls (the tests draw Q, K, V, dO from one stream). */
ORACLE_API void mfa_oracle_lcg_stream(uint64_t* state, uint64_t count, float mul, float add,
                                      float* out) {
  uint64_t s = *state;
  for (uint64_t i = 0; i < count; ++i) {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    const float r = (float)(int32_t)(uint32_t)s / (float)2147483647;
    out[i] = r * mul + add;
  }
  *state = s;
}

/* ---------------------------------------------------------------- 16-bit conversions */

ORACLE_API uint16_t mfa_oracle_f32_to_bf16_rne(float x) {
  /* KernelRegressionTests.bf16Bytes (KernelRegressionTests.swift:52-59). */
  uint32_t bits;
  memcpy(&bits, &x, 4);
  const uint32_t lsb = (bits >> 16) & 1u;
  bits = bits + 0x7FFFu + lsb;
  return (uint16_t)(bits >> 16);
}

ORACLE_API uint16_t mfa_oracle_f32_to_bf16_trunc(float x) {
  /* MTLContext+Buffers.swift:38-44 / QuantizedTensor.from BF16 copy
   * (GEMMQuantization.swift:830-836): upper 16 bits. */
  uint32_t bits;
  memcpy(&bits, &x, 4);
  return (uint16_t)(bits >> 16);
}

ORACLE_API float mfa_oracle_bf16_to_f32(uint16_t b) {
  const uint32_t bits = (uint32_t)b << 16;
  float x;
  memcpy(&x, &bits, 4);
  return x;
}

/* IEEE binary16 round-to-nearest-even (Swift Float16(x)). */
ORACLE_API uint16_t mfa_oracle_f32_to_f16(float x) {
  uint32_t f;
  memcpy(&f, &x, 4);
  const uint32_t sign = (f >> 16) & 0x8000u;
  const uint32_t absf = f & 0x7FFFFFFFu;
  if (absf >= 0x7F800000u) /* inf / nan */
    return (uint16_t)(sign | 0x7C00u | (absf > 0x7F800000u ? 0x200u : 0u));
  if (absf >= 0x477FF000u) return (uint16_t)(sign | 0x7C00u); /* rounds to >= 65520 -> inf */
  if (absf < 0x38800000u) {                                   /* subnormal half or zero */
    const int shift = 126 - (int)(absf >> 23);
    if (shift > 24) return (uint16_t)sign;
    uint32_t mant = (absf & 0x7FFFFFu) | 0x800000u;
    const uint32_t rem = mant & ((1u << shift) - 1u);
    const uint32_t half = 1u << (shift - 1);
    uint32_t h = mant >> shift;
    if (rem > half || (rem == half && (h & 1u))) h += 1;
    return (uint16_t)(sign | h);
  }
  uint32_t h = ((absf >> 13) - (112u << 10));
  const uint32_t rem = absf & 0x1FFFu;
  if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h += 1;
  return (uint16_t)(sign | h);
}

ORACLE_API float mfa_oracle_f16_to_f32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1Fu;
  const uint32_t m = h & 0x3FFu;
  float out;
  if (e == 0) {
    out = ldexpf((float)m, -24);
    if (sign) out = -out;
    return out;
  }
  uint32_t bits;
  if (e == 31)
    bits = sign | 0x7F800000u | (m << 13);
  else
    bits = sign | ((e + 112u) << 23) | (m << 13);
  memcpy(&out, &bits, 4);
  return out;
}

/* Round a float array through a 16-bit storage format: kind 1 = fp16 RNE, 2 = bf16 RNE,
 * 3 = bf16 truncation.  out may alias in. */
ORACLE_API void mfa_oracle_round16(const float* in, uint64_t n, int kind, float* out) {
  for (uint64_t i = 0; i < n; ++i) {
    if (kind == 1)
      out[i] = mfa_oracle_f16_to_f32(mfa_oracle_f32_to_f16(in[i]));
    else if (kind == 2)
      out[i] = mfa_oracle_bf16_to_f32(mfa_oracle_f32_to_bf16_rne(in[i]));
    else
      out[i] = mfa_oracle_bf16_to_f32(mfa_oracle_f32_to_bf16_trunc(in[i]));
  }
}

/* ---------------------------------------------------------------- attention */

typedef struct mfa_oracle_attention_args {
  int32_t B, H, Hkv, R, C, D;
  float scale;               /* softmax scale; <= 0 means 1/sqrt(D) */
  int32_t causal;            /* mask col > row */
  int32_t window;            /* mask row > col + window_size */
  uint32_t window_size;
  const float* amask;        /* additive [B, H, R, C] or NULL */
  const uint32_t* ranges;    /* uint32 pairs [B, Hkv, R] or NULL: mask col not in [x, y) */
  const float* Q;            /* [B, H, R, D] */
  const float* K;            /* [B, Hkv, C, D] */
  const float* V;            /* [B, Hkv, C, D] */
} mfa_oracle_attention_args;

static float resolve_scale(const mfa_oracle_attention_args* a) {
  return a->scale > 0.f ? a->scale : 1.0f / sqrtf((float)a->D);
}

/* Masked raw score row x_j (pre-scale), the GPU's S after masking. */
static void score_row(const mfa_oracle_attention_args* a, int b, int h, int r, double* x) {
  const int kvh = h % a->Hkv; /* AttentionKernel+Source.swift:80-86 */
  const float* q = a->Q + (((int64_t)b * a->H + h) * a->R + r) * a->D;
  const float* kb = a->K + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
  const float* am = a->amask ? a->amask + (((int64_t)b * a->H + h) * a->R + r) * a->C : NULL;
  uint32_t lo = 0, hi = 0;
  if (a->ranges) {
    const uint32_t* rp = a->ranges + 2 * (((int64_t)b * a->Hkv + kvh) * a->R + r);
    lo = rp[0];
    hi = rp[1];
  }
  /* Causal rows stop at colLimit = row + 1 (KernelRegressionTests.swift:92): the columns
   * past it are masked whatever their score, so their dot products are not computed. */
  const int climit = a->causal ? (r + 1 < a->C ? r + 1 : a->C) : a->C;
  for (int c = 0; c < a->C; ++c) {
    if (c >= climit) {
      x[c] = (double)kMaskValue;
      continue;
    }
    const float* k = kb + (int64_t)c * a->D;
    double dot = 0.0;
    for (int d = 0; d < a->D; ++d) dot += (double)q[d] * (double)k[d];
    if (am) dot += (double)am[c];
    int masked = 0;
    if (a->causal && c > r) masked = 1;
    if (a->window && (int64_t)r > (int64_t)c + (int64_t)a->window_size) masked = 1;
    if (a->ranges && ((uint32_t)c < lo || (uint32_t)c >= hi)) masked = 1;
    x[c] = masked ? (double)kMaskValue : dot;
  }
}

/* Softmax row in base 2: P_j = exp2(c·x_j - M), returns L = M + log2(Σ). */
static double softmax_row(int C, double c2, double* x) {
  double m = -INFINITY;
  for (int j = 0; j < C; ++j) m = fmax(m, c2 * x[j]);
  double sum = 0.0;
  for (int j = 0; j < C; ++j) {
    x[j] = exp2(c2 * x[j] - m);
    sum += x[j];
  }
  for (int j = 0; j < C; ++j) x[j] /= sum;
  return m + log2(sum);
}

/* inferenceAttention + createLTerm (Network.swift:137-290), batched.  O [B,H,R,D] fp32,
 * L [B,H,R] in the GPU convention (log2 units). */
ORACLE_API int mfa_oracle_attention_forward(const mfa_oracle_attention_args* a, float* O,
                                            float* L) {
  const double c2 = (double)(1.442695041f * resolve_scale(a));
  const int64_t rows = (int64_t)a->B * a->H * a->R;
#pragma omp parallel
  {
    double* x = (double*)malloc(sizeof(double) * (a->C > 0 ? a->C : 1));
    double* acc = (double*)malloc(sizeof(double) * (a->D > 0 ? a->D : 1));
#pragma omp for schedule(dynamic, 16)
    for (int64_t idx = 0; idx < rows; ++idx) {
      const int r = (int)(idx % a->R);
      const int h = (int)((idx / a->R) % a->H);
      const int b = (int)(idx / ((int64_t)a->R * a->H));
      const int kvh = h % a->Hkv;
      score_row(a, b, h, r, x);
      const double lse = softmax_row(a->C, c2, x);
      const float* vb = a->V + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
      for (int d = 0; d < a->D; ++d) acc[d] = 0.0;
      for (int c = 0; c < a->C; ++c) {
        const double p = x[c];
        if (p == 0.0) continue;
        const float* v = vb + (int64_t)c * a->D;
        for (int d = 0; d < a->D; ++d) acc[d] += p * (double)v[d];
      }
      float* o = O + idx * a->D;
      for (int d = 0; d < a->D; ++d) o[d] = (float)acc[d];
      if (L) L[idx] = (float)lse;
    }
    free(x);
    free(acc);
  }
  return 0;
}

/* derivativeV / derivativeK / derivativeQ + createDTerm (Network.swift:213-409) with a
 * general dO (QuantizedAttentionTest.swift:887-936).  Outputs: D [B,H,R] = scale·rowsum(dO∘O)
 * (GPU convention), dQ [B,H,R,D], dK/dV [B,Hkv,C,D] summed over every query head that maps
 * to the kv head (the reference's GQA backward does not reduce: SURVEY.md §8a quirk 2). */
ORACLE_API int mfa_oracle_attention_backward(const mfa_oracle_attention_args* a,
                                             const float* dO, float* Dout, float* dQ,
                                             float* dK, float* dV) {
  const float scale = resolve_scale(a);
  const double c2 = (double)(1.442695041f * scale);
  const int64_t kvsz = (int64_t)a->B * a->Hkv * a->C * a->D;
  memset(dK, 0, sizeof(float) * kvsz);
  memset(dV, 0, sizeof(float) * kvsz);
  double* dKacc = (double*)calloc(kvsz > 0 ? kvsz : 1, sizeof(double));
  double* dVacc = (double*)calloc(kvsz > 0 ? kvsz : 1, sizeof(double));
  const int64_t nslices = (int64_t)a->B * a->Hkv;
  /* Parallel over (b, kv head) so dK/dV accumulation is race free. */
#pragma omp parallel
  {
    double* x = (double*)malloc(sizeof(double) * (a->C > 0 ? a->C : 1));
    double* dp = (double*)malloc(sizeof(double) * (a->C > 0 ? a->C : 1));
    double* o = (double*)malloc(sizeof(double) * (a->D > 0 ? a->D : 1));
    double* dq = (double*)malloc(sizeof(double) * (a->D > 0 ? a->D : 1));
#pragma omp for schedule(dynamic, 1)
    for (int64_t sl = 0; sl < nslices; ++sl) {
      const int b = (int)(sl / a->Hkv);
      const int kvh = (int)(sl % a->Hkv);
      const float* kb = a->K + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
      const float* vb = a->V + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
      double* dkb = dKacc + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
      double* dvb = dVacc + (((int64_t)b * a->Hkv + kvh) * a->C) * a->D;
      for (int h = 0; h < a->H; ++h) {
        if (h % a->Hkv != kvh) continue;
        for (int r = 0; r < a->R; ++r) {
          const int64_t row = ((int64_t)b * a->H + h) * a->R + r;
          const float* q = a->Q + row * a->D;
          const float* go = dO + row * a->D;
          score_row(a, b, h, r, x);
          (void)softmax_row(a->C, c2, x);
          /* O row and D term (createDTerm). */
          for (int d = 0; d < a->D; ++d) o[d] = 0.0;
          for (int c = 0; c < a->C; ++c) {
            if (x[c] == 0.0) continue;
            const float* v = vb + (int64_t)c * a->D;
            for (int d = 0; d < a->D; ++d) o[d] += x[c] * (double)v[d];
          }
          double Dn = 0.0;
          for (int d = 0; d < a->D; ++d) Dn += (double)go[d] * o[d];
          if (Dout) Dout[row] = (float)((double)scale * Dn);
          /* dP = dO·V^T, dS = P∘(dP - D)·scale. */
          for (int c = 0; c < a->C; ++c) {
            const float* v = vb + (int64_t)c * a->D;
            double s = 0.0;
            for (int d = 0; d < a->D; ++d) s += (double)go[d] * (double)v[d];
            dp[c] = x[c] * (s - Dn) * (double)scale;
          }
          for (int d = 0; d < a->D; ++d) dq[d] = 0.0;
          for (int c = 0; c < a->C; ++c) {
            const double ds = dp[c];
            const double p = x[c];
            const float* k = kb + (int64_t)c * a->D;
            double* dkr = dkb + (int64_t)c * a->D;
            double* dvr = dvb + (int64_t)c * a->D;
            for (int d = 0; d < a->D; ++d) {
              dq[d] += ds * (double)k[d];
              dkr[d] += ds * (double)q[d];
              dvr[d] += p * (double)go[d];
            }
          }
          for (int d = 0; d < a->D; ++d) dQ[row * a->D + d] = (float)dq[d];
        }
      }
    }
    free(x);
    free(dp);
    free(o);
    free(dq);
  }
  for (int64_t i = 0; i < kvsz; ++i) {
    dK[i] = (float)dKacc[i];
    dV[i] = (float)dVacc[i];
  }
  free(dKacc);
  free(dVacc);
  return 0;
}

/* ---------------------------------------------------------------- quantisation */
/* Precision codes: 3 = INT8, 4 = INT4 (GEMMOperandPrecision raw values). */

static float absmax_range(const float* x, int64_t r0, int64_t r1, int64_t c0, int64_t c1,
                          int64_t cols, uint64_t count) {
  float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
  for (int64_t r = r0; r < r1; ++r)
    for (int64_t c = c0; c < c1; ++c) {
      const uint64_t idx = (uint64_t)(r * cols + c);
      if (idx < count) {
        mn = fminf(mn, x[idx]);
        mx = fmaxf(mx, x[idx]);
      }
    }
  return fmaxf(fabsf(mn), fabsf(mx));
}

/* calculateTensorWiseParameters (GEMMQuantization.swift:305-350): scale = absmax/127 (INT8)
 * or absmax/7 (INT4), zero point 0. */
ORACLE_API float mfa_oracle_quant_scale_tensor(const float* x, uint64_t count, int prec) {
  float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
  for (uint64_t i = 0; i < count; ++i) {
    mn = fminf(mn, x[i]);
    mx = fmaxf(mx, x[i]);
  }
  const float absmax = fmaxf(fabsf(mn), fabsf(mx));
  return prec == 3 ? absmax / 127.0f : absmax / 7.0f;
}

/* calculateBlockWiseParameters (:353-421): row-major block order over [rows, cols]. */
ORACLE_API void mfa_oracle_quant_scales_block(const float* x, uint64_t count, uint32_t rows,
                                              uint32_t cols, uint32_t bs, int prec,
                                              float* scales) {
  const uint32_t nbr = (rows + bs - 1) / bs, nbc = (cols + bs - 1) / bs;
  for (uint32_t br = 0; br < nbr; ++br)
    for (uint32_t bc = 0; bc < nbc; ++bc) {
      const int64_t r0 = (int64_t)br * bs, r1 = r0 + bs < rows ? r0 + bs : rows;
      const int64_t c0 = (int64_t)bc * bs, c1 = c0 + bs < cols ? c0 + bs : cols;
      const float am = absmax_range(x, r0, r1, c0, c1, cols, count);
      scales[br * nbc + bc] = prec == 3 ? am / 127.0f : am / 7.0f;
    }
}

/* calculateRowWiseParameters (:424-479). */
ORACLE_API void mfa_oracle_quant_scales_row(const float* x, uint64_t count, uint32_t rows,
                                            uint32_t cols, int prec, float* scales) {
  for (uint32_t r = 0; r < rows; ++r) {
    const float am = absmax_range(x, r, r + 1, 0, cols, cols, count);
    scales[r] = prec == 3 ? am / 127.0f : am / 7.0f;
  }
}

static int32_t swift_round_to_int(float v) {
  /* Int32(round(v)): Swift traps on NaN / out of range; clamp instead. */
  const float r = roundf(v);
  if (!(r == r)) return 0;
  if (r >= 2147483647.0f) return 2147483647;
  if (r <= -2147483648.0f) return (-2147483647 - 1);
  return (int32_t)r;
}

static int8_t clamp_i8(int64_t v) { return (int8_t)(v < -128 ? -128 : (v > 127 ? 127 : v)); }
static uint8_t nib(int64_t v) { return (uint8_t)(v < 0 ? 0 : (v > 15 ? 15 : v)); }

/* quantize (GEMMQuantization.swift:487-521). */
ORACLE_API void mfa_oracle_quantize(const float* x, uint64_t count, int prec, float scale,
                                    int32_t zp, uint8_t* out) {
  if (prec == 3) {
    for (uint64_t i = 0; i < count; ++i)
      ((int8_t*)out)[i] = clamp_i8((int64_t)swift_round_to_int(x[i] / scale) + zp);
  } else {
    for (uint64_t i = 0; i < count; i += 2) {
      const int64_t v1 = (int64_t)swift_round_to_int(x[i] / scale) + zp;
      const int64_t v2 = i + 1 < count ? (int64_t)swift_round_to_int(x[i + 1] / scale) + zp : 0;
      out[i / 2] = (uint8_t)((nib(v2 + 8) << 4) | nib(v1 + 8));
    }
  }
}

/* quantizeBlockwise (:567-623). */
ORACLE_API void mfa_oracle_quantize_block(const float* x, uint64_t count, uint32_t cols,
                                          uint32_t bs, int prec, const float* scales,
                                          const int32_t* zps, uint8_t* out) {
  const uint32_t nbc = (cols + bs - 1) / bs;
#define BI(i) ((uint32_t)(((i) / cols) / bs) * nbc + (uint32_t)(((i) % cols) / bs))
  if (prec == 3) {
    for (uint64_t i = 0; i < count; ++i) {
      const uint32_t b = BI(i);
      ((int8_t*)out)[i] =
          clamp_i8((int64_t)swift_round_to_int(x[i] / scales[b]) + (zps ? zps[b] : 0));
    }
  } else {
    for (uint64_t i = 0; i < count; i += 2) {
      const uint32_t b0 = BI(i);
      const int64_t v1 = (int64_t)swift_round_to_int(x[i] / scales[b0]) + (zps ? zps[b0] : 0);
      uint8_t byte = nib(v1 + 8);
      if (i + 1 < count) {
        const uint32_t b1 = BI(i + 1);
        const int64_t v2 =
            (int64_t)swift_round_to_int(x[i + 1] / scales[b1]) + (zps ? zps[b1] : 0);
        byte |= (uint8_t)(nib(v2 + 8) << 4);
      }
      out[i / 2] = byte;
    }
  }
#undef BI
}

/* dequantize (:529-558). */
ORACLE_API void mfa_oracle_dequantize(const uint8_t* in, uint64_t count, int prec, float scale,
                                      int32_t zp, float* out) {
  for (uint64_t i = 0; i < count; ++i) {
    int32_t q;
    if (prec == 3)
      q = ((const int8_t*)in)[i];
    else
      q = (int32_t)((i & 1) ? (in[i / 2] >> 4) : (in[i / 2] & 15)) - 8;
    out[i] = ((float)q - (float)zp) * scale;
  }
}

/* dequantizeBlockwise (:629-676). */
ORACLE_API void mfa_oracle_dequantize_block(const uint8_t* in, uint64_t count, uint32_t cols,
                                            uint32_t bs, int prec, const float* scales,
                                            const int32_t* zps, float* out) {
  const uint32_t nbc = (cols + bs - 1) / bs;
  for (uint64_t i = 0; i < count; ++i) {
    const uint32_t b = (uint32_t)((i / cols) / bs) * nbc + (uint32_t)((i % cols) / bs);
    int32_t q;
    if (prec == 3)
      q = ((const int8_t*)in)[i];
    else
      q = (int32_t)((i & 1) ? (in[i / 2] >> 4) : (in[i / 2] & 15)) - 8;
    out[i] = ((float)q - (float)(zps ? zps[b] : 0)) * scales[b];
  }
}

/* ---------------------------------------------------------------- GEMM */

/* C[M,N] = A[M,K]·B[K,N] (+ C), row-major, double accumulation. */
ORACLE_API void mfa_oracle_gemm(const float* A, const float* B, float* C, int M, int N, int K,
                                int load_previous_c) {
#pragma omp parallel for schedule(static)
  for (int i = 0; i < M; ++i) {
    double* acc = (double*)calloc((size_t)N, sizeof(double));
    for (int k = 0; k < K; ++k) {
      const double a = A[(int64_t)i * K + k];
      const float* b = B + (int64_t)k * N;
      for (int j = 0; j < N; ++j) acc[j] += a * (double)b[j];
    }
    for (int j = 0; j < N; ++j)
      C[(int64_t)i * N + j] = (float)(acc[j] + (load_previous_c ? C[(int64_t)i * N + j] : 0.0));
    free(acc);
  }
}

/* HadamardRotation.swift:111-136 (the MSL kernel hadamard_rotate), one block after another:
 * stage s pairs elements 2^s apart, (a, b) -> (a + b, a - b); then x *= scale, scale being
 * the FP32 1/sqrt(N) (see mfa_hadamard_scale in include/mfa/mfa.h). */
ORACLE_API void mfa_oracle_hadamard(float* data, int block_size, int64_t num_blocks, float scale) {
  int log2n = 0;
  while ((1 << log2n) < block_size) ++log2n;
  for (int64_t g = 0; g < num_blocks; ++g) {
    float* block = data + g * block_size;
    for (int s = 0; s < log2n; ++s) {
      const int stride = 1 << s, pair = stride * 2;
      for (int i = 0; i < block_size; i += pair)
        for (int j = 0; j < stride; ++j) {
          const float a = block[i + j], b = block[i + j + stride];
          block[i + j] = a + b;
          block[i + j + stride] = a - b;
        }
    }
    for (int i = 0; i < block_size; ++i) block[i] *= scale;
  }
}

/* ---------------------------------------------------------------- CPU baseline */

/* Threads the oracle may use (bench.py's cpu_baseline reports it as `cores`). */
ORACLE_API int mfa_oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}
