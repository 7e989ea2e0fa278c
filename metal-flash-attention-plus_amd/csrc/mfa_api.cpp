// mfa_api.cpp — host layer behind include/mfa/mfa.h.
//
// This replaces the reference's Swift host code: descriptor -> kernel plan
// (AttentionDescriptor.kernelDescriptor, AttentionKernel.init), buffer-slot binding and grid
// sizing (MultiHeadAttention.dispatchBatched / backward, QuantizedAttention.forward /
// backwardQuery / backwardKeyValue, MLAOptimizedGEMMMFA.forward).  Instead of generating and
// JIT-compiling Metal source per shape, every configuration maps onto one of a fixed set of
// precompiled gfx950 kernel instantiations (see mfa_dispatch.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>

#include "../../include/mfa/mfa.h"
#include "mfa_dispatch.h"
#include "mfa_launch.h"
#include "mfa_params.h"

namespace {

thread_local std::string g_last_error;

mfa_status_t fail(mfa_status_t code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  if (getenv("MFA_DEBUG")) fprintf(stderr, "[mfa] %s\n", buf);
  return code;
}

mfa_status_t hip_status(hipError_t e, const char* what) {
  if (e == hipSuccess) return MFA_SUCCESS;
  return fail(MFA_ERR_LAUNCH, "%s: %s", what, hipGetErrorString(e));
}

// Queries over an empty key sequence have no softmax (every row would divide by zero); the
// reference rejects non-positive sequence lengths when it builds a descriptor
// (QuantizedAttention.swift:791).  An empty query sequence is a no-op instead.
mfa_status_t check_keys(int R, int C) {
  if (R > 0 && C <= 0)
    return fail(MFA_ERR_INVALID_DESCRIPTOR,
                "key sequence length %d with %d queries: softmax over no keys", C, R);
  return MFA_SUCCESS;
}

// Backward over an empty query sequence: dK = dV = 0 (sums over no queries), written with two
// memsets and no kernel; a plan query records nothing.
mfa_status_t zero_kv_grads(float* dk, float* dv, size_t elems, hipStream_t stream) {
  if (elems == 0 || mfa::plan_capture()) return MFA_SUCCESS;
  if (hipMemsetAsync(dk, 0, elems * sizeof(float), stream) != hipSuccess ||
      hipMemsetAsync(dv, 0, elems * sizeof(float), stream) != hipSuccess)
    return fail(MFA_ERR_LAUNCH, "zeroing dK / dV for an empty query sequence");
  return MFA_SUCCESS;
}

int precision_size(int p) {
  switch (p) {
    case MFA_PRECISION_FP32: return 4;
    case MFA_PRECISION_FP16:
    case MFA_PRECISION_BF16: return 2;
    default: return 1;
  }
}

bool is_quantized(int p) { return p == MFA_PRECISION_INT8 || p == MFA_PRECISION_INT4; }

// Padded head dimension of the register-resident kernels, or 0 above 256: the D-blocked
// kernels (attention_bigd.hip) take any larger D, as the reference's last parameter-table row
// does (AttentionDescriptor+Parameters.swift:44-69).
int pad_head(int D) {
  if (D <= 32) return 32;
  if (D <= 64) return 64;
  if (D <= 128) return 128;
  if (D <= 256) return 256;
  return 0;
}
constexpr int kBigD = 0;

// Library-owned scratch for buffers the caller does not pass (L in forward:
// MultiHeadAttention.swift:296-319 allocates one per call; MLA's decompressed K/V, Q~/O~ and
// split-KV partials).  One buffer per (device, stream, use): calls on different streams never
// share one.  Growth is stream-ordered (hipFreeAsync + hipMallocAsync on the call's stream),
// so the old buffer is released only after the work queued before it on that stream.
struct ScratchKey {
  int dev;
  hipStream_t stream;
  int slot;
  bool operator<(const ScratchKey& o) const {
    if (dev != o.dev) return dev < o.dev;
    if (stream != o.stream) return (uintptr_t)stream < (uintptr_t)o.stream;
    return slot < o.slot;
  }
};
struct ScratchBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  size_t zeroed = 0;  // leading bytes known to be zero (arrival counters every launch resets)
};
struct Scratch {
  std::mutex mu;
  std::map<ScratchKey, ScratchBuf> bufs;
} g_scratch;

// zero_bytes: the first bytes of the buffer must be zero when the call's kernel starts, e.g.
// arrival counters that every launch leaves at zero.  The zeroed prefix is tracked per buffer:
// a call whose counter region is longer than the previous call's (a different shape in the
// same buffer) zeroes it again, since the bytes past the old prefix hold partial states.
mfa_status_t scratch(size_t bytes, void** out, int slot, hipStream_t stream, size_t zero_bytes = 0) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fail(MFA_ERR_NO_DEVICE, "no HIP device");
  std::lock_guard<std::mutex> lock(g_scratch.mu);
  auto& b = g_scratch.bufs[ScratchKey{dev, stream, slot}];
  if (b.bytes < bytes) {
    if (b.ptr) (void)hipFreeAsync(b.ptr, stream);
    b = ScratchBuf();
    void* p = nullptr;
    hipError_t e = hipMallocAsync(&p, bytes, stream);
    if (e != hipSuccess) return hip_status(e, "hipMallocAsync(scratch)");
    b.ptr = p;
    b.bytes = bytes;
  }
  // Under stream capture the memset is only recorded into the graph, not run: a captured call
  // always records its own memset (the graph may replay after eager calls that left partial
  // states in its counter region), and afterwards no prefix is known to be zero, so the next
  // eager call on this stream zeroes again.
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  const bool capturing =
      hipStreamIsCapturing(stream, &cs) == hipSuccess && cs == hipStreamCaptureStatusActive;
  if (zero_bytes > b.zeroed || (capturing && zero_bytes > 0)) {
    const hipError_t e = hipMemsetAsync(b.ptr, 0, zero_bytes, stream);
    if (e != hipSuccess) return hip_status(e, "hipMemsetAsync(scratch)");
  }
  // After this call's launch only its own counter prefix is known to be zero again: the bytes
  // behind it hold this call's partial states.
  b.zeroed = capturing ? 0 : zero_bytes;
  *out = b.ptr;
  return MFA_SUCCESS;
}

// ---------------------------------------------------------------------------------------
// Precision policy (AttentionDescriptor+Precisions.swift:12-242), gfx950 register column.
struct Precisions {
  int mem[MFA_OPERAND_COUNT];
  int reg[MFA_OPERAND_COUNT];
};

Precisions resolve_precisions(const mfa_attention_descriptor_t& d) {
  Precisions p;
  for (int i = 0; i < MFA_OPERAND_COUNT; ++i) p.mem[i] = p.reg[i] = -1;
  const int input = d.input_memory_precision == MFA_PRECISION_UNSET ? MFA_PRECISION_FP16
                                                                     : d.input_memory_precision;
  const int in_mem = d.low_precision_inputs ? input : MFA_PRECISION_FP32;
  p.mem[MFA_OPERAND_Q] = p.mem[MFA_OPERAND_K] = p.mem[MFA_OPERAND_V] = in_mem;
  p.mem[MFA_OPERAND_dO] = in_mem;
  p.mem[MFA_OPERAND_L] = d.low_precision_intermediates ? MFA_PRECISION_FP16 : MFA_PRECISION_FP32;
  p.mem[MFA_OPERAND_D] = d.low_precision_intermediates ? MFA_PRECISION_BF16 : MFA_PRECISION_FP32;
  p.mem[MFA_OPERAND_O] = p.mem[MFA_OPERAND_dV] = p.mem[MFA_OPERAND_dK] = p.mem[MFA_OPERAND_dQ] =
      MFA_PRECISION_FP32;
  // Registers as the gfx950 kernels hold them: MFMA operands in the input type, every
  // accumulator (S, dP, O, dV, dK, dQ) FP32, P and dS rounded to the MFMA operand type.
  const int in_reg = in_mem;
  p.reg[MFA_OPERAND_Q] = p.reg[MFA_OPERAND_K] = p.reg[MFA_OPERAND_V] = in_reg;
  p.reg[MFA_OPERAND_dO] = in_reg;
  p.reg[MFA_OPERAND_L] = p.reg[MFA_OPERAND_D] = MFA_PRECISION_FP32;
  p.reg[MFA_OPERAND_S] = p.reg[MFA_OPERAND_dP] = MFA_PRECISION_FP32;
  p.reg[MFA_OPERAND_P] = p.reg[MFA_OPERAND_dS] = in_reg;
  p.reg[MFA_OPERAND_O] = p.reg[MFA_OPERAND_dV] = p.reg[MFA_OPERAND_dK] =
      p.reg[MFA_OPERAND_dQ] = MFA_PRECISION_FP32;
  return p;
}

int elem_of(int prec) {
  switch (prec) {
    case MFA_PRECISION_FP32: return 0;
    case MFA_PRECISION_FP16: return 1;
    case MFA_PRECISION_BF16: return 2;
    default: return -1;
  }
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Stand-in device address for buffers a plan query does not have (never dereferenced: launches
// are recorded, not issued).  256-byte aligned like any hipMalloc result.
constexpr uintptr_t kPlanDummy = 0x100000;

mfa::Operand make_operand(const void* ptr, int prec, int B, int Hx, int S, int D,
                          const int64_t* strides, int transposed) {
  mfa::Operand op;
  memset(&op, 0, sizeof(op));
  op.ptr = ptr;
  op.prec = prec;
  if (strides) {
    op.sb = strides[0]; op.sh = strides[1]; op.ss = strides[2]; op.sd = strides[3];
  } else if (transposed) {
    // Column-major within a head: element (s, d) at d * S + s
    // (AttentionKernelDescriptor.transposeState, AttentionKernelDescriptor.swift:34-47).
    op.sd = S; op.ss = 1; op.sh = (int64_t)S * D; op.sb = (int64_t)Hx * S * D;
  } else {
    op.sd = 1; op.ss = D; op.sh = (int64_t)S * D; op.sb = (int64_t)Hx * S * D;
  }
  const int es = precision_size(prec);
  const int vbytes = prec == MFA_PRECISION_INT8 ? 8 : 16;
  op.vec = (op.sd == 1) && ((uintptr_t)ptr % vbytes == 0) && ((op.ss * es) % vbytes == 0) &&
           ((op.sh * es) % vbytes == 0) && ((op.sb * es) % vbytes == 0) &&
           prec != MFA_PRECISION_INT4;
  op.scale = 1.f;
  op.zp = 0;
  op.cols = D;
  (void)B;
  return op;
}

struct MaskPlan {
  mfa::MaskArgs args;
};

mfa_status_t plan_masks(const mfa_attention_descriptor_t& base, const void* mask, int R, int C,
                        mfa::MaskArgs* out) {
  memset(out, 0, sizeof(*out));
  switch (base.sparsity_pattern) {
    case MFA_SPARSITY_NONE:
    case MFA_SPARSITY_CUSTOM:  // treated as none (AttentionDescriptor.swift:226-229)
      break;
    case MFA_SPARSITY_CAUSAL: out->causal = 1; break;
    case MFA_SPARSITY_SLIDING_WINDOW:
      out->window = 1;
      out->window_size = base.window_size;
      break;
    default: return fail(MFA_ERR_INVALID_DESCRIPTOR, "unknown sparsity pattern %d",
                         base.sparsity_pattern);
  }
  if (base.has_sparse_mask) {
    switch (base.mask_type) {
      case MFA_MASK_DENSE: out->amask = (const float*)mask; break;
      case MFA_MASK_SPARSE_RANGES: out->ranges = (const uint32_t*)mask; break;
      case MFA_MASK_BLOCK_SPARSE:
        // HAS_BLOCK_SPARSE only enables the mask block; no predicate reads the buffer
        // and the external additive mask is skipped (AttentionKernel+Softmax.swift:306, :371).
        break;
      default: return fail(MFA_ERR_INVALID_DESCRIPTOR, "unknown mask type %d", base.mask_type);
    }
  } else {
    out->amask = (const float*)mask;  // forward(maskBuffer:) dense additive mask
  }
  // Fully masked tiles may be skipped only when no row is masked everywhere (otherwise the
  // reference's finite mask value makes such a row a uniform average over every key).
  const bool rows_safe = !out->ranges && (!out->window || (int64_t)R <= (int64_t)C + out->window_size);
  out->skip_ok = rows_safe ? 1 : 0;
  return MFA_SUCCESS;
}

// attention_fwd_v2.hip: also D = 256, but needs a positive scale and, with causal / window
// masks, no fully masked row (skip_ok), since it masks with -inf.
bool fwd2_eligible(const mfa::FwdParams& p, int elem, int DP, int kvsrc) {
  if (const char* e = mfa::dev_env("MFA_FWD_GEN")) {
    if (e[0] == '1') return false;
  }
  if (elem != 1 && elem != 2) return false;
  if (kvsrc != 0 || (DP != 64 && DP != 128 && DP != 256)) return false;
  if (!(p.c_log2 > 0.f)) return false;
  // Rows that end up masked everywhere need the reference's finite-mask result: with sparse
  // ranges the kernel writes them after its loop; otherwise they must not occur (skip_ok).
  if ((p.mask.causal || p.mask.window) && !p.mask.skip_ok && !p.mask.ranges) return false;
  if (p.D % 8 != 0 || p.mask.amask) return false;
  if (p.mask.ranges && DP > 128) return false;
  if (!p.q.vec || !p.k.vec || !p.v.vec) return false;
  const int prec = elem == 1 ? MFA_PRECISION_FP16 : MFA_PRECISION_BF16;
  if (p.q.prec != prec || p.k.prec != prec || p.v.prec != prec) return false;
  if (p.k.bscale || p.v.bscale) return false;
  if ((int64_t)p.C * p.k.ss * 2 >= ((int64_t)1 << 31) ||
      (int64_t)p.C * p.v.ss * 2 >= ((int64_t)1 << 31))
    return false;
  return p.q.sd == 1 && p.k.sd == 1 && p.v.sd == 1 && p.o_sd == 1;
}

hipError_t launch_forward(const mfa::FwdParams& p, int elem, int DP, int kvsrc, hipStream_t s) {
  if (DP == kBigD) return mfa::fwd_bigd_dispatch(p, elem, s);
  if (const char* e = mfa::dev_env("MFA_DISABLE_FAST")) {
    if (e[0] == '1') return mfa::fwd_dispatch(p, elem, DP, kvsrc, kvsrc, s);
  }
  if (fwd2_eligible(p, elem, DP, kvsrc)) {
    // Causal shapes with enough work take the stream-split kernel, which needs a workspace
    // (arrival counters + partial states, library scratch slot 10).
    size_t zb = 0;
    const size_t wsb = mfa::fwd_stream_workspace_bytes(p, elem, DP, &zb);
    if (wsb) {
      mfa::FwdParams q = p;
      if (mfa::plan_capture()) q.ws = (void*)kPlanDummy;
      else if (scratch(wsb, &q.ws, 10, s, zb) != MFA_SUCCESS) q.ws = nullptr;
      if (q.ws) {
        hipError_t e = mfa::fwd_stream_dispatch(q, elem, DP, s);
        if (e != hipErrorNotSupported) return e;
      }
    }
    hipError_t e = mfa::fwd2_dispatch(p, elem, DP, s);
    if (e != hipErrorNotSupported) return e;
  }
  return mfa::fwd_dispatch(p, elem, DP, kvsrc, kvsrc, s);
}

// Transposed layouts (column-major within a head: element (s, d) at d·S + s,
// AttentionKernelDescriptor.swift:34-47, leadingDimension AttentionKernel.swift:299-313).
// createTransposeState maps transposeState.O to O and dO and Q / K / V to dQ / dK / dV
// (AttentionDescriptor.swift:150-165); every entry point honours all of them except the
// absorbed-MLA extension, whose operands are library-internal (it rejects any).
mfa_status_t check_transposes(const mfa_attention_descriptor_t& d, bool ok, const char* what) {
  if (!d.has_transpose_state || ok) return MFA_SUCCESS;
  if (d.transpose_o || d.transpose_q || d.transpose_k || d.transpose_v)
    return fail(MFA_ERR_UNSUPPORTED, "%s: transposed operands are not supported", what);
  return MFA_SUCCESS;
}

// Row / column element strides of an FP32 output (O, dQ, dK, dV) of S rows inside its dense
// (batch, head) slice of S·D elements.
void out_strides(int S, int D, bool transposed, int64_t* ss, int64_t* sd) {
  *ss = transposed ? 1 : D;
  *sd = transposed ? S : 1;
}

float resolve_scale(const mfa_attention_descriptor_t& d, int head_dim) {
  // AttentionKernel.swift:63-68: default 1/sqrt(head_dim).
  if (d.has_softmax_scale) return d.softmax_scale;
  return 1.0f / std::sqrt((float)head_dim);
}

}  // namespace

void mfa_api_set_error(const char* msg) {
  g_last_error = msg;
  if (getenv("MFA_DEBUG")) fprintf(stderr, "[mfa] %s\n", msg);
}

// =========================================================================================
extern "C" {

const char* mfa_version(void) { return "mfa-cdna4 0.1.0 (gfx950)"; }
const char* mfa_last_error(void) { return g_last_error.c_str(); }

int mfa_abi_version(void) { return MFA_ABI_VERSION; }

int mfa_release_scratch(void* stream) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  std::lock_guard<std::mutex> lock(g_scratch.mu);
  int n = 0;
  for (auto it = g_scratch.bufs.begin(); it != g_scratch.bufs.end();) {
    if (it->first.dev == dev && (!stream || it->first.stream == (hipStream_t)stream)) {
      if (it->second.ptr) {
        (void)hipFreeAsync(it->second.ptr, it->first.stream);
        ++n;
      }
      it = g_scratch.bufs.erase(it);
    } else {
      ++it;
    }
  }
  return n;
}

int mfa_kernel_attribute_count(void) { return (int)mfa::lds_attr_entries(); }

int mfa_operand_buffer_binding(mfa_operand_t operand) {
  switch (operand) {
    case MFA_OPERAND_Q: return 0;
    case MFA_OPERAND_K: return 1;
    case MFA_OPERAND_V: return 2;
    case MFA_OPERAND_O: return 3;
    case MFA_OPERAND_L: return 4;
    case MFA_OPERAND_D: return 5;
    case MFA_OPERAND_dO: return 6;
    case MFA_OPERAND_dV: return 7;
    case MFA_OPERAND_dK: return 8;
    case MFA_OPERAND_dQ: return 9;
    default: return -1;
  }
}

void mfa_attention_descriptor_init(mfa_attention_descriptor_t* d) {
  memset(d, 0, sizeof(*d));
  d->input_memory_precision = MFA_PRECISION_UNSET;
  d->sparsity_pattern = MFA_SPARSITY_NONE;
  d->mask_type = MFA_MASK_DENSE;
  d->num_kv_heads = 1;
}

void mfa_quantized_configuration_init(mfa_quantized_configuration_t* c) {
  memset(c, 0, sizeof(*c));
  c->query_precision = MFA_PRECISION_FP16;
  c->key_precision = MFA_PRECISION_INT8;
  c->value_precision = MFA_PRECISION_INT8;
  c->strategy_version = 1;  // QuantizationStrategy.currentVersion
  c->mixed_precision_intermediates = 1;
}

mfa_status_t mfa_attention_kernel_descriptor(const mfa_attention_descriptor_t* desc,
                                             mfa_kernel_type_t type,
                                             mfa_kernel_descriptor_t* out) {
  if (!desc || !out) return fail(MFA_ERR_INVALID_ARGUMENT, "null descriptor");
  if (!desc->has_matrix_dimensions || !desc->has_transpose_state)
    return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  memset(out, 0, sizeof(*out));
  const Precisions pr = resolve_precisions(*desc);
  const int D = desc->head;
  if (D <= 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "head dimension 0");
  const int DP = pad_head(D);
  const int elem = elem_of(pr.mem[MFA_OPERAND_Q]);
  if (elem < 0) return fail(MFA_ERR_UNSUPPORTED, "input precision");
  int bp = 0, bt = 0, nw = 0;
  if (DP == kBigD) {
    bp = 128;
    bt = 32;
  } else if (type == MFA_KERNEL_FORWARD || type == MFA_KERNEL_MLA_COMPRESSED) {
    mfa::fwd_block_config(elem, DP, &bp, &bt, &nw);
  } else {
    mfa::bwd_block_config(elem, DP, &bp, &bt, &nw);
  }
  out->block_parallelization = (uint16_t)bp;
  out->block_traversal = (uint16_t)bt;
  // Head block = whole padded head (accumulators stay in registers), clamped to the padded
  // head dimension as AttentionDescriptor.swift:90-105 does; above 256 the head-dimension
  // chunk the D-blocked kernels stream (the reference's Bd, :96-104 of its README).
  out->block_head = DP == kBigD ? (uint16_t)(elem == 0 ? mfa::kBigChunk32 : mfa::kBigChunk16)
                                : (uint16_t)std::min(DP, (D + 7) / 8 * 8);
  out->head_dimension = (uint16_t)D;
  out->sequence_length = std::max(desc->row, desc->column);
  for (int i = 0; i < MFA_OPERAND_COUNT; ++i) {
    out->memory_precisions[i] = pr.mem[i];
    out->register_precisions[i] = pr.reg[i];
    out->cache_state[i] = 0;
    out->transpose_state[i] = 0;
  }
  switch (type) {
    case MFA_KERNEL_FORWARD:
    case MFA_KERNEL_MLA_COMPRESSED:
      out->cache_state[MFA_OPERAND_Q] = out->cache_state[MFA_OPERAND_O] = 1;
      break;
    case MFA_KERNEL_BACKWARD_QUERY:
      out->cache_state[MFA_OPERAND_Q] = out->cache_state[MFA_OPERAND_dO] =
          out->cache_state[MFA_OPERAND_dQ] = 1;
      break;
    case MFA_KERNEL_BACKWARD_KEY_VALUE:
      out->cache_state[MFA_OPERAND_K] = out->cache_state[MFA_OPERAND_V] =
          out->cache_state[MFA_OPERAND_dK] = out->cache_state[MFA_OPERAND_dV] = 1;
      break;
  }
  out->transpose_state[MFA_OPERAND_Q] = out->transpose_state[MFA_OPERAND_dQ] = desc->transpose_q;
  out->transpose_state[MFA_OPERAND_K] = out->transpose_state[MFA_OPERAND_dK] = desc->transpose_k;
  out->transpose_state[MFA_OPERAND_V] = out->transpose_state[MFA_OPERAND_dV] = desc->transpose_v;
  out->transpose_state[MFA_OPERAND_O] = out->transpose_state[MFA_OPERAND_dO] = desc->transpose_o;
  // gfx950 stages every tile through LDS with register prefetch.
  out->prefer_async_cache = 1;
  out->prefer_async_load = 0;
  out->has_softmax_scale = desc->has_softmax_scale;
  out->softmax_scale = desc->softmax_scale;
  out->type = type;
  out->masking_strategy_override = -1;
  return MFA_SUCCESS;
}

mfa_status_t mfa_attention_kernel_create(const mfa_kernel_descriptor_t* k,
                                         mfa_attention_kernel_t* out) {
  if (!k || !out) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  if (k->block_parallelization == 0 || k->head_dimension == 0)
    return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  memset(out, 0, sizeof(*out));
  const int DP = pad_head(k->head_dimension);
  const int elem = elem_of(k->memory_precisions[MFA_OPERAND_Q]);
  if (elem < 0) return fail(MFA_ERR_UNSUPPORTED, "input precision");
  out->block_parallelization = k->block_parallelization;
  out->block_traversal = k->block_traversal;
  out->block_head = k->block_head;
  out->threadgroup_size = (uint16_t)(k->block_parallelization / 32 * 64);
  out->softmax_scale = k->has_softmax_scale ? k->softmax_scale
                                            : 1.0f / std::sqrt((float)k->head_dimension);
  out->type = k->type;
  const char* en = elem == 0 ? "f32" : elem == 1 ? "f16" : "bf16";
  switch (k->type) {
    case MFA_KERNEL_FORWARD:
    case MFA_KERNEL_MLA_COMPRESSED:
      out->threadgroup_memory_allocation =
          (uint32_t)(DP == kBigD ? mfa::bigd_lds_bytes(0, elem) : mfa::fwd_lds_bytes(elem, DP));
      snprintf(out->variant, sizeof(out->variant), "mfa_fwd_%s_d%d_bq%d_bk%d", en, DP,
               k->block_parallelization, k->block_traversal);
      break;
    case MFA_KERNEL_BACKWARD_QUERY:
      out->threadgroup_memory_allocation =
          (uint32_t)(DP == kBigD ? mfa::bigd_lds_bytes(1, elem) : mfa::bwd_lds_bytes(0, elem, DP));
      snprintf(out->variant, sizeof(out->variant), "mfa_bwd_q_%s_d%d_bq%d_bk%d", en, DP,
               k->block_parallelization, k->block_traversal);
      break;
    case MFA_KERNEL_BACKWARD_KEY_VALUE:
      out->threadgroup_memory_allocation =
          (uint32_t)(DP == kBigD ? mfa::bigd_lds_bytes(1, elem) : mfa::bwd_lds_bytes(1, elem, DP));
      snprintf(out->variant, sizeof(out->variant), "mfa_bwd_kv_%s_d%d_bk%d_bq%d", en, DP,
               k->block_parallelization, k->block_traversal);
      break;
  }
  // The kernel a call of this descriptor's shape (one batch item and head, R = C =
  // sequence_length, dense, contiguous) launches: variant, workgroup size and LDS come from
  // the plan query, so they name the instantiation that runs.
  if (k->sequence_length > 0) {
    mfa_multihead_descriptor_t md;
    memset(&md, 0, sizeof(md));
    mfa_attention_descriptor_init(&md.base);
    const int qmem = k->memory_precisions[MFA_OPERAND_Q];
    md.base.low_precision_inputs = qmem != MFA_PRECISION_FP32;
    md.base.input_memory_precision = qmem;
    md.base.low_precision_intermediates = k->memory_precisions[MFA_OPERAND_L] == MFA_PRECISION_FP16;
    md.base.has_matrix_dimensions = 1;
    md.base.row = md.base.column = k->sequence_length;
    md.base.head = k->head_dimension;
    md.base.has_transpose_state = 1;
    md.base.transpose_q = k->transpose_state[MFA_OPERAND_Q];
    md.base.transpose_k = k->transpose_state[MFA_OPERAND_K];
    md.base.transpose_v = k->transpose_state[MFA_OPERAND_V];
    md.base.transpose_o = k->transpose_state[MFA_OPERAND_O];
    md.base.has_softmax_scale = 1;
    md.base.softmax_scale = out->softmax_scale;
    const mfa_multihead_shape_t sh = {1, 1, k->sequence_length, k->head_dimension, 0};
    md.query_shape = md.key_shape = md.value_shape = sh;
    md.broadcast_mode = MFA_BROADCAST_STANDARD;
    const mfa_kernel_type_t t =
        k->type == MFA_KERNEL_MLA_COMPRESSED ? MFA_KERNEL_FORWARD : (mfa_kernel_type_t)k->type;
    mfa_kernel_plan_t plan;
    const mfa_status_t st = mfa_multihead_plan(&md, t, nullptr, &plan);
    if (st != MFA_SUCCESS) return st;
    if (plan.count > 0) {
      snprintf(out->variant, sizeof(out->variant), "%s", plan.launches[0].name);
      out->threadgroup_size = (uint16_t)plan.launches[0].threads;
      out->threadgroup_memory_allocation = plan.launches[0].lds_bytes;
    }
  }
  return MFA_SUCCESS;
}

int mfa_multihead_broadcast_compatible(const mfa_multihead_descriptor_t* d) {
  const mfa_multihead_shape_t& q = d->query_shape;
  const mfa_multihead_shape_t& k = d->key_shape;
  const mfa_multihead_shape_t& v = d->value_shape;
  const bool same_b = q.batch_size == k.batch_size && k.batch_size == v.batch_size;
  const bool same_d = q.head_dimension == k.head_dimension && k.head_dimension == v.head_dimension;
  switch (d->broadcast_mode) {
    case MFA_BROADCAST_STANDARD:
      return same_b && q.num_heads == k.num_heads && k.num_heads == v.num_heads && same_d &&
             k.sequence_length == v.sequence_length;
    case MFA_BROADCAST_GROUPED_QUERY: {
      const uint32_t n = d->broadcast_param;
      return same_b && n > 0 && k.num_heads == n && v.num_heads == n && q.num_heads % n == 0 &&
             same_d && k.sequence_length == v.sequence_length;
    }
    case MFA_BROADCAST_MULTI_QUERY:
      return same_b && k.num_heads == 1 && v.num_heads == 1 && same_d &&
             k.sequence_length == v.sequence_length;
    case MFA_BROADCAST_CROSS_ATTENTION: {
      const uint32_t s = d->broadcast_param;
      return same_b && q.num_heads == k.num_heads && k.num_heads == v.num_heads && same_d &&
             k.sequence_length == s && v.sequence_length == s;
    }
    case MFA_BROADCAST_CUSTOM:
      // The reference only compares the shapes with the ones the case carries
      // (MultiHeadAttentionDescriptor.swift:97-106), which here are the descriptor's own; but the kernels still index K and V with one head count and one sequence length and
      // map query head h to kv head h % Hkv: shapes they cannot address are rejected here
      // rather than read out of bounds.
      return same_b && same_d && k.num_heads == v.num_heads && k.num_heads > 0 &&
             q.num_heads % k.num_heads == 0 && k.sequence_length == v.sequence_length;
    default:
      return 0;
  }
}

}  // extern "C"

// =========================================================================================
// Forward.
namespace {

struct MHAPlan {
  int B, H, Hkv, R, C, D, DP, elem;
  float scale;
  Precisions pr;
  mfa::MaskArgs mask;
};

mfa_status_t plan_multihead(const mfa_multihead_descriptor_t* desc, const void* mask,
                            MHAPlan* pl) {
  if (!desc) return fail(MFA_ERR_INVALID_ARGUMENT, "null descriptor");
  if (!mfa_multihead_broadcast_compatible(desc))
    return fail(MFA_ERR_INVALID_DESCRIPTOR, "Incompatible tensor shapes for broadcast mode %d",
                desc->broadcast_mode);
  const mfa_attention_descriptor_t& base = desc->base;
  if (!base.has_transpose_state) return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  pl->B = (int)desc->query_shape.batch_size;
  pl->H = (int)desc->query_shape.num_heads;
  pl->Hkv = (int)desc->key_shape.num_heads;
  pl->R = (int)desc->query_shape.sequence_length;
  pl->C = (int)desc->key_shape.sequence_length;
  pl->D = (int)desc->query_shape.head_dimension;
  if (pl->B <= 0 || pl->H <= 0 || pl->Hkv <= 0 || pl->D <= 0)
    return fail(MFA_ERR_INVALID_DESCRIPTOR, "empty shape");
  pl->DP = pad_head(pl->D);
  pl->pr = resolve_precisions(base);
  pl->elem = elem_of(pl->pr.mem[MFA_OPERAND_Q]);
  if (pl->elem < 0) return fail(MFA_ERR_UNSUPPORTED, "input precision %d", pl->pr.mem[MFA_OPERAND_Q]);
  pl->scale = resolve_scale(base, pl->D);
  return plan_masks(base, mask, pl->R, pl->C, &pl->mask);
}

}  // namespace

extern "C" mfa_status_t mfa_multihead_forward(const mfa_multihead_descriptor_t* desc,
                                              const mfa_attention_buffers_t* buf,
                                              void* stream) {
  if (!buf) return fail(MFA_ERR_INVALID_ARGUMENT, "null buffers");
  MHAPlan pl;
  mfa_status_t st = plan_multihead(desc, buf->mask, &pl);
  if (st != MFA_SUCCESS) return st;
  if (pl.R == 0) return MFA_SUCCESS;  // empty Q / O may be null (a zero-size allocation)
  if ((st = check_keys(pl.R, pl.C)) != MFA_SUCCESS) return st;
  if (!buf->Q || !buf->K || !buf->V || !buf->O)
    return fail(MFA_ERR_INVALID_ARGUMENT, "forward requires Q, K, V, O");
  const mfa_attention_descriptor_t& base = desc->base;
  const int prec = pl.pr.mem[MFA_OPERAND_Q];

  mfa::FwdParams p;
  memset(&p, 0, sizeof(p));
  p.q = make_operand(buf->Q, prec, pl.B, pl.H, pl.R, pl.D, buf->Q_strides, base.transpose_q);
  p.k = make_operand(buf->K, prec, pl.B, pl.Hkv, pl.C, pl.D, buf->K_strides, base.transpose_k);
  p.v = make_operand(buf->V, prec, pl.B, pl.Hkv, pl.C, pl.D, buf->V_strides, base.transpose_v);
  p.o = (float*)buf->O;
  out_strides(pl.R, pl.D, base.transpose_o, &p.o_ss, &p.o_sd);
  p.o_sh = (int64_t)pl.R * pl.D;
  p.o_sb = (int64_t)pl.H * pl.R * pl.D;
  p.l_f16 = pl.pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  void* L = buf->L;
  if (!L) {
    if (mfa::plan_capture()) L = (void*)kPlanDummy;  // plan query: nothing is allocated
    else if ((st = scratch((size_t)pl.B * pl.H * pl.R * 4, &L, 0, (hipStream_t)stream)) != MFA_SUCCESS)
      return st;
  }
  p.l = L;
  p.B = pl.B; p.H = pl.H; p.Hkv = pl.Hkv; p.R = pl.R; p.C = pl.C; p.D = pl.D;
  int bq, bk, nw;
  mfa::fwd_block_config(pl.elem, pl.DP, &bq, &bk, &nw);
  p.nblk = (pl.R + bq - 1) / bq;
  p.c_log2 = 1.442695041f * pl.scale;  // dotProductScale (AttentionKernel+Softmax.swift:17-25)
  p.o_mul = 1.f;
  p.mask = pl.mask;
  return hip_status(launch_forward(p, pl.elem, pl.DP, 0, (hipStream_t)stream), "mfa_fwd launch");
}

// =========================================================================================
// Quantized forward (QuantizedAttention.forward, QuantizedAttention.swift:135-263).
namespace {

int src_kind(int prec) {
  if (prec == MFA_PRECISION_INT8) return 1;
  if (prec == MFA_PRECISION_INT4) return 2;
  return 0;
}

mfa_status_t quant_operand(const mfa_quantized_tensor_t* t, int cfg_prec, int B, int Hx, int S,
                           int D, mfa::Operand* op, float* fold, int transposed) {
  if (!t || !t->data) return fail(MFA_ERR_INVALID_ARGUMENT, "null quantized tensor");
  const int prec = cfg_prec;
  *op = make_operand(t->data, prec, B, Hx, S, D, nullptr, transposed);
  *fold = 1.f;
  if (is_quantized(prec)) {
    if (t->block_scales) {
      if (t->block_size == 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "blockwise tensor with block size 0");
      op->bscale = t->block_scales;
      op->bzp = t->block_zero_points;
      op->bsize = (int)t->block_size;
      // The block grid is over the memory view (AttentionKernel+Accumulate.swift:461-472):
      // [S][D] rows, or [D][S] rows for a transposed operand (row = d, col = seq,
      // ceil(leadingDimension / BLOCK_SIZE_K) blocks per row, leadingDimension = S).
      op->qtr = transposed ? 1 : 0;
      op->cols = transposed ? S : D;
      op->bcols = (op->cols + (int)t->block_size - 1) / (int)t->block_size;
    } else {
      *fold = t->scale;
      op->zp = t->zero_point;
      // (q - zp) must stay exact in the 16-bit MFMA operand.
      if (t->zero_point < -128 || t->zero_point > 128)
        return fail(MFA_ERR_UNSUPPORTED, "zero point %d outside [-128, 128]", t->zero_point);
    }
  }
  return MFA_SUCCESS;
}

// The integer-matrix-core kernel (attention_fwd_i8.hip): FP16/BF16 Q, INT8 K/V with one
// per-tensor scale and zero point 0, D % 16 == 0, D <= 128, no additive mask or sparse
// ranges, dense rows.  Anything else runs the dequantise-exact path.
bool i8mma_eligible(const mfa::FwdParams& p, int elem, int qp, int kp, int vp) {
  if (elem != 1 && elem != 2) return false;
  if (is_quantized(qp) || kp != MFA_PRECISION_INT8 || vp != MFA_PRECISION_INT8) return false;
  if (p.k.bscale || p.v.bscale || p.k.zp != 0 || p.v.zp != 0) return false;
  if (p.D % 16 != 0 || p.D > 128 || p.mask.amask || p.mask.ranges) return false;
  if (p.q.sd != 1 || p.k.sd != 1 || p.v.sd != 1 || p.o_sd != 1) return false;
  if (p.q.ss % 8 || p.q.sh % 8 || p.q.sb % 8) return false;
  if (p.k.ss % 16 || p.k.sh % 16 || p.k.sb % 16) return false;
  if (p.v.ss % 4 || p.v.sh % 4 || p.v.sb % 4) return false;
  // Per-head K/V byte ranges are addressed with 32-bit buffer offsets.
  if ((int64_t)p.C * p.k.ss >= (int64_t)1 << 31 || (int64_t)p.C * p.v.ss >= (int64_t)1 << 31) return false;
  return ((uintptr_t)p.q.ptr % 16 == 0) && ((uintptr_t)p.k.ptr % 16 == 0) &&
         ((uintptr_t)p.v.ptr % 4 == 0);
}

// The split-KV decode kernel (attention_decode.hip): FP16/BF16 Q, per-tensor INT8 or INT4
// K/V with the same row layout, 16-byte rows (INT4: D % 32 == 0, 16-byte packed rows), D <= 256,
// no mask but causal, dense O rows.
bool decode_eligible(const mfa::FwdParams& p, int elem, int qp, int kp, int vp) {
  if (const char* e = mfa::dev_env("MFA_DECODE")) {
    if (e[0] == '0') return false;
  }
  if (elem != 1 && elem != 2) return false;
  if (is_quantized(qp) || kp != vp || (kp != MFA_PRECISION_INT8 && kp != MFA_PRECISION_INT4))
    return false;
  const int sh = kp == MFA_PRECISION_INT4 ? 1 : 0;  // element -> byte offsets
  if (p.k.bscale || p.v.bscale) return false;
  if (p.D % (16 << sh) != 0 || p.D > 256 || p.C <= 0 || !(p.c_log2 > 0.f)) return false;
  // Causal: key <= query index, masked per lane in the kernel; keys past R are never read.
  // Window: keys below query index - window masked per lane (-inf: exact only when no row is
  // masked everywhere, skip_ok).
  if (p.mask.amask || p.mask.ranges || (p.mask.window && !p.mask.skip_ok)) return false;
  if (p.q.sd != 1 || !p.q.vec || p.k.sd != 1 || p.v.sd != 1) return false;
  const int64_t al = 16 << sh;
  if (p.k.ss != p.v.ss || p.k.ss % al || p.k.sh % al || p.k.sb % al || p.v.sh % al ||
      p.v.sb % al)
    return false;
  if ((uintptr_t)p.k.ptr % 16 || (uintptr_t)p.v.ptr % 16) return false;
  return ((int64_t)p.C * p.k.ss >> sh) < ((int64_t)1 << 31);
}

// The on-load shared-tile forward (attention_fwd_kv8.hip): FP16 or BF16 Q (the compute type),
// per-tensor INT8 or INT4 K/V (any zero point) or block-wise K/V (below), D % 16 == 0 with D <= 256 (padded to 64, 128
// or 256), no masks, dense rows with 16-byte aligned byte offsets.  Causal at D = 128 runs the
// mirrored shared-tile kernel's on-load instantiation where that schedule applies
// (attention_fwd_v2.hip fwd_share_kv8_dispatch; the pass elsewhere).  MFA_KV8=0 routes these
// through the dequantisation pass instead (A/B).
bool kv8_eligible(const mfa::FwdParams& p, int elem, int qp, int kp, int vp, int DP) {
  if (const char* e = mfa::dev_env("MFA_KV8")) {
    if (e[0] == '0') return false;
  }
  if (!((elem == 1 && qp == MFA_PRECISION_FP16) || (elem == 2 && qp == MFA_PRECISION_BF16)))
    return false;
  if (kp != vp || (kp != MFA_PRECISION_INT8 && kp != MFA_PRECISION_INT4)) return false;
  // Block-wise scales (round 6): both K and V block-wise, untransposed, D <= 128, block sizes
  // a multiple of a thread's chunk (16 elements; 8 at D = 64), so each chunk takes one scale.
  if (!p.k.bscale != !p.v.bscale) return false;
  if (p.k.bscale) {
    // The pass + tuned 16-bit kernel is faster where it runs (>= 128 query rows per kv head):
    // the on-load widening of (q - zp)·s costs 0.83-0.94x of it at C3, D = 64 and causal C2
    // (profiles/r06j_ab_kv8_blockwise.txt; each element is widened once per
    // pair of query blocks that reads it, 32 times at C3, where the pass widens it once).  Below that the pass does not pay and the on-load
    // kernel replaces the generic dequantise-on-store kernel.  MFA_KV8_BW=1 takes the on-load
    // kernel at any size (no 16-bit scratch copy), =0 never (A/B).
    const char* e = mfa::dev_env("MFA_KV8_BW");
    if (e && e[0] == '0') return false;
    if (!(e && e[0] == '1') && (int64_t)p.R * (p.H / p.Hkv) >= 128) return false;
    const int ce = DP == 64 ? 8 : 16;
    if (DP > 128 || p.k.qtr || p.v.qtr || p.k.bsize % ce || p.v.bsize % ce) return false;
  }
  if ((DP != 64 && DP != 128 && DP != 256) || p.D % 16 != 0 || !(p.c_log2 > 0.f)) return false;
  const int sh = kp == MFA_PRECISION_INT4 ? 1 : 0;  // element -> byte offsets
  if (p.mask.amask || p.mask.ranges) return false;
  // Causal / window: tiles no row of a block sees are skipped, exact only when no row is
  // masked everywhere (skip_ok).
  if ((p.mask.causal || p.mask.window) && !p.mask.skip_ok) return false;
  if (p.q.sd != 1 || !p.q.vec || p.o_sd != 1) return false;
  if (p.k.sd != 1 || p.v.sd != 1) return false;
  for (const mfa::Operand* o : {&p.k, &p.v})
    if (o->ss % (16 << sh) || o->sh % (16 << sh) || o->sb % (16 << sh) ||
        (uintptr_t)o->ptr % 16)
      return false;
  // Byte offsets are 32-bit, including the prefetch of tile t + 2 (up to 2·64 rows past C).
  const int64_t rows = (int64_t)p.C + 256;
  return (rows * p.k.ss >> sh) < ((int64_t)1 << 31) && (rows * p.v.ss >> sh) < ((int64_t)1 << 31);
}

// Quantised operands go through one dequantisation pass into a dense 16-bit copy
// (kv_dequant.hip) when the compute type is 16-bit, D % 8 == 0 and each kv head serves at
// least 128 query rows: every element is then converted once per call instead of once per
// query block that reads it, and the tuned 16-bit kernels run (bit-identical operands).
// Decode-like shapes (few query rows) keep reading the quantised tensors directly, except
// above D = 256, where the D-blocked kernels take 16-bit operands only.
bool dequant_pass_needed(int D) { return pad_head(D) == kBigD; }
bool dequant_pass_worth(int R, int H, int Hkv, int D, int elem) {
  if (dequant_pass_needed(D)) return true;
  if (const char* e = mfa::dev_env("MFA_NO_DEQUANT_PASS")) {
    if (e[0] == '1') return false;
  }
  return (elem == 1 || elem == 2) && D % 8 == 0 && D <= 256 && (int64_t)R * (H / Hkv) >= 128;
}

// Replaces a quantised *op ([B, Hx, S, D]) by a dense 16-bit operand over this stream's
// scratch `slot`, filled by one kv_dequant launch.  Folded per-tensor scales stay folded.
mfa_status_t dequant_copy(mfa::Operand* op, int B, int Hx, int S, int D, int elem, int slot,
                          hipStream_t stream) {
  void* buf = nullptr;
  if (mfa::plan_capture()) {
    buf = (void*)kPlanDummy;
  } else {
    const mfa_status_t st = scratch((size_t)B * Hx * S * D * 2, &buf, slot, stream);
    if (st != MFA_SUCCESS) return st;
  }
  const mfa_status_t st =
      hip_status(mfa::kv_dequant_dispatch(*op, B, Hx, S, D, elem, buf, stream), "dequant pass");
  if (st != MFA_SUCCESS) return st;
  *op = make_operand(buf, elem == 1 ? MFA_PRECISION_FP16 : MFA_PRECISION_BF16, B, Hx, S, D,
                     nullptr, 0);
  return MFA_SUCCESS;
}

}  // namespace

extern "C" mfa_status_t mfa_quantized_forward(const mfa_quantized_descriptor_t* desc,
                                              const mfa_quantized_tensor_t* query,
                                              const mfa_quantized_tensor_t* key,
                                              const mfa_quantized_tensor_t* value, float* output,
                                              void* logsumexp, const void* mask, void* stream) {
  if (!desc) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  const mfa_attention_descriptor_t& base = desc->base;
  if (!base.has_matrix_dimensions) return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  const int B = desc->batch_size ? (int)desc->batch_size : 1;
  const int H = desc->num_heads ? (int)desc->num_heads : 1;
  const int Hkv = desc->num_kv_heads ? (int)desc->num_kv_heads : H;
  const int R = (int)base.row, C = (int)base.column, D = (int)base.head;
  if (D <= 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "head dimension %d", D);
  const int DP = pad_head(D);
  const bool tq = base.has_transpose_state && base.transpose_q;
  const bool tk = base.has_transpose_state && base.transpose_k;
  const bool tv = base.has_transpose_state && base.transpose_v;
  const bool to = base.has_transpose_state && base.transpose_o;
  const mfa_quantized_configuration_t& cfg = desc->config;
  const int qp = cfg.query_precision, kp = cfg.key_precision, vp = cfg.value_precision;
  // Compute element type: the floating-point input type, FP16 when every input is integer.
  int elem = -1;
  for (int p : {qp, kp, vp}) {
    if (!is_quantized(p)) {
      const int e = elem_of(p);
      if (elem >= 0 && e != elem) return fail(MFA_ERR_UNSUPPORTED, "mixed floating-point input precisions");
      elem = e;
    }
  }
  if (elem < 0) elem = 1;
  if (src_kind(kp) != src_kind(vp))
    return fail(MFA_ERR_UNSUPPORTED, "K and V must share a precision class");
  if (elem == 0 && (is_quantized(qp) || is_quantized(kp)))
    return fail(MFA_ERR_UNSUPPORTED, "FP32 query with quantized K/V");
  mfa_status_t st;
  if (R == 0) return MFA_SUCCESS;  // empty query / output may be null
  if ((st = check_keys(R, C)) != MFA_SUCCESS) return st;
  if (!output) return fail(MFA_ERR_INVALID_ARGUMENT, "null output");

  mfa::FwdParams p;
  memset(&p, 0, sizeof(p));
  float fq = 1.f, fk = 1.f, fv = 1.f;
  if ((st = quant_operand(query, qp, B, H, R, D, &p.q, &fq, tq)) != MFA_SUCCESS) return st;
  if ((st = quant_operand(key, kp, B, Hkv, C, D, &p.k, &fk, tk)) != MFA_SUCCESS) return st;
  if ((st = quant_operand(value, vp, B, Hkv, C, D, &p.v, &fv, tv)) != MFA_SUCCESS) return st;
  p.o = output;
  out_strides(R, D, to, &p.o_ss, &p.o_sd);
  p.o_sh = (int64_t)R * D; p.o_sb = (int64_t)H * R * D;
  const Precisions pr = resolve_precisions(base);
  p.l_f16 = pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  void* L = logsumexp;
  if (!L) {
    if (mfa::plan_capture()) L = (void*)kPlanDummy;  // plan query: nothing is allocated
    else if ((st = scratch((size_t)B * H * R * 4, &L, 0, (hipStream_t)stream)) != MFA_SUCCESS)
      return st;
  }
  p.l = L;
  p.B = B; p.H = H; p.Hkv = Hkv; p.R = R; p.C = C; p.D = D;
  int bq, bk, nw;
  mfa::fwd_block_config(elem, DP, &bq, &bk, &nw);
  p.nblk = (R + bq - 1) / bq;
  const float scale = resolve_scale(base, D);
  p.c_log2 = 1.442695041f * scale * fq * fk;
  p.o_mul = fv;
  if ((st = plan_masks(base, mask, R, C, &p.mask)) != MFA_SUCCESS) return st;
  if (cfg.integer_matmul && i8mma_eligible(p, elem, qp, kp, vp)) {
    mfa::FwdParams pi = p;
    pi.nblk = (R + 127) / 128;
    return hip_status(mfa::fwd_i8mma_dispatch(pi, elem, (hipStream_t)stream),
                      "mfa_fwd (integer matmul) launch");
  }
  if (decode_eligible(p, elem, qp, kp, vp) && !dequant_pass_worth(R, H, Hkv, D, elem)) {
    // Decode / KV-cache shapes: split-KV kernel reading the INT8 bytes (attention_decode.hip).
    // The split-KV partials workspace (scratch slot 9), unless one split per unit merges in
    // LDS (decode_workspace_bytes returns 0: nothing is allocated).
    void* ws = nullptr;
    const size_t wsb = mfa::decode_workspace_bytes(B, Hkv, (H / Hkv) * R,
                                                   mfa::decode_keys(R, C, p.mask.causal), D);
    if (wsb && mfa::plan_capture()) {
      ws = (void*)kPlanDummy;
    } else if (wsb && (st = scratch(wsb, &ws, 9, (hipStream_t)stream)) != MFA_SUCCESS) {
      return st;
    }
    const hipError_t e = mfa::fwd_decode_dispatch(p, elem, ws, (hipStream_t)stream);
    if (e != hipErrorNotSupported) return hip_status(e, "mfa_fwd (decode) launch");
  }
  if (kv8_eligible(p, elem, qp, kp, vp, DP)) {
    // Causal at D = 128: the mirrored shared-tile schedule where it applies; otherwise (and
    // for window masks, D = 64 / 256) the adjacent-pair on-load kernel with the masks.
    hipError_t e = hipErrorNotSupported;
    if (p.mask.causal && !p.mask.window)
      e = mfa::fwd_share_kv8_dispatch(p, elem, DP, src_kind(kp), (hipStream_t)stream);
    if (e == hipErrorNotSupported)
      e = mfa::fwd_kv8_dispatch(p, elem, DP, src_kind(kp), (hipStream_t)stream);
    if (e != hipErrorNotSupported) return hip_status(e, "mfa_fwd (INT8 K/V on load) launch");
  }
  int kvsrc = src_kind(kp);
  if (dequant_pass_worth(R, H, Hkv, D, elem)) {
    hipStream_t s = (hipStream_t)stream;
    if (kvsrc > 0) {
      if ((st = dequant_copy(&p.k, B, Hkv, C, D, elem, 6, s)) != MFA_SUCCESS) return st;
      if ((st = dequant_copy(&p.v, B, Hkv, C, D, elem, 7, s)) != MFA_SUCCESS) return st;
      kvsrc = 0;
    }
    if (is_quantized(qp) && (st = dequant_copy(&p.q, B, H, R, D, elem, 8, s)) != MFA_SUCCESS)
      return st;
  }
  return hip_status(launch_forward(p, elem, DP, kvsrc, (hipStream_t)stream),
                    "mfa_fwd (quantized) launch");
}

// Runtime-quantising forward (QuantizedAttention.swift:278-372): quantize Q, K, V on the GPU,
// then the quantized forward.
extern "C" mfa_status_t mfa_quantized_forward_from_float(
    const mfa_quantized_descriptor_t* desc, const void* query, const void* key, const void* value,
    int32_t query_precision, int32_t key_precision, int32_t value_precision,
    int32_t target_precision, int32_t mode, uint32_t block_size, float* output, void* logsumexp,
    const void* mask, void* stream) {
  if (!desc) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  const mfa_attention_descriptor_t& base = desc->base;
  if (!base.has_matrix_dimensions) return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  const int precs[3] = {query_precision, key_precision, value_precision};
  for (int p : precs)
    if (p != MFA_PRECISION_FP32 && p != MFA_PRECISION_FP16 && p != MFA_PRECISION_BF16)
      return fail(MFA_ERR_UNSUPPORTED, "runtime quantization input precision %d", p);
  mfa_quantized_descriptor_t d = *desc;
  mfa_quantized_tensor_t t[3];
  memset(t, 0, sizeof(t));
  const void* in[3] = {query, key, value};
  if (!is_quantized(target_precision)) {
    // No quantization parameters needed: the buffers as they are (:425-441).
    d.config.query_precision = query_precision;
    d.config.key_precision = key_precision;
    d.config.value_precision = value_precision;
    for (int i = 0; i < 3; ++i) {
      t[i].data = in[i];
      t[i].precision = precs[i];
      t[i].scale = 1.f;
    }
    return mfa_quantized_forward(&d, &t[0], &t[1], &t[2], output, logsumexp, mask, stream);
  }
  if (mode != MFA_QUANT_TENSOR_WISE && mode != MFA_QUANT_BLOCKWISE)
    return fail(MFA_ERR_UNSUPPORTED, "runtime quantization mode %d for attention", mode);
  if (mode == MFA_QUANT_BLOCKWISE && block_size == 0)
    return fail(MFA_ERR_INVALID_ARGUMENT, "blockwise quantization with block size 0");
  const int B = desc->batch_size ? (int)desc->batch_size : 1;
  const int H = desc->num_heads ? (int)desc->num_heads : 1;
  const int Hkv = desc->num_kv_heads ? (int)desc->num_kv_heads : H;
  const uint64_t R = base.row, C = base.column, D = base.head;
  if (R == 0) return MFA_SUCCESS;
  if (!query || !key || !value || !output)
    return fail(MFA_ERR_INVALID_ARGUMENT, "null Q / K / V / output");
  hipStream_t s = (hipStream_t)stream;
  if (mode == MFA_QUANT_TENSOR_WISE && !mfa::plan_capture()) {
    // Tensor-wise scales are read back to the host between quantising and the forward (one
    // stream synchronisation), which a stream under graph capture cannot do.
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(MFA_ERR_UNSUPPORTED,
                  "tensor-wise runtime quantization synchronises the stream: not under graph "
                  "capture (blockwise mode keeps its scales on the device)");
  }
  // Each buffer is quantised as its memory view (GEMMQuantization.swift:561-575): [S][D] rows
  // per head, or [D][S] for a transposed operand (AttentionDescriptor transposeState), so the
  // blockwise grid is the one the forward indexes (quant_operand).
  const bool tr[3] = {base.has_transpose_state && base.transpose_q,
                      base.has_transpose_state && base.transpose_k,
                      base.has_transpose_state && base.transpose_v};
  const uint64_t seq[3] = {R, C, C};
  const uint64_t heads[3] = {(uint64_t)B * H, (uint64_t)B * Hkv, (uint64_t)B * Hkv};
  uint64_t rows[3], cols[3];
  for (int i = 0; i < 3; ++i) {
    rows[i] = heads[i] * (tr[i] ? D : seq[i]);
    cols[i] = tr[i] ? seq[i] : D;
  }
  float host_scale[3] = {1.f, 1.f, 1.f};
  float* dev_scale[3] = {nullptr, nullptr, nullptr};
  auto al = [](size_t x) { return (x + 255) / 256 * 256; };
  for (int i = 0; i < 3; ++i) {
    const uint64_t count = rows[i] * cols[i];
    const size_t qb = al(target_precision == MFA_PRECISION_INT8 ? count : (count + 1) / 2);
    const uint64_t nb = mode == MFA_QUANT_BLOCKWISE
                            ? ((rows[i] + block_size - 1) / block_size) * ((cols[i] + block_size - 1) / block_size)
                            : 0;
    const size_t ws = al(mfa_quantize_workspace_size(count, (uint32_t)rows[i], (uint32_t)cols[i], mode, block_size));
    const size_t bytes = qb + 256 + ws + 2 * al(nb * 4);
    void* buf = nullptr;
    if (mfa::plan_capture()) return fail(MFA_ERR_UNSUPPORTED, "plan query of the runtime-quantising forward");
    mfa_status_t st = scratch(bytes, &buf, 11 + i, s);
    if (st != MFA_SUCCESS) return st;
    char* c = (char*)buf;
    dev_scale[i] = (float*)(c + qb);
    void* work = c + qb + 256;
    float* bsc = nb ? (float*)(c + qb + 256 + ws) : nullptr;
    int32_t* bzp = nb ? (int32_t*)(c + qb + 256 + ws + al(nb * 4)) : nullptr;
    st = mfa_quantize(in[i], precs[i], count, (uint32_t)rows[i], (uint32_t)cols[i], target_precision, mode,
                      block_size, c, dev_scale[i], bsc, bzp, ws ? work : nullptr, stream);
    if (st != MFA_SUCCESS) return st;
    t[i].data = c;
    t[i].precision = target_precision;
    t[i].block_scales = bsc;
    t[i].block_zero_points = bzp;
    t[i].block_size = nb ? block_size : 0;
  }
  if (mode == MFA_QUANT_TENSOR_WISE) {
    for (int i = 0; i < 3; ++i)
      if (hipMemcpyAsync(&host_scale[i], dev_scale[i], 4, hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail(MFA_ERR_LAUNCH, "reading back the tensor-wise scales");
    if (hipStreamSynchronize(s) != hipSuccess) return fail(MFA_ERR_LAUNCH, "stream synchronisation");
    for (int i = 0; i < 3; ++i) t[i].scale = host_scale[i];
  }
  d.config.query_precision = d.config.key_precision = d.config.value_precision = target_precision;
  return mfa_quantized_forward(&d, &t[0], &t[1], &t[2], output, logsumexp, mask, stream);
}

// =========================================================================================
// Host utilities.
extern "C" int mfa_masking_sequence_bucket(int sequence_length) {
  // MaskingStrategyHeuristic.sequenceBucket (MaskingStrategyHeuristic.swift:47-60).
  static const int anchors[] = {64, 128, 256, 512, 768, 1024, 1536, 2048, 3072, 4096};
  int best = anchors[0];
  int best_delta = std::abs(sequence_length - best);
  for (int i = 1; i < 10; ++i) {
    const int delta = std::abs(sequence_length - anchors[i]);
    if (delta < best_delta) {
      best = anchors[i];
      best_delta = delta;
    }
  }
  return best;
}

extern "C" int mfa_masking_default_rule(int s, int h) {
  // MaskingStrategyHeuristic.defaultRule (MaskingStrategyHeuristic.swift:111-136);
  // 1 = bitmask, 0 = elementWise.
  if (h == 192) return 1;
  if (s >= 4096) return 0;
  if (s >= 1792 && s <= 2560) return 1;
  if (h == 128) return s <= 256 ? 1 : 0;
  if (s <= 256) return 1;
  if (h == 256 && s >= 1024) return 0;
  return 1;
}

extern "C" void mfa_sparse_build_sliding_window(uint32_t n, uint32_t window, uint32_t* out) {
  // SparseMQABuilder.buildSlidingWindow (SparseMQABuilder.swift:4-28).
  const int64_t capped = std::max<int64_t>(1, (int64_t)window);
  const int64_t half = capped / 2;
  for (int64_t i = 0; i < (int64_t)n; ++i) {
    out[2 * i] = (uint32_t)std::max<int64_t>(0, i - half);
    out[2 * i + 1] = (uint32_t)std::min<int64_t>((int64_t)n, i + half);
  }
}

extern "C" void mfa_sparse_build_block_sparse(const uint8_t* pattern, uint32_t rows,
                                              uint32_t cols, uint32_t block_size,
                                              uint32_t* out) {
  // SparseMQABuilder.buildBlockSparse (SparseMQABuilder.swift:30-62).
  for (uint32_t r = 0; r < rows; ++r) {
    int64_t first = -1, last = -1;
    for (uint32_t c = 0; c < cols; ++c)
      if (pattern[(size_t)r * cols + c]) {
        if (first < 0) first = c;
        last = c;
      }
    if (first >= 0) {
      const int64_t maxc = (int64_t)cols * block_size;
      out[2 * r] = (uint32_t)(first * block_size);
      out[2 * r + 1] = (uint32_t)std::min<int64_t>((last + 1) * block_size, maxc);
    } else {
      out[2 * r] = 0;
      out[2 * r + 1] = 0;
    }
  }
}

// =========================================================================================
// Backward (MultiHeadAttention.backward, MultiHeadAttention.swift:574-707).
namespace {

enum BwdPhase { PHASE_QUERY = 1, PHASE_KV = 2, PHASE_BOTH = 3 };

// The tuned backward kernels (attention_bwd_fast.hip) cover 16-bit Q/K/V/dO with contiguous
// 16-byte aligned rows, D % 8 == 0, and no mask or skippable causal / window masks.
// kv_quant: the backwardKeyValue kernel, which reads K and V once per workgroup into
// registers, takes per-tensor quantised K/V (INT8/INT4, dense rows) directly.
bool bwd_fast_eligible(const mfa::BwdParams& p, int elem, int DP, int ksrc, int qsrc,
                       bool kv_quant = false) {
  if (const char* e = mfa::dev_env("MFA_DISABLE_FAST")) {
    if (e[0] == '1') return false;
  }
  if (elem != 1 && elem != 2) return false;
  if (DP != 64 && DP != 128 && DP != 256) return false;
  if (qsrc != 0 || p.D % 8 != 0) return false;
  if (ksrc != 0 && !kv_quant) return false;
  const int prec = elem == 1 ? MFA_PRECISION_FP16 : MFA_PRECISION_BF16;
  for (const mfa::Operand* op : {&p.q, &p.k, &p.v, &p.dO_op}) {
    const bool kvq = ksrc != 0 && (op == &p.k || op == &p.v);
    if (kvq) {
      if (!is_quantized(op->prec) || op->sd != 1 || op->bscale) return false;
      continue;
    }
    if (op->prec != prec || !op->vec || op->sd != 1 || op->bscale) return false;
  }
  // Additive masks and ranges run the kernels' element-wise mask instantiation (16-bit K/V),
  // which also covers fully masked rows, so it needs no skip_ok.
  const bool msk = p.mask.amask || p.mask.ranges;
  if (msk && ksrc != 0) return false;
  // The backwardKeyValue mask tile moves by 16-byte LDS-DMA: 16-byte aligned rows.
  if (p.mask.amask && (p.C % 4 != 0 || ((uintptr_t)p.mask.amask & 15) != 0)) return false;
  if ((p.mask.causal || p.mask.window) && !p.mask.skip_ok && !msk) return false;
  // Dense O, dQ, dK, dV rows.
  if (p.o_sd != 1 || p.dq_sd != 1 || p.dk_sd != 1 || p.dv_sd != 1) return false;
  // Tiles are addressed per head with 32-bit buffer offsets.
  const int64_t lim = (int64_t)1 << 31;
  if ((ksrc == 0 && ((int64_t)p.C * p.k.ss * 2 >= lim || (int64_t)p.C * p.v.ss * 2 >= lim)) ||
      (int64_t)p.R * p.q.ss * 2 >= lim || (int64_t)p.R * p.dO_op.ss * 2 >= lim)
    return false;
  return true;
}

// kv_widen: quantised K/V (16-bit Q) may run the tuned key-phase kernel, which widens them in
// registers (quantized_backward decides it; false everywhere else).
// q_widen: the same for the query phase, whose kernel stages the stored K/V bytes through an
// LDS byte ring and widens them there (kv_bytes.h).
mfa_status_t run_backward(const mfa::BwdParams& base_p, int elem, int DP, int ksrc, int qsrc,
                          int phase, hipStream_t stream, bool kv_widen = false,
                          bool q_widen = false) {
  mfa::BwdParams p = base_p;
  if (mfa_status_t st = check_keys(p.R, p.C)) return st;
  if (p.R == 0)
    return (phase & PHASE_KV) ? zero_kv_grads(p.dk, p.dv, (size_t)p.B * p.Hkv * p.C * p.D, stream)
                              : MFA_SUCCESS;
  int bp, bt, nw;
  mfa::bwd_block_config(elem, DP, &bp, &bt, &nw);
  const bool big = DP == kBigD;
  const bool fast = !big && bwd_fast_eligible(p, elem, DP, ksrc, qsrc);
  if (phase & PHASE_QUERY) {
    p.nblk = (p.R + bp - 1) / bp;
    if (p.R > 0) {
      const bool fast_q = fast || (!big && ksrc > 0 && q_widen);
      hipError_t e = big      ? mfa::bwd_bigd_dispatch(p, 0, elem, stream)
                     : fast_q ? mfa::bwd_fast_dispatch(p, 0, elem, DP, stream)
                              : hipErrorNotSupported;
      if (big && e == hipErrorNotSupported)
        return fail(MFA_ERR_UNSUPPORTED, "head dimension %d: mixed operand precisions", p.D);
      if (e == hipErrorNotSupported) e = mfa::bwd_q_dispatch(p, elem, DP, ksrc, ksrc, stream);
      mfa_status_t st = hip_status(e, "mfa_bwd_q launch");
      if (st != MFA_SUCCESS) return st;
    }
  }
  if (phase & PHASE_KV) {
    p.nblk = (p.C + bp - 1) / bp;
    if (p.C > 0) {
      // Quantised K/V with 16-bit Q: the tuned kernel widens them in registers when
      // quantized_backward chose that (kv_widen); otherwise the generic kernel dequantises.
      const bool fast_kv = fast || (!big && ksrc > 0 && kv_widen);
      // D = 256 calls the tuned kernel does not take (strides, transposes): the generic kernel.
      // MFA_BWD256_BIGD=1 runs the D-blocked kernel in two 128-column slices instead (measured
      // 3x slower: each slice recomputes S and dP over all 256 columns on 32-row tiles).
      const char* b256 = mfa::dev_env("MFA_BWD256_BIGD");
      const bool blocked = !big && !fast_kv && DP == 256 && elem != 0 && ksrc == 0 && qsrc == 0 &&
                           b256 && b256[0] == '1';
      hipError_t e = big || blocked ? mfa::bwd_bigd_dispatch(p, 1, elem, stream)
                     : fast_kv      ? mfa::bwd_fast_dispatch(p, 1, elem, DP, stream)
                                    : hipErrorNotSupported;
      if (big && e == hipErrorNotSupported)
        return fail(MFA_ERR_UNSUPPORTED, "head dimension %d: mixed operand precisions", p.D);
      if (e == hipErrorNotSupported) e = mfa::bwd_kv_dispatch(p, elem, DP, ksrc, qsrc, stream);
      mfa_status_t st = hip_status(e, "mfa_bwd_kv launch");
      if (st != MFA_SUCCESS) return st;
    }
  }
  return MFA_SUCCESS;
}

mfa_status_t multihead_backward(const mfa_multihead_descriptor_t* desc,
                                const mfa_attention_buffers_t* buf, void* stream, int phase) {
  if (!buf) return fail(MFA_ERR_INVALID_ARGUMENT, "null buffers");
  const bool need_q = phase & PHASE_QUERY, need_kv = phase & PHASE_KV;
  MHAPlan pl;
  mfa_status_t st = plan_multihead(desc, buf->mask, &pl);
  if (st != MFA_SUCCESS) return st;
  if ((st = check_keys(pl.R, pl.C)) != MFA_SUCCESS) return st;
  // With no queries only dK / dV are written (zeros); the empty row operands may be null.
  if (pl.R > 0 ? (!buf->Q || !buf->K || !buf->V || !buf->L || !buf->D || !buf->dO ||
                  (need_q && (!buf->O || !buf->dQ)) || (need_kv && (!buf->dK || !buf->dV)))
               : (need_kv && pl.C > 0 && (!buf->dK || !buf->dV)))
    return fail(MFA_ERR_INVALID_ARGUMENT, "backward requires Q K V O L D dO and the gradients");
  const mfa_attention_descriptor_t& base = desc->base;
  const int prec = pl.pr.mem[MFA_OPERAND_Q];
  mfa::BwdParams p;
  memset(&p, 0, sizeof(p));
  p.q = make_operand(buf->Q, prec, pl.B, pl.H, pl.R, pl.D, buf->Q_strides, base.transpose_q);
  p.k = make_operand(buf->K, prec, pl.B, pl.Hkv, pl.C, pl.D, buf->K_strides, base.transpose_k);
  p.v = make_operand(buf->V, prec, pl.B, pl.Hkv, pl.C, pl.D, buf->V_strides, base.transpose_v);
  p.dO_op = make_operand(buf->dO, pl.pr.mem[MFA_OPERAND_dO], pl.B, pl.H, pl.R, pl.D, nullptr,
                         base.transpose_o);
  p.o = (const float*)buf->O;
  p.l = buf->L;
  p.l_f16 = pl.pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  p.dD = buf->D;
  p.d_bf16 = pl.pr.mem[MFA_OPERAND_D] == MFA_PRECISION_BF16;
  p.dq = (float*)buf->dQ;
  p.dk = (float*)buf->dK;
  p.dv = (float*)buf->dV;
  out_strides(pl.R, pl.D, base.transpose_o, &p.o_ss, &p.o_sd);
  out_strides(pl.R, pl.D, base.transpose_q, &p.dq_ss, &p.dq_sd);
  out_strides(pl.C, pl.D, base.transpose_k, &p.dk_ss, &p.dk_sd);
  out_strides(pl.C, pl.D, base.transpose_v, &p.dv_ss, &p.dv_sd);
  p.B = pl.B; p.H = pl.H; p.Hkv = pl.Hkv; p.R = pl.R; p.C = pl.C; p.D = pl.D;
  p.group = pl.H / pl.Hkv;
  p.c_log2 = 1.442695041f * pl.scale;
  p.scale = pl.scale;
  p.dscale = pl.scale;
  p.dq_mul = 1.f;
  p.dk_mul = 1.f;
  p.mask = pl.mask;
  return run_backward(p, pl.elem, pl.DP, 0, 0, phase, (hipStream_t)stream);
}

}  // namespace

extern "C" mfa_status_t mfa_multihead_backward(const mfa_multihead_descriptor_t* desc,
                                               const mfa_attention_buffers_t* buffers,
                                               void* stream) {
  return multihead_backward(desc, buffers, stream, PHASE_BOTH);
}
extern "C" mfa_status_t mfa_multihead_backward_query(const mfa_multihead_descriptor_t* desc,
                                                     const mfa_attention_buffers_t* buffers,
                                                     void* stream) {
  return multihead_backward(desc, buffers, stream, PHASE_QUERY);
}
extern "C" mfa_status_t mfa_multihead_backward_key_value(const mfa_multihead_descriptor_t* desc,
                                                         const mfa_attention_buffers_t* buffers,
                                                         void* stream) {
  return multihead_backward(desc, buffers, stream, PHASE_KV);
}

// Quantized backward (QuantizedAttention.backwardQuery / backwardKeyValue,
// QuantizedAttention.swift:1012-1181).
namespace {

mfa_status_t quantized_backward(const mfa_quantized_descriptor_t* desc,
                                const mfa_quantized_tensor_t* query,
                                const mfa_quantized_tensor_t* key,
                                const mfa_quantized_tensor_t* value, const float* output,
                                const void* grad_output, const void* logsumexp,
                                float* grad_query, float* grad_key, float* grad_value,
                                void* d_values, int phase, void* stream) {
  if (!desc) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  if ((phase & PHASE_KV) && (!grad_key || !grad_value))
    return fail(MFA_ERR_INVALID_ARGUMENT, "backwardKeyValue requires gradKey and gradValue");
  const mfa_attention_descriptor_t& base = desc->base;
  if (!base.has_matrix_dimensions) return fail(MFA_ERR_INVALID_DESCRIPTOR, "Descriptor was incomplete.");
  const int B = desc->batch_size ? (int)desc->batch_size : 1;
  const int H = desc->num_heads ? (int)desc->num_heads : 1;
  const int Hkv = desc->num_kv_heads ? (int)desc->num_kv_heads : H;
  const int R = (int)base.row, C = (int)base.column, D = (int)base.head;
  if (D <= 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "head dimension %d", D);
  if (mfa_status_t st = check_keys(R, C)) return st;
  if (R == 0)  // no queries: the row operands may be null (zero-size allocations)
    return (phase & PHASE_KV) ? zero_kv_grads(grad_key, grad_value, (size_t)B * Hkv * C * D,
                                              (hipStream_t)stream)
                              : MFA_SUCCESS;
  if (!grad_output || !logsumexp || !d_values)
    return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  if ((phase & PHASE_QUERY) && (!output || !grad_query))
    return fail(MFA_ERR_INVALID_ARGUMENT, "backwardQuery requires output and gradQuery");
  const int DP = pad_head(D);
  const bool tr = base.has_transpose_state;
  const bool tq = tr && base.transpose_q, tk = tr && base.transpose_k;
  const bool tv = tr && base.transpose_v, to = tr && base.transpose_o;
  const mfa_quantized_configuration_t& cfg = desc->config;
  const int qp = cfg.query_precision, kp = cfg.key_precision, vp = cfg.value_precision;
  int elem = -1;
  for (int pz : {qp, kp, vp}) {
    if (!is_quantized(pz)) {
      const int e = elem_of(pz);
      if (elem >= 0 && e != elem) return fail(MFA_ERR_UNSUPPORTED, "mixed floating-point input precisions");
      elem = e;
    }
  }
  if (elem < 0) elem = 1;
  if (src_kind(kp) != src_kind(vp))
    return fail(MFA_ERR_UNSUPPORTED, "K and V must share a precision class");
  if (elem == 0 && (is_quantized(qp) || is_quantized(kp)))
    return fail(MFA_ERR_UNSUPPORTED, "FP32 query with quantized K/V");
  const Precisions pr = resolve_precisions(base);
  if (elem == 0 && pr.mem[MFA_OPERAND_dO] != MFA_PRECISION_FP32)
    return fail(MFA_ERR_UNSUPPORTED, "FP32 kernels need FP32 dO");
  if (elem != 0 && pr.mem[MFA_OPERAND_dO] != MFA_PRECISION_FP32 &&
      elem_of(pr.mem[MFA_OPERAND_dO]) != elem)
    return fail(MFA_ERR_UNSUPPORTED, "dO precision must be FP32 or the input precision");

  mfa::BwdParams p;
  memset(&p, 0, sizeof(p));
  float fq = 1.f, fk = 1.f, fv = 1.f;
  mfa_status_t st;
  if ((st = quant_operand(query, qp, B, H, R, D, &p.q, &fq, tq)) != MFA_SUCCESS) return st;
  if ((st = quant_operand(key, kp, B, Hkv, C, D, &p.k, &fk, tk)) != MFA_SUCCESS) return st;
  if ((st = quant_operand(value, vp, B, Hkv, C, D, &p.v, &fv, tv)) != MFA_SUCCESS) return st;
  p.dO_op = make_operand(grad_output, pr.mem[MFA_OPERAND_dO], B, H, R, D, nullptr, to);
  out_strides(R, D, to, &p.o_ss, &p.o_sd);
  out_strides(R, D, tq, &p.dq_ss, &p.dq_sd);
  out_strides(C, D, tk, &p.dk_ss, &p.dk_sd);
  out_strides(C, D, tv, &p.dv_ss, &p.dv_sd);
  p.o = output;
  p.l = logsumexp;
  p.l_f16 = pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  p.dD = d_values;
  p.d_bf16 = pr.mem[MFA_OPERAND_D] == MFA_PRECISION_BF16;
  p.dq = grad_query;
  p.dk = grad_key;
  p.dv = grad_value;
  p.B = B; p.H = H; p.Hkv = Hkv; p.R = R; p.C = C; p.D = D;
  p.group = H / Hkv;
  const float scale = resolve_scale(base, D);
  p.c_log2 = 1.442695041f * scale * fq * fk;
  p.scale = scale * fv;
  p.dscale = scale;
  p.dq_mul = fk;
  p.dk_mul = fq;
  if ((st = plan_masks(base, nullptr, R, C, &p.mask)) != MFA_SUCCESS) return st;
  int ksrc = src_kind(kp), qsrc = src_kind(qp);
  // backwardKeyValue alone with 16-bit Q: its kernel reads each key block's K/V rows once per
  // workgroup into registers and widens them there, so the pass would only add traffic
  // (MFA_KV_REGS=0 keeps the pass: A/B, bit-identity tests).
  // Where no pass runs (small problems), the key phase widens in registers too, unless
  // MFA_KV_REGS=0.
  const char* kvr = mfa::dev_env("MFA_KV_REGS");
  const bool kv_widen = ksrc > 0 && qsrc == 0 && !(kvr && kvr[0] == '0') &&
                        !dequant_pass_needed(D) && bwd_fast_eligible(p, elem, DP, ksrc, qsrc, true);
  // The query phase can take them on load too (LDS byte ring, kv_bytes.h) when the stored rows
  // suit 16-byte (INT8) / 8-byte (INT4) chunks: per-tensor, D % 16 == 0, 16-byte aligned rows
  // and heads.  It does so where the pass is not worth running (few query rows per kv head,
  // where the generic kernel read the quantised K/V before).  Above that the pass stays: that
  // kernel runs one wave per SIMD, so nothing hides the widening's LDS round trips and VALU,
  // which every query block repeats for every K/V tile (measured 1.34x the pass path's time at
  // B4 H32 S4096 D128 INT8, 1.19x at D = 256).  MFA_BWDQ_BYTES=1 / 0 forces
  // the byte ring / the pass (A/B, bit-identity tests).
  const char* qb = mfa::dev_env("MFA_BWDQ_BYTES");
  bool q_widen = kv_widen && D % 16 == 0 &&
                 (qb ? qb[0] == '1' : !dequant_pass_worth(R, H, Hkv, D, elem));
  if (q_widen) {
    const int sh = ksrc == 2 ? 1 : 0;
    for (const mfa::Operand* o : {&p.k, &p.v})
      if (o->ss % (16 << sh) || o->sh % (16 << sh) || o->sb % (16 << sh) ||
          (uintptr_t)o->ptr % 16 || (((int64_t)C + 128) * o->ss >> sh) >= ((int64_t)1 << 31))
        q_widen = false;
  }
  const bool kv_regs = kv_widen && (!(phase & PHASE_QUERY) || q_widen);
  if (dequant_pass_worth(R, H, Hkv, D, elem) && !kv_regs) {
    hipStream_t s = (hipStream_t)stream;
    if (ksrc > 0) {
      if ((st = dequant_copy(&p.k, B, Hkv, C, D, elem, 6, s)) != MFA_SUCCESS) return st;
      if ((st = dequant_copy(&p.v, B, Hkv, C, D, elem, 7, s)) != MFA_SUCCESS) return st;
      ksrc = 0;
    }
    if (qsrc > 0) {
      if ((st = dequant_copy(&p.q, B, H, R, D, elem, 8, s)) != MFA_SUCCESS) return st;
      qsrc = 0;
    }
  }
  return run_backward(p, elem, DP, ksrc, qsrc, phase, (hipStream_t)stream, kv_widen, q_widen);
}

}  // namespace

extern "C" mfa_status_t mfa_quantized_backward_query(
    const mfa_quantized_descriptor_t* desc, const mfa_quantized_tensor_t* query,
    const mfa_quantized_tensor_t* key, const mfa_quantized_tensor_t* value, const float* output,
    const void* grad_output, const void* logsumexp, float* grad_query, void* d_values,
    void* stream) {
  return quantized_backward(desc, query, key, value, output, grad_output, logsumexp, grad_query,
                            nullptr, nullptr, d_values, PHASE_QUERY, stream);
}

extern "C" mfa_status_t mfa_quantized_backward_key_value(
    const mfa_quantized_descriptor_t* desc, const mfa_quantized_tensor_t* query,
    const mfa_quantized_tensor_t* key, const mfa_quantized_tensor_t* value,
    const void* grad_output, const void* logsumexp, const void* d_values, float* grad_key,
    float* grad_value, void* stream) {
  return quantized_backward(desc, query, key, value, nullptr, grad_output, logsumexp, nullptr,
                            grad_key, grad_value, (void*)d_values, PHASE_KV, stream);
}

// =========================================================================================
// Plan query: the dispatchers above run with launches recorded (mfa_launch.h).
namespace {

struct CaptureScope {
  mfa::PlanCapture cap;
  mfa::PlanCapture* prev;
  CaptureScope() : prev(mfa::plan_capture()) { mfa::plan_capture() = &cap; }
  ~CaptureScope() { mfa::plan_capture() = prev; }
  void copy_to(mfa_kernel_plan_t* out) const {
    out->count = cap.count;
    out->total = cap.total;
    for (int i = 0; i < cap.count; ++i) {
      static_assert(sizeof(out->launches[i].name) == sizeof(cap.rec[i].name), "name size");
      memcpy(out->launches[i].name, cap.rec[i].name, sizeof(out->launches[i].name));
      out->launches[i].threads = cap.rec[i].threads;
      out->launches[i].lds_bytes = cap.rec[i].lds_bytes;
      out->launches[i].workgroups = cap.rec[i].workgroups;
    }
  }
};

template <class T>
void fill_dummy(T*& p) {
  if (!p) p = (T*)kPlanDummy;
}

}  // namespace

extern "C" mfa_status_t mfa_multihead_plan(const mfa_multihead_descriptor_t* desc,
                                           mfa_kernel_type_t type,
                                           const mfa_attention_buffers_t* buffers,
                                           mfa_kernel_plan_t* out) {
  if (!desc || !out) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  memset(out, 0, sizeof(*out));
  mfa_attention_buffers_t b;
  if (buffers) b = *buffers;
  else memset(&b, 0, sizeof(b));
  fill_dummy(b.Q); fill_dummy(b.K); fill_dummy(b.V); fill_dummy(b.O);
  fill_dummy(b.D); fill_dummy(b.dO); fill_dummy(b.dV); fill_dummy(b.dK); fill_dummy(b.dQ);
  if (type != MFA_KERNEL_FORWARD) fill_dummy(b.L);  // forward: NULL L plans the scratch case
  if (desc->base.has_sparse_mask) fill_dummy(b.mask);
  CaptureScope scope;
  mfa_status_t st;
  switch (type) {
    case MFA_KERNEL_FORWARD: st = mfa_multihead_forward(desc, &b, nullptr); break;
    case MFA_KERNEL_BACKWARD_QUERY: st = multihead_backward(desc, &b, nullptr, PHASE_QUERY); break;
    case MFA_KERNEL_BACKWARD_KEY_VALUE: st = multihead_backward(desc, &b, nullptr, PHASE_KV); break;
    default: return fail(MFA_ERR_UNSUPPORTED, "no multihead plan for kernel type %d", (int)type);
  }
  if (st == MFA_SUCCESS) scope.copy_to(out);
  return st;
}

extern "C" int mfa_last_launches(mfa_kernel_plan_t* out) {
  mfa::LaunchLog& log = mfa::launch_log();
  const uint64_t n = std::min<uint64_t>(log.total, 4);
  if (out) {
    memset(out, 0, sizeof(*out));
    out->count = (int32_t)n;
    out->total = (int32_t)std::min<uint64_t>(log.total, 1u << 30);
    for (uint64_t j = 0; j < n; ++j) {
      const int i = (int)((log.total - n + j) % mfa::LaunchLog::kMax);
      mfa::kernel_symbol_name(log.handle[i], out->launches[j].name, sizeof(out->launches[j].name));
      out->launches[j].threads = log.threads[i];
      out->launches[j].lds_bytes = log.lds[i];
      out->launches[j].workgroups = log.workgroups[i];
    }
  }
  const int total = (int)std::min<uint64_t>(log.total, 1u << 30);
  log.total = 0;
  return total;
}

extern "C" mfa_status_t mfa_quantized_plan(const mfa_quantized_descriptor_t* desc,
                                           mfa_kernel_type_t type,
                                           const mfa_quantized_tensor_t* query,
                                           const mfa_quantized_tensor_t* key,
                                           const mfa_quantized_tensor_t* value,
                                           mfa_kernel_plan_t* out) {
  if (!desc || !out) return fail(MFA_ERR_INVALID_ARGUMENT, "null argument");
  memset(out, 0, sizeof(*out));
  mfa_quantized_tensor_t t[3];
  const mfa_quantized_tensor_t* in[3] = {query, key, value};
  const int precs[3] = {desc->config.query_precision, desc->config.key_precision,
                        desc->config.value_precision};
  for (int i = 0; i < 3; ++i) {
    if (in[i]) {
      t[i] = *in[i];
    } else {
      memset(&t[i], 0, sizeof(t[i]));
      t[i].precision = precs[i];
      t[i].scale = 1.f;
    }
    fill_dummy(t[i].data);
  }
  float* const fd = (float*)kPlanDummy;
  void* const vd = (void*)kPlanDummy;
  CaptureScope scope;
  mfa_status_t st;
  switch (type) {
    case MFA_KERNEL_FORWARD:
      st = mfa_quantized_forward(desc, &t[0], &t[1], &t[2], fd, nullptr, nullptr, nullptr);
      break;
    case MFA_KERNEL_BACKWARD_QUERY:
      st = quantized_backward(desc, &t[0], &t[1], &t[2], fd, vd, vd, fd, nullptr, nullptr, vd,
                              PHASE_QUERY, nullptr);
      break;
    case MFA_KERNEL_BACKWARD_KEY_VALUE:
      st = quantized_backward(desc, &t[0], &t[1], &t[2], nullptr, vd, vd, nullptr, fd, fd, vd,
                              PHASE_KV, nullptr);
      break;
    default: return fail(MFA_ERR_UNSUPPORTED, "no quantized plan for kernel type %d", (int)type);
  }
  if (st == MFA_SUCCESS) scope.copy_to(out);
  return st;
}

// =========================================================================================
// MLA (MLAOptimizedGEMMMFA.forward, MLAOptimizedGEMMMFA.swift:158-240) + the attention forward
// its caller runs on the decompressed BSHD K/V (stride pattern KernelRegressionTests.swift:
// 398-465).
extern "C" mfa_status_t mfa_mla_forward(const mfa_mla_descriptor_t* desc, const void* kv_latent,
                                        const void* w_k, const void* w_v, const void* query,
                                        void* decompressed_k, void* decompressed_v,
                                        float* output, void* logsumexp, void* stream) {
  if (!desc || !kv_latent || !w_k || !w_v || !query || !output)
    return fail(MFA_ERR_INVALID_ARGUMENT, "MLA forward requires latent, weights, query, output");
  const int prec = desc->precision;
  if (prec != MFA_PRECISION_FP16 && prec != MFA_PRECISION_BF16)
    return fail(MFA_ERR_UNSUPPORTED, "MLA precision must be FP16 or BF16");
  const int B = (int)desc->batch_size, H = (int)desc->num_heads;
  const int Sq = (int)desc->sequence_length_q, Skv = (int)desc->sequence_length_kv;
  const int D = (int)desc->head_dim, Lat = (int)desc->kv_latent_dim;
  if (B <= 0 || H <= 0 || D <= 0 || Lat <= 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "empty MLA shape");
  const int DP = pad_head(D);
  // The decompressed K/V are written by this call in BSHD (their transpose flags do not
  // apply); a transposed query and output are honoured.
  const bool tq = desc->base.has_transpose_state && desc->base.transpose_q;
  const bool to = desc->base.has_transpose_state && desc->base.transpose_o;
  const int64_t kv_elems = (int64_t)B * Skv * H * D;
  hipStream_t s = (hipStream_t)stream;
  mfa_status_t st;
  void* kb = decompressed_k;
  void* vb = decompressed_v;
  if (!kb != !vb)
    return fail(MFA_ERR_INVALID_ARGUMENT,
                "MLA forward: pass both decompressed K and V buffers, or neither");
  if (!kb) {
    void* both = nullptr;
    if ((st = scratch((size_t)kv_elems * 2 * 2, &both, 1, s)) != MFA_SUCCESS) return st;
    kb = both;
    vb = (char*)both + kv_elems * 2;
  }
  // K = latent · W_k and V = latent · W_v in one launch (grid z = 2).
  mfa::GemmParams g;
  memset(&g, 0, sizeof(g));
  g.a = kv_latent;
  g.b[0] = w_k; g.b[1] = w_v;
  g.c[0] = kb; g.c[1] = vb;
  g.M = B * Skv; g.N = H * D; g.K = Lat;
  g.lda = Lat; g.ldb = H * D; g.ldc = H * D;
  g.prec_c = prec;
  if (B * Skv > 0) {
    st = hip_status(mfa::gemm_dispatch(g, prec, 2, s), "mfa_gemm (MLA decompress) launch");
    if (st != MFA_SUCCESS) return st;
  }
  if (Sq == 0) return MFA_SUCCESS;
  if ((st = check_keys(Sq, Skv)) != MFA_SUCCESS) return st;
  // Attention on BSHD K/V: element strides [S·H·D, D, H·D, 1].
  const int64_t kv_strides[4] = {(int64_t)Skv * H * D, D, (int64_t)H * D, 1};
  mfa::FwdParams p;
  memset(&p, 0, sizeof(p));
  p.q = make_operand(query, prec, B, H, Sq, D, nullptr, tq);
  p.k = make_operand(kb, prec, B, H, Skv, D, kv_strides, 0);
  p.v = make_operand(vb, prec, B, H, Skv, D, kv_strides, 0);
  p.o = output;
  out_strides(Sq, D, to, &p.o_ss, &p.o_sd);
  p.o_sh = (int64_t)Sq * D; p.o_sb = (int64_t)H * Sq * D;
  const Precisions pr = resolve_precisions(desc->base);
  p.l_f16 = pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  void* L = logsumexp;
  if (!L) {
    if ((st = scratch((size_t)B * H * Sq * 4, &L, 0, s)) != MFA_SUCCESS) return st;
  }
  p.l = L;
  p.B = B; p.H = H; p.Hkv = H; p.R = Sq; p.C = Skv; p.D = D;
  const int elem = elem_of(prec);
  int bq, bk, nw;
  mfa::fwd_block_config(elem, DP, &bq, &bk, &nw);
  p.nblk = (Sq + bq - 1) / bq;
  p.c_log2 = 1.442695041f * resolve_scale(desc->base, D);
  p.o_mul = 1.f;
  if ((st = plan_masks(desc->base, nullptr, Sq, Skv, &p.mask)) != MFA_SUCCESS) return st;
  return hip_status(launch_forward(p, elem, DP, 0, s), "mfa_fwd (MLA) launch");
}

// =========================================================================================
// Absorbed MLA: attention in the latent space, K/V never materialised.
// Q̃ = Q·W_kᵀ per head (general GEMM, B transposed), latent-space attention
// (attention_mla_latent.hip), O = Õ·W_v per head (16-bit GEMM).  Same result as
// mfa_mla_forward up to the rounding of Q̃ and Õ to the 16-bit precision (where the
// decompress path rounds K and V).
namespace {

// Key split of the latent attention: when the query blocks alone cannot fill the chip
// (decode shapes), aim at >= 512 workgroups, each split at least 4 tiles of 32 keys.
struct AbsorbedLayout {
  int nblk, nsplit, chunk;
  size_t qt_bytes;     // Q~ and O~, 16-bit, each
  size_t part_bytes;   // split-KV partial O (FP32) + (m, l) pairs, 0 without a split
  size_t total() const { return 2 * ((qt_bytes + 255) & ~(size_t)255) + part_bytes; }
};

AbsorbedLayout absorbed_layout(int B, int H, int Sq, int Skv, int Lat) {
  AbsorbedLayout a;
  const int R = H * Sq;
  a.nblk = (R + 31) / 32;
  a.nsplit = 1;
  a.chunk = Skv;
  const int blocks = a.nblk * B;
  const int tiles = (Skv + 31) / 32;
  int ns = (512 + blocks - 1) / blocks;
  ns = std::min(ns, std::max(1, tiles / 4));
  if (ns > 1) {
    const int per = (tiles + ns - 1) / ns;  // tiles per split
    a.chunk = per * 32;
    a.nsplit = (tiles + per - 1) / per;
  }
  a.qt_bytes = (size_t)B * R * Lat * 2;
  a.part_bytes = a.nsplit > 1 ? (size_t)B * a.nsplit * R * Lat * 4 + (size_t)B * a.nsplit * R * 8
                              : 0;
  return a;
}

}  // namespace

extern "C" size_t mfa_mla_absorbed_workspace_size(const mfa_mla_descriptor_t* desc) {
  if (!desc) return 0;
  return absorbed_layout((int)desc->batch_size, (int)desc->num_heads,
                         (int)desc->sequence_length_q, (int)desc->sequence_length_kv,
                         (int)desc->kv_latent_dim)
      .total();
}

extern "C" mfa_status_t mfa_mla_forward_absorbed(const mfa_mla_descriptor_t* desc,
                                                 const void* kv_latent, const void* w_k,
                                                 const void* w_v, const void* query,
                                                 void* workspace, float* output,
                                                 void* logsumexp, void* stream) {
  if (!desc || !kv_latent || !w_k || !w_v || !query || !output)
    return fail(MFA_ERR_INVALID_ARGUMENT, "MLA forward requires latent, weights, query, output");
  const int prec = desc->precision;
  if (prec != MFA_PRECISION_FP16 && prec != MFA_PRECISION_BF16)
    return fail(MFA_ERR_UNSUPPORTED, "MLA precision must be FP16 or BF16");
  const int B = (int)desc->batch_size, H = (int)desc->num_heads;
  const int Sq = (int)desc->sequence_length_q, Skv = (int)desc->sequence_length_kv;
  const int D = (int)desc->head_dim, Lat = (int)desc->kv_latent_dim;
  if (B <= 0 || H <= 0 || D <= 0 || Lat <= 0) return fail(MFA_ERR_INVALID_DESCRIPTOR, "empty MLA shape");
  if (Lat != 256 && Lat != 512)
    return fail(MFA_ERR_UNSUPPORTED, "absorbed MLA needs a latent dimension of 256 or 512 (got %d)", Lat);
  const int sp = desc->base.sparsity_pattern;
  if (sp != MFA_SPARSITY_NONE && sp != MFA_SPARSITY_CAUSAL)
    return fail(MFA_ERR_UNSUPPORTED, "absorbed MLA supports no mask or causal");
  mfa_status_t st0 = check_transposes(desc->base, false, "absorbed MLA forward");
  if (st0 != MFA_SUCCESS) return st0;
  if (Sq == 0) return MFA_SUCCESS;
  mfa_status_t st = check_keys(Sq, Skv);
  if (st != MFA_SUCCESS) return st;
  hipStream_t s = (hipStream_t)stream;
  // Q~, O~ and the split-KV partials, carved from the caller's workspace
  // (mfa_mla_absorbed_workspace_size bytes) or from this stream's scratch.
  const AbsorbedLayout al = absorbed_layout(B, H, Sq, Skv, Lat);
  void* ws = workspace;
  if (!ws && (st = scratch(al.total(), &ws, 2, s)) != MFA_SUCCESS) return st;
  char* qt = (char*)ws;
  char* ot = qt + ((al.qt_bytes + 255) & ~(size_t)255);
  char* part = ot + ((al.qt_bytes + 255) & ~(size_t)255);
  // One launch per GEMM over all (b, h): W_k / W_v slices depend on h only (bmod = H).
  auto general = [&](const void* a, const void* w, void* c, int M, int N, int K, int lda,
                     int ldc, int trans_b, int prec_c, int64_t sa, int64_t sc, int nbatch,
                     int bmod) {
    mfa::GemmGParams g;
    memset(&g, 0, sizeof(g));
    g.a = a; g.b = w; g.c = c;
    g.M = M; g.N = N; g.K = K;
    g.lda = lda; g.ldb = H * D; g.ldc = ldc;
    g.sa = sa; g.sb = D; g.sc = sc;
    g.prec_a = g.prec_b = prec; g.prec_c = prec_c;
    g.esz_a = g.esz_b = 2; g.esz_c = prec_c == MFA_PRECISION_FP32 ? 4 : 2;
    g.trans_b = trans_b;
    g.bmod = bmod;
    return hip_status(mfa::gemm_general_dispatch(g, nbatch, s), "absorbed MLA GEMM launch");
  };
  // Decode (S_q = 1): per head, the B query rows are one strided [B, D] matrix, so each head's
  // weight slice is read once (M = B) instead of once per batch item.
  const bool decode = Sq == 1 && B > 1;
  if (decode) {
    const hipError_t e = mfa::mla_qproj_dispatch(query, w_k, qt, B, H, D, Lat, elem_of(prec), s);
    if (e != hipErrorNotSupported) {
      if ((st = hip_status(e, "absorbed MLA query projection launch")) != MFA_SUCCESS) return st;
    } else if ((st = general(query, w_k, qt, B, Lat, D, H * D, H * Lat, 1, prec, D, Lat, H,
                             0)) != MFA_SUCCESS) {
      return st;
    }
  } else if (B > 1) {
    if ((st = general(query, w_k, qt, Sq, Lat, D, D, Lat, 1, prec, (int64_t)Sq * D,
                      (int64_t)Sq * Lat, B * H, H)) != MFA_SUCCESS)
      return st;
  }
  // Q̃[b,h] (Sq x Lat) = Q[b,h] (Sq x D) · W_k[:, hD:(h+1)D]ᵀ, batched over h.
  for (int b = 0; b < B && B == 1; ++b) {
    mfa_gemm_descriptor_t g;
    memset(&g, 0, sizeof(g));
    g.M = Sq; g.N = Lat; g.K = D;
    g.precision_a = g.precision_b = g.precision_c = prec;
    g.transpose_b = 1;
    g.lda = D; g.ldb = H * D; g.ldc = Lat;
    g.batch = H;
    g.stride_a = (uint64_t)Sq * D; g.stride_b = D; g.stride_c = (uint64_t)Sq * Lat;
    const char* qa = (const char*)query + (int64_t)b * H * Sq * D * 2;
    if ((st = mfa_gemm(&g, qa, w_k, qt + (int64_t)b * H * Sq * Lat * 2, stream)) != MFA_SUCCESS)
      return st;
  }
  // Latent-space attention.
  mfa::LatentParams lp;
  memset(&lp, 0, sizeof(lp));
  lp.q = qt; lp.lat = kv_latent; lp.olat = ot;
  const Precisions pr = resolve_precisions(desc->base);
  lp.l_f16 = pr.mem[MFA_OPERAND_L] == MFA_PRECISION_FP16;
  lp.l = logsumexp;
  lp.B = B; lp.R = H * Sq; lp.Sq = Sq; lp.Skv = Skv;
  lp.nblk = al.nblk;
  lp.c_log2 = 1.442695041f * resolve_scale(desc->base, D);
  lp.causal = sp == MFA_SPARSITY_CAUSAL;
  lp.nsplit = al.nsplit;
  lp.chunk = al.chunk;
  if (lp.nsplit > 1) {
    const size_t obytes = (size_t)B * lp.nsplit * lp.R * Lat * 4;
    lp.opart = (float*)part;
    lp.mlpart = (float2*)(part + obytes);
    // The merge pass applies W_v itself (FP32 Õ, one launch fewer).
    lp.wv = w_v;
    lp.out = output;
    lp.H = H;
    lp.D = D;
  }
  if ((st = hip_status(mfa::mla_latent_dispatch(lp, elem_of(prec), Lat, s),
                       "MLA latent attention launch")) != MFA_SUCCESS)
    return st;
  if (lp.wv) return MFA_SUCCESS;
  // O[b,h] (Sq x D, FP32) = Õ[b,h] (Sq x Lat) · W_v[:, hD:(h+1)D], batched over h.
  if (decode)
    return general(ot, w_v, output, B, D, Lat, H * Lat, H * D, 0, MFA_PRECISION_FP32, Lat, D, H,
                   0);
  if (B > 1)
    return general(ot, w_v, output, Sq, D, Lat, Lat, D, 0, MFA_PRECISION_FP32, (int64_t)Sq * Lat,
                   (int64_t)Sq * D, B * H, H);
  for (int b = 0; b < B; ++b) {
    mfa_gemm_descriptor_t g;
    memset(&g, 0, sizeof(g));
    g.M = Sq; g.N = D; g.K = Lat;
    g.precision_a = g.precision_b = prec;
    g.precision_c = MFA_PRECISION_FP32;
    g.lda = Lat; g.ldb = H * D; g.ldc = D;
    g.batch = H;
    g.stride_a = (uint64_t)Sq * Lat; g.stride_b = D; g.stride_c = (uint64_t)Sq * D;
    if ((st = mfa_gemm(&g, ot + (int64_t)b * H * Sq * Lat * 2, w_v,
                       output + (int64_t)b * H * Sq * D, stream)) != MFA_SUCCESS)
      return st;
  }
  return MFA_SUCCESS;
}
