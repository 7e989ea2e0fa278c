/*
 * mfa.h — C ABI of the MI355X (gfx950 / CDNA4) fused-attention library.
 *
 * This is the drop-in boundary for the hot path of bghira/metal-flash-attention-plus
 * (the reference; paths below are relative to its repository root).  Every entry point
 * cites the Swift interface it replaces.  The reference dispatches Metal command buffers;
 * here every launch enqueues onto a caller-provided hipStream_t (passed as void*) and
 * returns without synchronising, which is the analogue of encoding into a caller command
 * buffer (`MultiHeadAttention.encodeForward`, Sources/FlashAttention/Attention/
 * MultiHeadAttention.swift:197-234).
 *
 * Conventions (identical to the reference kernels):
 *   - All tensor pointers are DEVICE pointers owned by the caller (MTLBuffer analogue).
 *   - Logical layout is BHSD ([batch, heads, seq, head_dim]); strides are ELEMENT strides in
 *     BHSD order with the last dimension contiguous (MultiHeadAttention.swift:325-336).
 *   - O, dQ, dK, dV are FP32 in memory (AttentionDescriptor+Precisions.swift:143-146).
 *   - L (log-sum-exp) is stored in base-2 units premultiplied by log2(e):
 *     L = m + log2(l)  (AttentionKernel+Caching.swift:394-400); FP16 when
 *     low_precision_intermediates, else FP32.
 *   - D = softmax_scale * rowsum(dO ∘ O)  (AttentionKernel+Softmax.swift:233); BF16
 *     (upper 16 bits of the FP32 value) when low_precision_intermediates, else FP32.
 *   - GQA/MQA kv head = head % num_kv_heads (AttentionKernel+Source.swift:80-86).
 *
 * Errors: every function returns mfa_status_t; mfa_last_error() gives a thread-local
 * message.  The reference uses fatalError/precondition for invalid descriptors
 * (AttentionDescriptor.swift:95, AttentionKernel.swift:45, GEMMQuantization.swift:198-208)
 * and `nil`+print for pipeline failures (MultiHeadAttention.swift:44-47, :470-473).
 */
#ifndef MFA_MFA_H
#define MFA_MFA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MFA_ABI_VERSION 1

typedef enum mfa_status {
  MFA_SUCCESS = 0,
  MFA_ERR_INVALID_DESCRIPTOR = 1, /* fatalError("Descriptor was incomplete.") et al. */
  MFA_ERR_UNSUPPORTED = 2,        /* configuration the kernels do not implement */
  MFA_ERR_LAUNCH = 3,             /* hipLaunchKernel / runtime failure */
  MFA_ERR_INVALID_ARGUMENT = 4,   /* null pointer / bad size */
  MFA_ERR_NO_DEVICE = 5,
  /* Range sentinels (never valid values): the enum spans every int32, so a value a binding
     passes from outside the list is range-checked by the library instead of being
     undefined behaviour in C++. */
  MFA_STATUS_RANGE_MIN_ = -0x7fffffff - 1,
  MFA_STATUS_RANGE_MAX_ = 0x7fffffff
} mfa_status_t;

/* GEMMOperandPrecision (Sources/FlashAttention/GEMM/GEMMOperandPrecision.swift:22-27),
 * identical raw values. */
typedef enum mfa_precision {
  MFA_PRECISION_FP32 = 0,
  MFA_PRECISION_FP16 = 1,
  MFA_PRECISION_BF16 = 2,
  MFA_PRECISION_INT8 = 3,
  MFA_PRECISION_INT4 = 4,
  MFA_PRECISION_UNSET = -1, /* Swift `nil` for inputMemoryPrecision (resolves to FP16) */
  MFA_PRECISION_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_PRECISION_RANGE_MAX_ = 0x7fffffff
} mfa_precision_t;

/* AttentionKernelType (Attention/AttentionKernelType.swift:10-29). */
typedef enum mfa_kernel_type {
  MFA_KERNEL_FORWARD = 0,
  MFA_KERNEL_BACKWARD_QUERY = 1,
  MFA_KERNEL_BACKWARD_KEY_VALUE = 2,
  MFA_KERNEL_MLA_COMPRESSED = 3,
  MFA_KERNEL_TYPE_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_KERNEL_TYPE_RANGE_MAX_ = 0x7fffffff
} mfa_kernel_type_t;

/* AttentionOperand (Attention/AttentionOperand.swift:9-24); buffer slots of
 * AttentionOperand.bufferBinding (:50-67): Q0 K1 V2 O3 L4 D5 dO6 dV7 dK8 dQ9. */
typedef enum mfa_operand {
  MFA_OPERAND_Q = 0,
  MFA_OPERAND_K = 1,
  MFA_OPERAND_S = 2,
  MFA_OPERAND_P = 3,
  MFA_OPERAND_V = 4,
  MFA_OPERAND_O = 5,
  MFA_OPERAND_L = 6,
  MFA_OPERAND_D = 7,
  MFA_OPERAND_dO = 8,
  MFA_OPERAND_dV = 9,
  MFA_OPERAND_dP = 10,
  MFA_OPERAND_dS = 11,
  MFA_OPERAND_dK = 12,
  MFA_OPERAND_dQ = 13,
  MFA_OPERAND_COUNT = 14,
  MFA_OPERAND_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_OPERAND_RANGE_MAX_ = 0x7fffffff
} mfa_operand_t;

/* Returns the reference buffer slot of an operand, or -1 (AttentionOperand.swift:50-67). */
int mfa_operand_buffer_binding(mfa_operand_t operand);

/* SparsityPattern (AttentionDescriptor.swift:10-15). `custom` is accepted and treated as
 * none, exactly as AttentionDescriptor.setFunctionConstants does (:226-229). */
typedef enum mfa_sparsity {
  MFA_SPARSITY_NONE = 0,
  MFA_SPARSITY_CAUSAL = 1,
  MFA_SPARSITY_SLIDING_WINDOW = 2,
  MFA_SPARSITY_CUSTOM = 3,
  MFA_SPARSITY_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_SPARSITY_RANGE_MAX_ = 0x7fffffff
} mfa_sparsity_t;

/* SparseMaskDescriptor.MaskType (AttentionDescriptor.swift:47-51). */
typedef enum mfa_mask_type {
  MFA_MASK_DENSE = 0,         /* mask buffer = fp32 additive [B, H, R, C] added to QK^T */
  MFA_MASK_SPARSE_RANGES = 1, /* mask buffer = uint32x2 [B, H_kv, R] half-open key ranges */
  MFA_MASK_BLOCK_SPARSE = 2, /* flag only; ranges built by mfa_sparse_build_block_sparse */
  MFA_MASK_TYPE_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_MASK_TYPE_RANGE_MAX_ = 0x7fffffff
} mfa_mask_type_t;

/* AttentionDescriptor (AttentionDescriptor.swift:17-43). */
typedef struct mfa_attention_descriptor {
  int32_t low_precision_inputs;          /* Q, K, V, dO */
  int32_t input_memory_precision;        /* mfa_precision_t; MFA_PRECISION_UNSET = nil */
  int32_t low_precision_intermediates;   /* S, P, L, D, dP, dS */
  int32_t has_matrix_dimensions;         /* Optional matrixDimensions */
  uint32_t row;                          /* output sequence length R */
  uint32_t column;                       /* input sequence length C */
  uint16_t head;                         /* head dimension D */
  uint16_t reserved0;
  int32_t has_transpose_state;           /* Optional transposeState */
  int32_t transpose_q, transpose_k, transpose_v, transpose_o;
  int32_t sparsity_pattern;              /* mfa_sparsity_t */
  uint32_t window_size;                  /* slidingWindow(windowSize:) */
  int32_t has_softmax_scale;             /* Optional softmaxScale; default 1/sqrt(D) */
  float softmax_scale;
  int32_t has_sparse_mask;               /* Optional sparseMask */
  int32_t mask_type;                     /* mfa_mask_type_t */
  int32_t block_sparse_block_size;
  int32_t is_mqa;
  uint32_t num_kv_heads;
} mfa_attention_descriptor_t;

/* Fills the Swift default-initialised descriptor (AttentionDescriptor.init, :45). */
void mfa_attention_descriptor_init(mfa_attention_descriptor_t* desc);

/* AttentionKernelDescriptor (AttentionKernelDescriptor.swift:8-66). */
typedef struct mfa_kernel_descriptor {
  uint16_t block_parallelization;  /* blockDimensions.parallelization */
  uint16_t block_traversal;        /* blockDimensions.traversal */
  uint16_t block_head;             /* blockDimensions.head */
  uint16_t head_dimension;
  uint32_t sequence_length;        /* max(R, C) */
  int32_t cache_state[MFA_OPERAND_COUNT];          /* cached in registers? */
  int32_t memory_precisions[MFA_OPERAND_COUNT];    /* mfa_precision_t or -1 */
  int32_t register_precisions[MFA_OPERAND_COUNT];  /* mfa_precision_t or -1 */
  int32_t transpose_state[MFA_OPERAND_COUNT];
  int32_t prefer_async_cache;
  int32_t prefer_async_load;
  int32_t has_softmax_scale;
  float softmax_scale;
  int32_t type;                    /* mfa_kernel_type_t */
  int32_t masking_strategy_override; /* -1 none, 0 elementWise, 1 bitmask */
} mfa_kernel_descriptor_t;

/* AttentionDescriptor.kernelDescriptor(type:) (AttentionDescriptor.swift:80-190) with the
 * gfx950 parameter table in place of the Apple ones (AttentionDescriptor+Parameters.swift). */
mfa_status_t mfa_attention_kernel_descriptor(const mfa_attention_descriptor_t* desc,
                                             mfa_kernel_type_t type,
                                             mfa_kernel_descriptor_t* out);

/* AttentionKernel (AttentionKernel.swift:10-91): the compiled-plan view. `variant` is the
 * identifier of the HIP kernel instantiation that will run (createSource() has no HIP
 * meaning; this string replaces it for cache keys and logging). */
typedef struct mfa_attention_kernel {
  uint16_t block_parallelization;
  uint16_t block_traversal;
  uint16_t block_head;
  uint16_t threadgroup_size;                /* threads per workgroup (multiple of 64) */
  uint32_t threadgroup_memory_allocation;   /* LDS bytes per workgroup */
  float softmax_scale;
  int32_t type;
  char variant[96];
} mfa_attention_kernel_t;

mfa_status_t mfa_attention_kernel_create(const mfa_kernel_descriptor_t* kdesc,
                                         mfa_attention_kernel_t* out);

/* MultiHeadShape (MultiHeadAttentionDescriptor.swift:11-40). */
typedef struct mfa_multihead_shape {
  uint32_t batch_size;
  uint32_t num_heads;
  uint32_t sequence_length;
  uint16_t head_dimension;
  uint16_t reserved0;
} mfa_multihead_shape_t;

/* MultiHeadBroadcastMode (MultiHeadAttentionDescriptor.swift:43-109). */
typedef enum mfa_broadcast_mode {
  MFA_BROADCAST_STANDARD = 0,
  MFA_BROADCAST_GROUPED_QUERY = 1,
  MFA_BROADCAST_MULTI_QUERY = 2,
  MFA_BROADCAST_CROSS_ATTENTION = 3,
  MFA_BROADCAST_CUSTOM = 4,
  MFA_BROADCAST_MODE_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_BROADCAST_MODE_RANGE_MAX_ = 0x7fffffff
} mfa_broadcast_mode_t;

/* MultiHeadDispatchStrategy (MultiHeadAttentionDescriptor.swift:121-159). All strategies
 * run the batched 3-D grid here (the reference's perBatchHead binds its slots wrongly,
 * SURVEY.md §8a quirk 1). */
typedef enum mfa_dispatch_strategy {
  MFA_DISPATCH_PER_BATCH_HEAD = 0,
  MFA_DISPATCH_PER_BATCH = 1,
  MFA_DISPATCH_BATCHED = 2,
  MFA_DISPATCH_AUTO = 3,
  MFA_DISPATCH_STRATEGY_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_DISPATCH_STRATEGY_RANGE_MAX_ = 0x7fffffff
} mfa_dispatch_strategy_t;

/* MultiHeadAttentionDescriptor (MultiHeadAttentionDescriptor.swift:162-214). */
typedef struct mfa_multihead_descriptor {
  mfa_attention_descriptor_t base;
  mfa_multihead_shape_t query_shape;
  mfa_multihead_shape_t key_shape;
  mfa_multihead_shape_t value_shape;
  int32_t broadcast_mode;     /* mfa_broadcast_mode_t */
  uint32_t broadcast_param;   /* numKVHeads (groupedQuery) or kvSequenceLength (cross) */
  int32_t dispatch_strategy;  /* mfa_dispatch_strategy_t */
} mfa_multihead_descriptor_t;

/* MultiHeadBroadcastMode.isCompatible (MultiHeadAttentionDescriptor.swift:60-107). */
int mfa_multihead_broadcast_compatible(const mfa_multihead_descriptor_t* desc);

/* Buffers in reference slot order (AttentionOperand.bufferBinding) plus the strides
 * (slots 5-7 / 10-12 / 9-11) and the mask (slot 12 / 17 / 16).  Strides are HOST arrays
 * of 4 element strides in BHSD order (setBytes in the reference); NULL = contiguous. */
typedef struct mfa_attention_buffers {
  const void* Q;   /* slot 0 */
  const void* K;   /* slot 1 */
  const void* V;   /* slot 2 */
  void* O;         /* slot 3, fp32 dense [B, H, R, D] */
  void* L;         /* slot 4, [B, H, R]; may be NULL in forward (scratch allocated) */
  void* D;         /* slot 5, [B, H, R] */
  const void* dO;  /* slot 6 */
  void* dV;        /* slot 7, fp32 [B, H_kv, C, D] */
  void* dK;        /* slot 8, fp32 [B, H_kv, C, D] */
  void* dQ;        /* slot 9, fp32 [B, H, R, D] */
  const int64_t* Q_strides;
  const int64_t* K_strides;
  const int64_t* V_strides;
  const void* mask;  /* device pointer; meaning set by base.sparse_mask.mask_type */
} mfa_attention_buffers_t;

/* MultiHeadAttention.forward / encodeForward (MultiHeadAttention.swift:33-83, :197-234,
 * dispatchBatched :255-384): grid (ceil(R/Bp), H, B), writes O and L. */
mfa_status_t mfa_multihead_forward(const mfa_multihead_descriptor_t* desc,
                                   const mfa_attention_buffers_t* buffers, void* stream);

/* MultiHeadAttention.backward (MultiHeadAttention.swift:574-707): backwardQuery (D, dQ)
 * then backwardKeyValue (dK, dV) on the same stream.  Requires Q K V O L dO D dQ dK dV. */
mfa_status_t mfa_multihead_backward(const mfa_multihead_descriptor_t* desc,
                                    const mfa_attention_buffers_t* buffers, void* stream);
/* The two phases separately (AttentionKernelType.backwardQuery / .backwardKeyValue). */
mfa_status_t mfa_multihead_backward_query(const mfa_multihead_descriptor_t* desc,
                                          const mfa_attention_buffers_t* buffers,
                                          void* stream);
mfa_status_t mfa_multihead_backward_key_value(const mfa_multihead_descriptor_t* desc,
                                              const mfa_attention_buffers_t* buffers,
                                              void* stream);

/* Plan query: the kernels a call launches.  Runs the dispatcher of the call `type` names
 * (FORWARD = mfa_multihead_forward, BACKWARD_QUERY / BACKWARD_KEY_VALUE = the two backward
 * phases) with every launch recorded instead of issued, so the record is by construction
 * what that call launches for these shapes, environment overrides and — when `buffers` is
 * given — these pointers' alignment and strides (NULL: contiguous 256-byte aligned buffers).
 * Nothing is read, written or allocated on the device; no GPU is needed.  Replaces the
 * pipeline-state lookup of AttentionKernel / MultiHeadAttention.createPipeline
 * (MultiHeadAttention.swift:386-430) as the place callers learn the kernel. */
typedef struct mfa_kernel_launch {
  char name[96];          /* kernel instantiation, e.g. "mfa_fwd2_pair_kernel<f16,D128,BK64,NWG2>" */
  uint32_t threads;       /* workgroup size */
  uint32_t lds_bytes;     /* dynamic LDS per workgroup */
  uint64_t workgroups;    /* grid size */
} mfa_kernel_launch_t;

typedef struct mfa_kernel_plan {
  int32_t count;          /* launches recorded in `launches`, in issue order (0 for empty shapes) */
  int32_t total;          /* launches the call issues; total > count means the record holds
                           * only the first (plan) or last (launch log) four of them */
  mfa_kernel_launch_t launches[4];
} mfa_kernel_plan_t;

mfa_status_t mfa_multihead_plan(const mfa_multihead_descriptor_t* desc, mfa_kernel_type_t type,
                                const mfa_attention_buffers_t* buffers, mfa_kernel_plan_t* out);

/* The launches this host thread issued through the library since the previous call (the
 * last four, in issue order, named like a plan), then clears the record.  Returns how many
 * launches there were.  Lets a caller check that what ran is what the plan said. */
int mfa_last_launches(mfa_kernel_plan_t* out);

/* ---------------------------------------------------------------------------------- */
/* Quantization (Sources/FlashAttention/GEMM/GEMMQuantization.swift).                  */

/* QuantizationMode (GEMMQuantization.swift:27-42). */
typedef enum mfa_quantization_mode {
  MFA_QUANT_TENSOR_WISE = 0,
  MFA_QUANT_BLOCKWISE = 1,
  MFA_QUANT_ROW_WISE = 2,
  MFA_QUANTIZATION_MODE_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_QUANTIZATION_MODE_RANGE_MAX_ = 0x7fffffff
} mfa_quantization_mode_t;

/* QuantizationStrategy (GEMMQuantization.swift:45-55). */
typedef enum mfa_quantization_strategy {
  MFA_QUANT_STRATEGY_LEGACY = 0,
  MFA_QUANT_STRATEGY_ASYMMETRIC = 1,
  MFA_QUANT_STRATEGY_SYMMETRIC = 2,
  MFA_QUANTIZATION_STRATEGY_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_QUANTIZATION_STRATEGY_RANGE_MAX_ = 0x7fffffff
} mfa_quantization_strategy_t;

/* A QuantizedTensor (GEMMQuantization.swift:681-700) as the kernels consume it.
 * For FP16/BF16/FP32 precisions the quantization fields are ignored. `data` is a device
 * pointer to the contiguous [B, H, S, D] tensor (INT4: two values per byte, element 2i in
 * the low nibble of byte i, GEMMQuantization.swift:500-515).  Blockwise scales are
 * device arrays indexed (row / bs) * ceil(cols / bs) + col / bs over the tensor's 2-D memory
 * view (GEMMQuantization.swift:561-575): [B*H*S rows, D cols] for a row-major operand, and
 * [B*H*D rows, S cols] for one the descriptor's transposeState marks transposed (row = head
 * dimension index, col = sequence index, as AttentionKernel+Accumulate.swift:461-472 and
 * AttentionKernel+OuterProduct.swift:301-316 index it). */
typedef struct mfa_quantized_tensor {
  const void* data;
  int32_t precision;           /* mfa_precision_t */
  float scale;                 /* per-tensor */
  int32_t zero_point;          /* per-tensor */
  const float* block_scales;   /* device, NULL unless blockwise */
  const int32_t* block_zero_points; /* device, NULL unless blockwise */
  uint32_t block_size;         /* blockSizeK */
} mfa_quantized_tensor_t;

/* QuantizedAttention.Configuration (QuantizedAttention.swift:12-41). */
typedef struct mfa_quantized_configuration {
  int32_t query_precision;  /* default FP16 */
  int32_t key_precision;    /* default INT8 */
  int32_t value_precision;  /* default INT8 */
  int32_t query_strategy, key_strategy, value_strategy;
  uint8_t strategy_version;
  /* Extension (no reference counterpart): 1 = INT8 K/V run on the integer matrix cores
   * (Q quantised per row in-kernel, P quantised to INT8; approximate).
   * 0 (default) = dequantise-exact, the reference's FP32-multiply semantics. */
  uint8_t integer_matmul;
  uint8_t reserved[2];
  int32_t mixed_precision_intermediates;
} mfa_quantized_configuration_t;

void mfa_quantized_configuration_init(mfa_quantized_configuration_t* cfg);

/* QuantizedAttention.QuantizedAttentionDescriptor (QuantizedAttention.swift:58-92) extended
 * with the multi-head shape the reference expresses through byte offsets. */
typedef struct mfa_quantized_descriptor {
  mfa_attention_descriptor_t base;
  mfa_quantized_configuration_t config;
  uint32_t batch_size;
  uint32_t num_heads;
  uint32_t num_kv_heads;
  uint32_t reserved0;
} mfa_quantized_descriptor_t;

/* QuantizedAttention.forward(query:key:value:output:descriptor:...) (:135-263). O fp32,
 * L base-2 (nullable).  `mask` is the dense fp32 additive mask or NULL. */
mfa_status_t mfa_quantized_forward(const mfa_quantized_descriptor_t* desc,
                                   const mfa_quantized_tensor_t* query,
                                   const mfa_quantized_tensor_t* key,
                                   const mfa_quantized_tensor_t* value, float* output,
                                   void* logsumexp, const void* mask, void* stream);

/* QuantizedAttention.forward(queryBuffer:keyBuffer:valueBuffer:output:queryShape:keyShape:
 * valueShape:queryPrecision:keyPrecision:valuePrecision:targetQuantization:quantizationMode:
 * descriptor:) (QuantizedAttention.swift:278-336; the uniform-settings overload :349-372 is this
 * call with one precision for all three).  Q, K and V arrive as FP32 / FP16 / BF16 device
 * tensors ([B, H, R, D], [B, H_kv, C, D], dense, shapes from the descriptor) and are quantized
 * on the GPU (mfa_quantize) to `target_precision` in `mode` (tensor-wise or blockwise with
 * `block_size`) into library scratch on `stream`, then run through mfa_quantized_forward with
 * the configuration's precisions replaced by the target for all three operands (every tensor
 * handed to that forward is then target-quantized, as in the reference).  A target that needs
 * no quantization parameters (FP16 / BF16 / FP32) wraps the buffers as they are (:425-441).
 * Tensor-wise scales are read back to the host before the forward (one synchronisation of
 * `stream`; the reference computes them on the CPU, :479-498), so tensor-wise mode on a stream
 * under graph capture returns MFA_ERR_UNSUPPORTED; blockwise scales stay on the device and the
 * call stays asynchronous.  Each buffer is quantised as its memory view (transposed operands
 * as [D][S] rows, see mfa_quantized_tensor_t).  Row-wise mode is not an attention input
 * layout: MFA_ERR_UNSUPPORTED. */
mfa_status_t mfa_quantized_forward_from_float(const mfa_quantized_descriptor_t* desc,
                                              const void* query, const void* key,
                                              const void* value, int32_t query_precision,
                                              int32_t key_precision, int32_t value_precision,
                                              int32_t target_precision, int32_t mode,
                                              uint32_t block_size, float* output,
                                              void* logsumexp, const void* mask, void* stream);

/* QuantizedAttention.backwardQuery (:1012-1097) and backwardKeyValue (:1102-1181).
 * dO/L/D/O use the base descriptor's memory precisions (FP32 unless low precision). */
mfa_status_t mfa_quantized_backward_query(const mfa_quantized_descriptor_t* desc,
                                          const mfa_quantized_tensor_t* query,
                                          const mfa_quantized_tensor_t* key,
                                          const mfa_quantized_tensor_t* value,
                                          const float* output, const void* grad_output,
                                          const void* logsumexp, float* grad_query,
                                          void* d_values, void* stream);
mfa_status_t mfa_quantized_backward_key_value(const mfa_quantized_descriptor_t* desc,
                                              const mfa_quantized_tensor_t* query,
                                              const mfa_quantized_tensor_t* key,
                                              const mfa_quantized_tensor_t* value,
                                              const void* grad_output, const void* logsumexp,
                                              const void* d_values, float* grad_key,
                                              float* grad_value, void* stream);

/* QuantizedKernelLayoutManifest (Attention/QuantizedKernelLayoutManifest.swift:8-266): the
 * buffer slot of every quantized-attention operand per kernel type, the reference FFI's
 * binding contract.  Keys in declaration order (Key, :16-56). */
typedef enum mfa_quantized_slot_key {
  MFA_QSLOT_Q_DATA = 0, MFA_QSLOT_K_DATA, MFA_QSLOT_V_DATA, MFA_QSLOT_OUTPUT,
  MFA_QSLOT_GRAD_OUTPUT, MFA_QSLOT_LOGSUMEXP, MFA_QSLOT_GRAD_QUERY, MFA_QSLOT_D_VALUES,
  MFA_QSLOT_GRAD_KEY, MFA_QSLOT_GRAD_VALUE, MFA_QSLOT_Q_SCALE, MFA_QSLOT_Q_ZERO_POINT,
  MFA_QSLOT_K_SCALE, MFA_QSLOT_K_ZERO_POINT, MFA_QSLOT_V_SCALE, MFA_QSLOT_V_ZERO_POINT,
  MFA_QSLOT_DIMS, MFA_QSLOT_STE_CLIP_RANGE, MFA_QSLOT_Q_BLOCK_SCALES,
  MFA_QSLOT_Q_BLOCK_ZERO_POINTS, MFA_QSLOT_K_BLOCK_SCALES, MFA_QSLOT_K_BLOCK_ZERO_POINTS,
  MFA_QSLOT_V_BLOCK_SCALES, MFA_QSLOT_V_BLOCK_ZERO_POINTS, MFA_QSLOT_Q_PRECOMPUTED_SUMS,
  MFA_QSLOT_K_PRECOMPUTED_SUMS, MFA_QSLOT_V_PRECOMPUTED_SUMS, MFA_QSLOT_Q_STRIDES,
  MFA_QSLOT_K_STRIDES, MFA_QSLOT_V_STRIDES, MFA_QSLOT_O_STRIDES, MFA_QSLOT_MASK_BUFFER,
  MFA_QSLOT_MASK_METADATA, MFA_QSLOT_NUM_HEADS, MFA_QSLOT_NUM_KEY_VALUE_HEADS,
  MFA_QSLOT_HEAD_DIMENSION, MFA_QSLOT_SEQUENCE_LENGTH, MFA_QSLOT_SCRATCH0, MFA_QSLOT_SCRATCH1,
  MFA_QSLOT_COUNT,
  MFA_QUANTIZED_SLOT_KEY_RANGE_MIN_ = -0x7fffffff - 1, /* range sentinel (see mfa_status) */
  MFA_QUANTIZED_SLOT_KEY_RANGE_MAX_ = 0x7fffffff
} mfa_quantized_slot_key_t;

/* Layout.index(key) of QuantizedKernelLayoutManifest.layout(for: kernel): the slot, or -1
 * when that kernel's layout does not bind the key. */
int mfa_quantized_slot(mfa_kernel_type_t kernel, mfa_quantized_slot_key_t key);
/* The whole layout: out[key] = mfa_quantized_slot(kernel, key) for key < min(n,
 * MFA_QSLOT_COUNT).  Returns how many keys have a slot, or -1 for an unknown kernel. */
int mfa_quantized_slot_table(mfa_kernel_type_t kernel, int32_t* out, int n);
/* Key.rawValue ("qData", ..., "scratch1"), NULL when out of range. */
const char* mfa_quantized_slot_name(mfa_quantized_slot_key_t key);

/* GLUON constants (AttentionKernel+GluonOptimizations.swift:12-22) and the predicate that
 * gates the GLUON softmax (:314-320, block traversal >= 512 and block head >= 64).  No
 * parameter table produces such a block, here or in the reference, so the standard
 * softmax always runs. */
#define MFA_GLUON_SPLIT_EXP_FACTOR 4
#define MFA_GLUON_CHANNEL_SYNC_POINTS 2
#define MFA_GLUON_SUBTILE_SIZE 16
void mfa_gluon_constants(uint8_t* split_exp_factor, uint8_t* channel_sync_points,
                         uint8_t* subtile_size);
int mfa_gluon_should_enable(uint16_t block_traversal, uint16_t block_head);

/* Plan query for the quantized calls (see mfa_multihead_plan): FORWARD =
 * mfa_quantized_forward, BACKWARD_QUERY / BACKWARD_KEY_VALUE = the backward phases.  The
 * tensors supply data pointers, scales and block layouts; NULL tensors plan per-tensor
 * scale 1, zero point 0, aligned contiguous data. */
mfa_status_t mfa_quantized_plan(const mfa_quantized_descriptor_t* desc, mfa_kernel_type_t type,
                                const mfa_quantized_tensor_t* query,
                                const mfa_quantized_tensor_t* key,
                                const mfa_quantized_tensor_t* value, mfa_kernel_plan_t* out);

/* GPU runtime quantization (GEMMQuantization.swift:305-623 semantics, bit-exact; the
 * reference does this on the CPU in QuantizedTensor.from, :720-860).
 * input: device tensor of `count` elements in `input_precision` (FP32/FP16/BF16), viewed as
 * 2-D [rows, cols] for blockwise/row-wise.  Writes `output` (INT8 bytes or packed INT4),
 * and the parameters: `scale_out` (device float[1]) for tensor-wise, `block_scales_out` /
 * `block_zero_points_out` (device arrays) for blockwise / row-wise.  `workspace` must hold
 * mfa_quantize_workspace_size() bytes. */
size_t mfa_quantize_workspace_size(uint64_t count, uint32_t rows, uint32_t cols,
                                   int32_t mode, uint32_t block_size);
mfa_status_t mfa_quantize(const void* input, int32_t input_precision, uint64_t count,
                          uint32_t rows, uint32_t cols, int32_t target_precision,
                          int32_t mode, uint32_t block_size, void* output, float* scale_out,
                          float* block_scales_out, int32_t* block_zero_points_out,
                          void* workspace, void* stream);
/* Dequantize (GEMMQuantization.swift:529-558 / :629-676) to FP32. */
mfa_status_t mfa_dequantize(const mfa_quantized_tensor_t* tensor, uint64_t count,
                            uint32_t cols, float* output, void* stream);

/* ---------------------------------------------------------------------------------- */
/* GEMM + MLA (Sources/FlashAttention/GEMM/GEMMDescriptor.swift, Attention/            */
/* MLAOptimizedGEMMMFA.swift).                                                          */

/* GEMMDescriptor (GEMMDescriptor.swift:11-47): C[M,N] = op(A)·op(B) (+ C when
 * load_previous_c, GEMMDescriptor.swift:400).  Row-major.  A is [M][K], or [K][M] when
 * transpose_a; B is [K][N], or [N][K] when transpose_b (GEMMDescriptor.swift:344-372).
 * Leading dimensions default to the packed ones (0) and must not be smaller than them
 * ("Leading block dimension was too small.", :359).  Memory precisions FP32 / FP16 / BF16,
 * chosen independently per operand (AdversarialShapeTest.swift:14-40). */
typedef struct mfa_gemm_descriptor {
  uint32_t M, N, K;
  int32_t precision_a, precision_b, precision_c; /* mfa_precision_t: FP32 / FP16 / BF16 */
  int32_t transpose_a, transpose_b;
  int32_t load_previous_c;
  uint32_t lda, ldb, ldc;                        /* 0 = packed */
  uint32_t batch;                                /* independent GEMMs (grid z) */
  uint64_t stride_a, stride_b, stride_c;         /* element strides between batch items */
} mfa_gemm_descriptor_t;

mfa_status_t mfa_gemm(const mfa_gemm_descriptor_t* desc, const void* A, const void* B,
                      void* C, void* stream);

/* GEMMKernelDescriptor(descriptor:) + GEMMKernel (GEMMKernelDescriptor.swift:8-60,
 * GEMMDescriptor.swift:110-246, GEMMKernel.swift): the plan mfa_gemm will run.  Register
 * precisions follow the gfx950 policy: A and B of one 16-bit type multiply on the 16-bit
 * matrix core, every other mix in FP32; C always accumulates in FP32 (the reference keeps
 * FP16 x FP16 -> FP16 in FP16 registers, GEMMDescriptor.swift:204-210). */
typedef struct mfa_gemm_kernel_descriptor {
  uint16_t block_m, block_n, block_k;
  uint16_t splits_m, splits_n;            /* waves along M and N */
  int32_t memory_precisions[3];           /* A, B, C */
  int32_t register_precisions[3];         /* A, B, C */
  int32_t transpose_a, transpose_b;
  int32_t load_previous_c;
  uint32_t lda, ldb, ldc;                 /* resolved leading dimensions */
  uint32_t threadgroup_size;
  uint32_t threadgroup_memory_allocation; /* LDS bytes per workgroup */
  uint32_t grid_x, grid_y, grid_z;        /* workgroups along N, M, batch */
  char variant[64];
} mfa_gemm_kernel_descriptor_t;

mfa_status_t mfa_gemm_kernel_descriptor(const mfa_gemm_descriptor_t* desc,
                                        mfa_gemm_kernel_descriptor_t* out);

/* MLAOptimizedGEMMMFA.forward (MLAOptimizedGEMMMFA.swift:158-240) followed by the
 * attention forward the reference's caller runs on the decompressed BSHD K/V
 * (KernelRegressionTests.swift:398-465 stride pattern).
 *   kv_latent [B*S_kv, latent_dim], w_k / w_v [latent_dim, H*D] (precision FP16/BF16),
 *   query BHSD [B, H, S_q, D] in the same precision, K/V scratch [B*S_kv, H*D] (caller
 *   provided or NULL → library-owned), output fp32 [B, H, S_q, D], L nullable. */
typedef struct mfa_mla_descriptor {
  mfa_attention_descriptor_t base; /* precision / sparsity / scale of the attention */
  uint32_t batch_size;
  uint32_t num_heads;
  uint32_t sequence_length_q;
  uint32_t sequence_length_kv;
  uint32_t head_dim;
  uint32_t kv_latent_dim;
  int32_t precision;                /* FP16 or BF16 for latent / weights / Q / K / V */
} mfa_mla_descriptor_t;

mfa_status_t mfa_mla_forward(const mfa_mla_descriptor_t* desc, const void* kv_latent,
                             const void* w_k, const void* w_v, const void* query,
                             void* decompressed_k, void* decompressed_v, float* output,
                             void* logsumexp, void* stream);

/* Absorbed MLA (the fused form of MLAOptimizedGEMMMFA.forward,
 * MLAOptimizedGEMMMFA.swift:213-239): attends in the latent space instead of materialising
 * K/V — Q̃_h = Q_h·W_k,hᵀ, Õ_h = softmax(scale·Q̃_h·latentᵀ)·latent, O_h = Õ_h·W_v,h — with
 * scale = softmax_scale of the base descriptor or 1/sqrt(head_dim).  Same arguments and
 * layouts as mfa_mla_forward; kv_latent_dim must be 256 or 512; masks: none or causal.
 * `workspace` (nullable → library-owned) holds Q̃, Õ and, for decode shapes, the split-KV
 * partials: mfa_mla_absorbed_workspace_size() bytes.  Library-owned buffers (here, the
 * decompressed K/V of mfa_mla_forward and a forward's NULL L) are kept per device and per
 * stream, so concurrent calls on different streams never share one. */
size_t mfa_mla_absorbed_workspace_size(const mfa_mla_descriptor_t* desc);
mfa_status_t mfa_mla_forward_absorbed(const mfa_mla_descriptor_t* desc, const void* kv_latent,
                                      const void* w_k, const void* w_v, const void* query,
                                      void* workspace, float* output, void* logsumexp,
                                      void* stream);

/* ---------------------------------------------------------------------------------- */
/* HadamardRotation (Sources/FlashAttention/Attention/HadamardRotation.swift).           */

/* rotate(buffer:blockSize:numBlocks:) (:43-88): in-place FWHT of every block of an FP32
 * buffer [num_blocks][block_size] (power of two, <= 1024; buffer 16-byte aligned when
 * block_size >= 4), then x *= mfa_hadamard_scale(block_size).  Enqueued on `stream`. */
mfa_status_t mfa_hadamard_rotate(float* buffer, uint32_t block_size, uint32_t num_blocks,
                                 void* stream);

/* rotateBatch(buffers:) (:91-109): every item validated first, then enqueued in order. */
typedef struct mfa_hadamard_item {
  float* buffer;
  uint32_t block_size;
  uint32_t num_blocks;
} mfa_hadamard_item_t;
mfa_status_t mfa_hadamard_rotate_batch(const mfa_hadamard_item_t* items, uint32_t count,
                                       void* stream);

/* The normalisation factor: FP32 1/sqrt(block_size), correctly rounded (the reference's
 * Metal rsqrt, :132, is exact for powers of 4; for odd powers of two its rounding is not
 * specified). */
float mfa_hadamard_scale(uint32_t block_size);

/* ---------------------------------------------------------------------------------- */
/* Host utilities mirrored from the reference.                                          */

/* MaskingStrategyHeuristic.sequenceBucket / defaultRule (MaskingStrategyHeuristic.swift:
 * 47-60, :111-136).  Returns 0 = elementWise, 1 = bitmask.  The two strategies are
 * numerically identical; on gfx950 the predicate is evaluated per element either way. */
int mfa_masking_sequence_bucket(int sequence_length);
int mfa_masking_default_rule(int sequence_length, int head_dimension);

/* SparseMQABuilder (Attention/SparseMQABuilder.swift:4-62), host arrays of uint32 pairs. */
void mfa_sparse_build_sliding_window(uint32_t sequence_length, uint32_t window_size,
                                     uint32_t* ranges_out);
void mfa_sparse_build_block_sparse(const uint8_t* pattern, uint32_t rows, uint32_t cols,
                                   uint32_t block_size, uint32_t* ranges_out);

/* Version / error / device utilities. */
const char* mfa_version(void);
const char* mfa_last_error(void);
int mfa_abi_version(void);

/* Releases the library scratch (L when the caller passes none, MLA / dequantisation buffers)
 * held for `stream` on the current device, stream-ordered (hipFreeAsync on that stream);
 * stream == NULL releases every stream's scratch on the current device.  A caller that
 * creates short-lived streams calls this before destroying one.  Returns the number of
 * buffers released.  (No reference counterpart: Metal buffers are reference-counted.) */
int mfa_release_scratch(void* stream);

/* Diagnostics: (kernel, device) pairs whose dynamic-LDS attribute the library has set. */
int mfa_kernel_attribute_count(void);

#ifdef __cplusplus
}
#endif

#endif /* MFA_MFA_H */
