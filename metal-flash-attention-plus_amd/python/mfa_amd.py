"""ctypes binding of libmfa_amd.so (include/mfa/mfa.h).

This is the binding a maintainer would add on the caller side of the C ABI (the reference's
production caller is an out-of-repo C++/PyTorch bridge, QuantizedAttention.swift:1552-1555).
It mirrors the reference's Swift surface — AttentionDescriptor, MultiHeadAttentionDescriptor,
MultiHeadAttention.forward/backward, QuantizedAttention, MLAOptimizedGEMMMFA — with device
memory supplied as torch tensors (PyTorch is only plumbing here: allocation + streams).

The library is REQUIRED: importing this module on a machine where libmfa_amd.so is missing
raises immediately; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import enum
import math
import os
import re
from typing import Optional, Sequence

_HERE = os.path.dirname(os.path.abspath(__file__))
_PKG = os.path.dirname(_HERE)
_REPO = os.path.dirname(_PKG)
LIB_PATH = os.environ.get("MFA_LIB", os.path.join(_PKG, "libmfa_amd.so"))
HEADER_PATH = os.path.join(_REPO, "include", "mfa", "mfa.h")


class MFAError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"mfa status {status}: {message}")
        self.status = status


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libmfa_amd.so not built: {LIB_PATH} (run __graft_entry__.build())")
    return ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)


lib = _load()


class Precision(enum.IntEnum):  # GEMMOperandPrecision.swift:22-27
    FP32 = 0
    FP16 = 1
    BF16 = 2
    INT8 = 3
    INT4 = 4
    UNSET = -1


class KernelType(enum.IntEnum):  # AttentionKernelType.swift:10-29
    forward = 0
    backwardQuery = 1
    backwardKeyValue = 2
    mlaCompressed = 3


class Operand(enum.IntEnum):  # AttentionOperand.swift:9-24
    Q = 0
    K = 1
    S = 2
    P = 3
    V = 4
    O = 5
    L = 6
    D = 7
    dO = 8
    dV = 9
    dP = 10
    dS = 11
    dK = 12
    dQ = 13


class Sparsity(enum.IntEnum):
    none = 0
    causal = 1
    slidingWindow = 2
    custom = 3


class MaskType(enum.IntEnum):
    dense = 0
    sparseRanges = 1
    blockSparse = 2


class Broadcast(enum.IntEnum):
    standard = 0
    groupedQuery = 1
    multiQuery = 2
    crossAttention = 3
    custom = 4


class QuantMode(enum.IntEnum):
    tensorWise = 0
    blockwise = 1
    rowWise = 2


OPERAND_COUNT = 14


class AttentionDescriptor(ctypes.Structure):
    _fields_ = [
        ("low_precision_inputs", ctypes.c_int32),
        ("input_memory_precision", ctypes.c_int32),
        ("low_precision_intermediates", ctypes.c_int32),
        ("has_matrix_dimensions", ctypes.c_int32),
        ("row", ctypes.c_uint32),
        ("column", ctypes.c_uint32),
        ("head", ctypes.c_uint16),
        ("reserved0", ctypes.c_uint16),
        ("has_transpose_state", ctypes.c_int32),
        ("transpose_q", ctypes.c_int32),
        ("transpose_k", ctypes.c_int32),
        ("transpose_v", ctypes.c_int32),
        ("transpose_o", ctypes.c_int32),
        ("sparsity_pattern", ctypes.c_int32),
        ("window_size", ctypes.c_uint32),
        ("has_softmax_scale", ctypes.c_int32),
        ("softmax_scale", ctypes.c_float),
        ("has_sparse_mask", ctypes.c_int32),
        ("mask_type", ctypes.c_int32),
        ("block_sparse_block_size", ctypes.c_int32),
        ("is_mqa", ctypes.c_int32),
        ("num_kv_heads", ctypes.c_uint32),
    ]

    @classmethod
    def make(cls, row=None, column=None, head=None, low_precision=False, precision=None,
             low_precision_intermediates=None, causal=False, window=None, scale=None,
             transpose=(False, False, False, False), sparse_mask: Optional[int] = None):
        d = cls()
        lib.mfa_attention_descriptor_init(ctypes.byref(d))
        if row is not None:
            d.has_matrix_dimensions = 1
            d.row, d.column, d.head = row, column, head
        d.has_transpose_state = 1
        d.transpose_q, d.transpose_k, d.transpose_v, d.transpose_o = [int(t) for t in transpose]
        d.low_precision_inputs = int(low_precision)
        d.low_precision_intermediates = int(
            low_precision if low_precision_intermediates is None else low_precision_intermediates)
        if precision is not None:
            d.input_memory_precision = int(precision)
        if causal:
            d.sparsity_pattern = Sparsity.causal
        if window is not None:
            d.sparsity_pattern = Sparsity.slidingWindow
            d.window_size = window
        if scale is not None:
            d.has_softmax_scale = 1
            d.softmax_scale = scale
        if sparse_mask is not None:
            d.has_sparse_mask = 1
            d.mask_type = int(sparse_mask)
        return d


class KernelDescriptor(ctypes.Structure):
    _fields_ = [
        ("block_parallelization", ctypes.c_uint16),
        ("block_traversal", ctypes.c_uint16),
        ("block_head", ctypes.c_uint16),
        ("head_dimension", ctypes.c_uint16),
        ("sequence_length", ctypes.c_uint32),
        ("cache_state", ctypes.c_int32 * OPERAND_COUNT),
        ("memory_precisions", ctypes.c_int32 * OPERAND_COUNT),
        ("register_precisions", ctypes.c_int32 * OPERAND_COUNT),
        ("transpose_state", ctypes.c_int32 * OPERAND_COUNT),
        ("prefer_async_cache", ctypes.c_int32),
        ("prefer_async_load", ctypes.c_int32),
        ("has_softmax_scale", ctypes.c_int32),
        ("softmax_scale", ctypes.c_float),
        ("type", ctypes.c_int32),
        ("masking_strategy_override", ctypes.c_int32),
    ]


class AttentionKernel(ctypes.Structure):
    _fields_ = [
        ("block_parallelization", ctypes.c_uint16),
        ("block_traversal", ctypes.c_uint16),
        ("block_head", ctypes.c_uint16),
        ("threadgroup_size", ctypes.c_uint16),
        ("threadgroup_memory_allocation", ctypes.c_uint32),
        ("softmax_scale", ctypes.c_float),
        ("type", ctypes.c_int32),
        ("variant", ctypes.c_char * 96),
    ]


class KernelLaunch(ctypes.Structure):
    _fields_ = [
        ("name", ctypes.c_char * 96),
        ("threads", ctypes.c_uint32),
        ("lds_bytes", ctypes.c_uint32),
        ("workgroups", ctypes.c_uint64),
    ]


class KernelPlan(ctypes.Structure):
    _fields_ = [
        ("count", ctypes.c_int32),
        ("total", ctypes.c_int32),
        ("launches", KernelLaunch * 4),
    ]

    def as_list(self, strict: bool = True) -> list[dict]:
        """The recorded launches; a plan (strict) whose call issues more launches than the
        record holds raises instead of returning a partial list."""
        if strict and self.total > self.count:
            raise MFAError(-1, f"kernel plan truncated: {self.total} launches, {self.count} recorded")
        return [{"name": self.launches[i].name.decode(), "threads": self.launches[i].threads,
                 "lds_bytes": self.launches[i].lds_bytes,
                 "workgroups": self.launches[i].workgroups} for i in range(self.count)]


class MultiHeadShape(ctypes.Structure):
    _fields_ = [
        ("batch_size", ctypes.c_uint32),
        ("num_heads", ctypes.c_uint32),
        ("sequence_length", ctypes.c_uint32),
        ("head_dimension", ctypes.c_uint16),
        ("reserved0", ctypes.c_uint16),
    ]


class MultiHeadDescriptor(ctypes.Structure):
    _fields_ = [
        ("base", AttentionDescriptor),
        ("query_shape", MultiHeadShape),
        ("key_shape", MultiHeadShape),
        ("value_shape", MultiHeadShape),
        ("broadcast_mode", ctypes.c_int32),
        ("broadcast_param", ctypes.c_uint32),
        ("dispatch_strategy", ctypes.c_int32),
    ]

    @classmethod
    def make(cls, base: AttentionDescriptor, B, H, R, D, Hkv=None, C=None, mode=None,
             strategy=3):
        Hkv = H if Hkv is None else Hkv
        C = R if C is None else C
        d = cls()
        d.base = base
        d.query_shape = MultiHeadShape(B, H, R, D, 0)
        d.key_shape = MultiHeadShape(B, Hkv, C, D, 0)
        d.value_shape = MultiHeadShape(B, Hkv, C, D, 0)
        if mode is None:
            if Hkv == H and C == R:
                mode, param = Broadcast.standard, 0
            elif Hkv == H:
                mode, param = Broadcast.crossAttention, C
            elif Hkv == 1 and C == R:
                mode, param = Broadcast.multiQuery, 0
            elif C == R:
                mode, param = Broadcast.groupedQuery, Hkv
            else:
                mode, param = Broadcast.custom, 0
        else:
            param = Hkv if mode == Broadcast.groupedQuery else (C if mode == Broadcast.crossAttention else 0)
        d.broadcast_mode = int(mode)
        d.broadcast_param = param
        d.dispatch_strategy = strategy
        return d


class AttentionBuffers(ctypes.Structure):
    _fields_ = [
        ("Q", ctypes.c_void_p),
        ("K", ctypes.c_void_p),
        ("V", ctypes.c_void_p),
        ("O", ctypes.c_void_p),
        ("L", ctypes.c_void_p),
        ("D", ctypes.c_void_p),
        ("dO", ctypes.c_void_p),
        ("dV", ctypes.c_void_p),
        ("dK", ctypes.c_void_p),
        ("dQ", ctypes.c_void_p),
        ("Q_strides", ctypes.POINTER(ctypes.c_int64)),
        ("K_strides", ctypes.POINTER(ctypes.c_int64)),
        ("V_strides", ctypes.POINTER(ctypes.c_int64)),
        ("mask", ctypes.c_void_p),
    ]


class QuantizedTensor(ctypes.Structure):
    _fields_ = [
        ("data", ctypes.c_void_p),
        ("precision", ctypes.c_int32),
        ("scale", ctypes.c_float),
        ("zero_point", ctypes.c_int32),
        ("block_scales", ctypes.c_void_p),
        ("block_zero_points", ctypes.c_void_p),
        ("block_size", ctypes.c_uint32),
    ]


class QuantizedConfiguration(ctypes.Structure):
    _fields_ = [
        ("query_precision", ctypes.c_int32),
        ("key_precision", ctypes.c_int32),
        ("value_precision", ctypes.c_int32),
        ("query_strategy", ctypes.c_int32),
        ("key_strategy", ctypes.c_int32),
        ("value_strategy", ctypes.c_int32),
        ("strategy_version", ctypes.c_uint8),
        ("integer_matmul", ctypes.c_uint8),
        ("reserved", ctypes.c_uint8 * 2),
        ("mixed_precision_intermediates", ctypes.c_int32),
    ]


class QuantizedDescriptor(ctypes.Structure):
    _fields_ = [
        ("base", AttentionDescriptor),
        ("config", QuantizedConfiguration),
        ("batch_size", ctypes.c_uint32),
        ("num_heads", ctypes.c_uint32),
        ("num_kv_heads", ctypes.c_uint32),
        ("reserved0", ctypes.c_uint32),
    ]


class GemmDescriptor(ctypes.Structure):
    _fields_ = [
        ("M", ctypes.c_uint32), ("N", ctypes.c_uint32), ("K", ctypes.c_uint32),
        ("precision_a", ctypes.c_int32), ("precision_b", ctypes.c_int32),
        ("precision_c", ctypes.c_int32),
        ("transpose_a", ctypes.c_int32), ("transpose_b", ctypes.c_int32),
        ("load_previous_c", ctypes.c_int32),
        ("lda", ctypes.c_uint32), ("ldb", ctypes.c_uint32), ("ldc", ctypes.c_uint32),
        ("batch", ctypes.c_uint32),
        ("stride_a", ctypes.c_uint64), ("stride_b", ctypes.c_uint64), ("stride_c", ctypes.c_uint64),
    ]


class GemmKernelDescriptor(ctypes.Structure):  # GEMMKernelDescriptor.swift:8-60
    _fields_ = [
        ("block_m", ctypes.c_uint16), ("block_n", ctypes.c_uint16), ("block_k", ctypes.c_uint16),
        ("splits_m", ctypes.c_uint16), ("splits_n", ctypes.c_uint16),
        ("memory_precisions", ctypes.c_int32 * 3),
        ("register_precisions", ctypes.c_int32 * 3),
        ("transpose_a", ctypes.c_int32), ("transpose_b", ctypes.c_int32),
        ("load_previous_c", ctypes.c_int32),
        ("lda", ctypes.c_uint32), ("ldb", ctypes.c_uint32), ("ldc", ctypes.c_uint32),
        ("threadgroup_size", ctypes.c_uint32),
        ("threadgroup_memory_allocation", ctypes.c_uint32),
        ("grid_x", ctypes.c_uint32), ("grid_y", ctypes.c_uint32), ("grid_z", ctypes.c_uint32),
        ("variant", ctypes.c_char * 64),
    ]


class MLADescriptor(ctypes.Structure):
    _fields_ = [
        ("base", AttentionDescriptor),
        ("batch_size", ctypes.c_uint32),
        ("num_heads", ctypes.c_uint32),
        ("sequence_length_q", ctypes.c_uint32),
        ("sequence_length_kv", ctypes.c_uint32),
        ("head_dim", ctypes.c_uint32),
        ("kv_latent_dim", ctypes.c_uint32),
        ("precision", ctypes.c_int32),
    ]


def _sig(name, restype, argtypes):
    fn = getattr(lib, name, None)
    if fn is None:
        return
    fn.restype = restype
    fn.argtypes = argtypes


_P = ctypes.POINTER
_V = ctypes.c_void_p
_sig("mfa_version", ctypes.c_char_p, [])
_sig("mfa_last_error", ctypes.c_char_p, [])
_sig("mfa_abi_version", ctypes.c_int, [])
_sig("mfa_release_scratch", ctypes.c_int, [ctypes.c_void_p])
_sig("mfa_kernel_attribute_count", ctypes.c_int, [])
_sig("mfa_operand_buffer_binding", ctypes.c_int, [ctypes.c_int])
_sig("mfa_attention_descriptor_init", None, [_P(AttentionDescriptor)])
_sig("mfa_attention_kernel_descriptor", ctypes.c_int,
     [_P(AttentionDescriptor), ctypes.c_int, _P(KernelDescriptor)])
_sig("mfa_attention_kernel_create", ctypes.c_int, [_P(KernelDescriptor), _P(AttentionKernel)])
_sig("mfa_multihead_broadcast_compatible", ctypes.c_int, [_P(MultiHeadDescriptor)])
for _n in ("mfa_multihead_forward", "mfa_multihead_backward", "mfa_multihead_backward_query",
           "mfa_multihead_backward_key_value"):
    _sig(_n, ctypes.c_int, [_P(MultiHeadDescriptor), _P(AttentionBuffers), _V])
_sig("mfa_multihead_plan", ctypes.c_int,
     [_P(MultiHeadDescriptor), ctypes.c_int, _P(AttentionBuffers), _P(KernelPlan)])
_sig("mfa_last_launches", ctypes.c_int, [_P(KernelPlan)])
_sig("mfa_quantized_slot", ctypes.c_int, [ctypes.c_int, ctypes.c_int])
_sig("mfa_quantized_slot_table", ctypes.c_int, [ctypes.c_int, _P(ctypes.c_int32), ctypes.c_int])
_sig("mfa_quantized_slot_name", ctypes.c_char_p, [ctypes.c_int])
_sig("mfa_gluon_constants", None, [_P(ctypes.c_uint8)] * 3)
_sig("mfa_gluon_should_enable", ctypes.c_int, [ctypes.c_uint16, ctypes.c_uint16])
_sig("mfa_quantized_configuration_init", None, [_P(QuantizedConfiguration)])
_sig("mfa_quantized_plan", ctypes.c_int,
     [_P(QuantizedDescriptor), ctypes.c_int, _P(QuantizedTensor), _P(QuantizedTensor),
      _P(QuantizedTensor), _P(KernelPlan)])
_sig("mfa_quantized_forward", ctypes.c_int,
     [_P(QuantizedDescriptor), _P(QuantizedTensor), _P(QuantizedTensor), _P(QuantizedTensor),
      _V, _V, _V, _V])
_sig("mfa_quantized_forward_from_float", ctypes.c_int,
     [_P(QuantizedDescriptor), _V, _V, _V, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
      ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32, _V, _V, _V, _V])
_sig("mfa_quantized_backward_query", ctypes.c_int,
     [_P(QuantizedDescriptor), _P(QuantizedTensor), _P(QuantizedTensor), _P(QuantizedTensor),
      _V, _V, _V, _V, _V, _V])
_sig("mfa_quantized_backward_key_value", ctypes.c_int,
     [_P(QuantizedDescriptor), _P(QuantizedTensor), _P(QuantizedTensor), _P(QuantizedTensor),
      _V, _V, _V, _V, _V, _V])
_sig("mfa_quantize_workspace_size", ctypes.c_size_t,
     [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint32])
_sig("mfa_quantize", ctypes.c_int,
     [_V, ctypes.c_int32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int32,
      ctypes.c_int32, ctypes.c_uint32, _V, _V, _V, _V, _V, _V])
_sig("mfa_dequantize", ctypes.c_int,
     [_P(QuantizedTensor), ctypes.c_uint64, ctypes.c_uint32, _V, _V])
_sig("mfa_gemm", ctypes.c_int, [_P(GemmDescriptor), _V, _V, _V, _V])
_sig("mfa_gemm_kernel_descriptor", ctypes.c_int, [_P(GemmDescriptor), _P(GemmKernelDescriptor)])
_sig("mfa_mla_forward", ctypes.c_int,
     [_P(MLADescriptor), _V, _V, _V, _V, _V, _V, _V, _V, _V])
_sig("mfa_mla_absorbed_workspace_size", ctypes.c_size_t, [_P(MLADescriptor)])
_sig("mfa_mla_forward_absorbed", ctypes.c_int,
     [_P(MLADescriptor), _V, _V, _V, _V, _V, _V, _V, _V])
_sig("mfa_hadamard_rotate", ctypes.c_int, [_V, ctypes.c_uint32, ctypes.c_uint32, _V])
_sig("mfa_hadamard_rotate_batch", ctypes.c_int, [_V, ctypes.c_uint32, _V])
_sig("mfa_hadamard_scale", ctypes.c_float, [ctypes.c_uint32])
_sig("mfa_masking_sequence_bucket", ctypes.c_int, [ctypes.c_int])
_sig("mfa_masking_default_rule", ctypes.c_int, [ctypes.c_int, ctypes.c_int])
_sig("mfa_sparse_build_sliding_window", None, [ctypes.c_uint32, ctypes.c_uint32, _V])
_sig("mfa_sparse_build_block_sparse", None,
     [_V, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, _V])


def header_functions(path: str = HEADER_PATH) -> list[str]:
    """Names of every function declared in include/mfa/mfa.h."""
    text = open(path).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(mfa_[a-z0-9_]+)\s*\(", text)))


def check(status: int):
    if status != 0:
        raise MFAError(status, lib.mfa_last_error().decode())


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _stream(stream) -> Optional[int]:
    if stream is not None:
        return stream
    import torch
    return torch.cuda.current_stream().cuda_stream


def _strides(s: Optional[Sequence[int]]):
    if s is None:
        return None
    arr = (ctypes.c_int64 * 4)(*[int(x) for x in s])
    return ctypes.cast(arr, ctypes.POINTER(ctypes.c_int64)), arr


def kernel_descriptor(desc: AttentionDescriptor, kind: KernelType) -> KernelDescriptor:
    out = KernelDescriptor()
    check(lib.mfa_attention_kernel_descriptor(ctypes.byref(desc), int(kind), ctypes.byref(out)))
    return out


def attention_kernel(kdesc: KernelDescriptor) -> AttentionKernel:
    out = AttentionKernel()
    check(lib.mfa_attention_kernel_create(ctypes.byref(kdesc), ctypes.byref(out)))
    return out


def make_buffers(**kw) -> tuple[AttentionBuffers, list]:
    keep = []
    b = AttentionBuffers()
    for name in ("Q", "K", "V", "O", "L", "D", "dO", "dV", "dK", "dQ", "mask"):
        t = kw.get(name)
        setattr(b, name, _ptr(t))
    for name in ("Q_strides", "K_strides", "V_strides"):
        s = _strides(kw.get(name))
        if s is not None:
            setattr(b, name, s[0])
            keep.append(s[1])
    return b, keep


def multihead_plan(desc: MultiHeadDescriptor, kind: KernelType = KernelType.forward,
                   **buffers) -> list[dict]:
    """Kernels the call `kind` launches for `desc` (and, if given, these tensors' pointers
    and strides): [{name, threads, lds_bytes, workgroups}, ...] in issue order.  Needs no GPU."""
    out = KernelPlan()
    if buffers:
        b, keep = make_buffers(**buffers)
        bp = ctypes.byref(b)
    else:
        bp = None
    check(lib.mfa_multihead_plan(ctypes.byref(desc), int(kind), bp, ctypes.byref(out)))
    return out.as_list()


def quantized_plan(desc: "QuantizedDescriptor", kind: KernelType = KernelType.forward,
                   query=None, key=None, value=None) -> list[dict]:
    """mfa_quantized_plan: the kernels a quantized call launches (see multihead_plan)."""
    out = KernelPlan()
    ref = lambda t: None if t is None else ctypes.byref(t)
    check(lib.mfa_quantized_plan(ctypes.byref(desc), int(kind), ref(query), ref(key), ref(value),
                                 ctypes.byref(out)))
    return out.as_list()


QSLOT_COUNT = 39


def quantized_layout(kind: KernelType) -> dict[str, int]:
    """QuantizedKernelLayoutManifest.layout(for:).dictionary(): key name -> slot (-1 = the
    layout lists the key but gives it no slot); keys the layout does not list are absent."""
    out = (ctypes.c_int32 * QSLOT_COUNT)()
    if lib.mfa_quantized_slot_table(int(kind), out, QSLOT_COUNT) < 0:
        raise ValueError(kind)
    return {lib.mfa_quantized_slot_name(k).decode(): out[k] for k in range(QSLOT_COUNT)}


def gluon_constants() -> tuple[int, int, int]:
    """(SPLIT_EXP_FACTOR, CHANNEL_SYNC_POINTS, SUBTILE_SIZE)."""
    v = [ctypes.c_uint8() for _ in range(3)]
    lib.mfa_gluon_constants(*[ctypes.byref(x) for x in v])
    return tuple(x.value for x in v)


def last_launches() -> list[dict]:
    """mfa_last_launches: the kernels this thread launched since the previous call."""
    out = KernelPlan()
    lib.mfa_last_launches(ctypes.byref(out))
    return out.as_list(strict=False)


class MultiHeadAttention:
    """MultiHeadAttention (MultiHeadAttention.swift:11-708) over the C ABI."""

    def forward(self, desc: MultiHeadDescriptor, query, key, value, output, logsumexp=None,
                mask=None, query_strides=None, key_strides=None, value_strides=None,
                stream=None):
        b, keep = make_buffers(Q=query, K=key, V=value, O=output, L=logsumexp, mask=mask,
                               Q_strides=query_strides, K_strides=key_strides,
                               V_strides=value_strides)
        check(lib.mfa_multihead_forward(ctypes.byref(desc), ctypes.byref(b), _stream(stream)))

    encodeForward = forward

    def backward(self, desc: MultiHeadDescriptor, query, key, value, output, d_output,
                 logsumexp, d_query, d_key, d_value, d_buffer, mask=None, stream=None,
                 phase: str = "both"):
        b, keep = make_buffers(Q=query, K=key, V=value, O=output, dO=d_output, L=logsumexp,
                               dQ=d_query, dK=d_key, dV=d_value, D=d_buffer, mask=mask)
        fn = {"both": lib.mfa_multihead_backward, "query": lib.mfa_multihead_backward_query,
              "keyValue": lib.mfa_multihead_backward_key_value}[phase]
        check(fn(ctypes.byref(desc), ctypes.byref(b), _stream(stream)))


def quantized_tensor(data, precision: Precision, scale=1.0, zero_point=0, block_scales=None,
                     block_zero_points=None, block_size=0) -> QuantizedTensor:
    t = QuantizedTensor()
    t.data = _ptr(data)
    t.precision = int(precision)
    t.scale = float(scale)
    t.zero_point = int(zero_point)
    t.block_scales = _ptr(block_scales)
    t.block_zero_points = _ptr(block_zero_points)
    t.block_size = int(block_size)
    t._keep = (data, block_scales, block_zero_points)  # the struct holds raw device pointers
    return t


def quantized_descriptor(base: AttentionDescriptor, q_prec=Precision.FP16, k_prec=Precision.INT8,
                         v_prec=Precision.INT8, B=1, H=1, Hkv=None,
                         integer_matmul=False) -> QuantizedDescriptor:
    d = QuantizedDescriptor()
    d.base = base
    lib.mfa_quantized_configuration_init(ctypes.byref(d.config))
    d.config.query_precision = int(q_prec)
    d.config.key_precision = int(k_prec)
    d.config.value_precision = int(v_prec)
    d.config.integer_matmul = 1 if integer_matmul else 0
    d.batch_size, d.num_heads = B, H
    d.num_kv_heads = H if Hkv is None else Hkv
    return d


class QuantizedAttention:
    """QuantizedAttention (QuantizedAttention.swift:9-1560) over the C ABI."""

    def forward(self, desc: QuantizedDescriptor, query: QuantizedTensor, key: QuantizedTensor,
                value: QuantizedTensor, output, logsumexp=None, mask=None, stream=None):
        check(lib.mfa_quantized_forward(ctypes.byref(desc), ctypes.byref(query),
                                        ctypes.byref(key), ctypes.byref(value), _ptr(output),
                                        _ptr(logsumexp), _ptr(mask), _stream(stream)))

    def forward_from_buffers(self, desc: QuantizedDescriptor, query, key, value, output,
                             target: Precision, mode: "QuantMode" = None, block_size=0,
                             logsumexp=None, mask=None, stream=None, precisions=None):
        """forward(queryBuffer:keyBuffer:valueBuffer:...:targetQuantization:quantizationMode:
        descriptor:) (QuantizedAttention.swift:278-372): FP32/FP16/BF16 device tensors,
        quantized on the GPU to `target`, then the quantized forward."""
        import torch
        tp = {torch.float32: Precision.FP32, torch.float16: Precision.FP16,
              torch.bfloat16: Precision.BF16}
        qp, kp, vp = precisions or (tp[query.dtype], tp[key.dtype], tp[value.dtype])
        mode = QuantMode.tensorWise if mode is None else mode
        check(lib.mfa_quantized_forward_from_float(
            ctypes.byref(desc), _ptr(query), _ptr(key), _ptr(value), int(qp), int(kp), int(vp),
            int(target), int(mode), int(block_size), _ptr(output), _ptr(logsumexp), _ptr(mask),
            _stream(stream)))

    def backwardQuery(self, desc, query, key, value, output, grad_output, logsumexp, grad_query,
                      d_values, stream=None):
        check(lib.mfa_quantized_backward_query(
            ctypes.byref(desc), ctypes.byref(query), ctypes.byref(key), ctypes.byref(value),
            _ptr(output), _ptr(grad_output), _ptr(logsumexp), _ptr(grad_query), _ptr(d_values),
            _stream(stream)))

    def backwardKeyValue(self, desc, query, key, value, grad_output, logsumexp, d_values,
                         grad_key, grad_value, stream=None):
        check(lib.mfa_quantized_backward_key_value(
            ctypes.byref(desc), ctypes.byref(query), ctypes.byref(key), ctypes.byref(value),
            _ptr(grad_output), _ptr(logsumexp), _ptr(d_values), _ptr(grad_key),
            _ptr(grad_value), _stream(stream)))


def quantize(x, target: Precision, mode: QuantMode = QuantMode.tensorWise, rows=None, cols=None,
             block_size=0, stream=None):
    """GPU runtime quantisation (bit-exact with GEMMQuantization.swift).  Returns
    (data, scale_tensor, block_scales, block_zero_points)."""
    import torch
    prec = {torch.float32: Precision.FP32, torch.float16: Precision.FP16,
            torch.bfloat16: Precision.BF16}[x.dtype]
    n = x.numel()
    rows = rows if rows is not None else (x.shape[0] if x.dim() >= 2 else 1)
    cols = cols if cols is not None else (n // rows)
    nbytes = n if target == Precision.INT8 else (n + 1) // 2
    data = torch.empty(nbytes, dtype=torch.uint8, device=x.device)
    scale = torch.empty(1, dtype=torch.float32, device=x.device)
    if mode == QuantMode.blockwise:
        nb = ((rows + block_size - 1) // block_size) * ((cols + block_size - 1) // block_size)
    elif mode == QuantMode.rowWise:
        nb = rows
    else:
        nb = 0
    bs = torch.empty(max(nb, 1), dtype=torch.float32, device=x.device)
    bz = torch.empty(max(nb, 1), dtype=torch.int32, device=x.device)
    ws = torch.empty(max(int(lib.mfa_quantize_workspace_size(n, rows, cols, int(mode), block_size)), 16),
                     dtype=torch.uint8, device=x.device)
    check(lib.mfa_quantize(_ptr(x), int(prec), n, rows, cols, int(target), int(mode), block_size,
                           _ptr(data), _ptr(scale), _ptr(bs), _ptr(bz), _ptr(ws), _stream(stream)))
    return data, scale, (bs if nb else None), (bz if nb else None)


def gemm_descriptor(M, N, K, prec_a: Precision, prec_c: Precision, prec_b=None,
                    transpose_a=False, transpose_b=False, lda=0, ldb=0, ldc=0,
                    load_previous_c=False, batch=1, stride_a=0, stride_b=0, stride_c=0):
    """GEMMDescriptor (GEMMDescriptor.swift:11-47) as the C struct; prec_b defaults to prec_a."""
    d = GemmDescriptor()
    d.M, d.N, d.K = M, N, K
    d.precision_a = int(prec_a)
    d.precision_b = int(prec_a if prec_b is None else prec_b)
    d.precision_c = int(prec_c)
    d.transpose_a, d.transpose_b = int(bool(transpose_a)), int(bool(transpose_b))
    d.lda, d.ldb, d.ldc = lda, ldb, ldc
    d.load_previous_c = int(load_previous_c)
    d.batch = batch
    d.stride_a, d.stride_b, d.stride_c = stride_a, stride_b, stride_c
    return d


def gemm_kernel_descriptor(d: GemmDescriptor) -> GemmKernelDescriptor:
    """GEMMKernelDescriptor(descriptor:) (GEMMDescriptor.swift:110-246): the plan mfa_gemm runs."""
    out = GemmKernelDescriptor()
    check(lib.mfa_gemm_kernel_descriptor(ctypes.byref(d), ctypes.byref(out)))
    return out


def gemm(A, B, C, M, N, K, prec_a: Precision, prec_c: Precision, load_previous_c=False,
         stream=None, batch=1, stride_a=0, stride_b=0, stride_c=0, prec_b=None,
         transpose_a=False, transpose_b=False, lda=0, ldb=0, ldc=0):
    """C = op(A)·op(B) (+ C): GEMMKernel encode of a GEMMDescriptor (GEMMKernel+Source.swift)."""
    d = gemm_descriptor(M, N, K, prec_a, prec_c, prec_b, transpose_a, transpose_b, lda, ldb, ldc,
                        load_previous_c, batch, stride_a, stride_b, stride_c)
    check(lib.mfa_gemm(ctypes.byref(d), _ptr(A), _ptr(B), _ptr(C), _stream(stream)))


class HadamardItem(ctypes.Structure):  # rotateBatch tuple (HadamardRotation.swift:91-95)
    _fields_ = [("buffer", ctypes.c_void_p), ("block_size", ctypes.c_uint32),
                ("num_blocks", ctypes.c_uint32)]


class HadamardRotation:
    """HadamardRotation (Attention/HadamardRotation.swift:22-180): group-wise FWHT of FP32
    device buffers [num_blocks, block_size], in place, on the HIP kernel."""

    def rotate(self, buffer, block_size: int, num_blocks: int, stream=None):
        import torch
        if buffer.dtype != torch.float32:
            raise MFAError(4, "HadamardRotation.rotate: the buffer must be FP32")
        if buffer.numel() < block_size * num_blocks:
            raise MFAError(4, "HadamardRotation.rotate: buffer smaller than blockSize * numBlocks")
        check(lib.mfa_hadamard_rotate(_ptr(buffer), block_size, num_blocks, _stream(stream)))
        return buffer

    def rotate_batch(self, items, stream=None):
        import torch
        arr = (HadamardItem * max(len(items), 1))()
        for i, (buf, bs, nb) in enumerate(items):
            if buf.dtype != torch.float32 or buf.numel() < bs * nb:
                raise MFAError(4, "HadamardRotation.rotateBatch: bad buffer")
            arr[i] = HadamardItem(buf.data_ptr(), bs, nb)
        check(lib.mfa_hadamard_rotate_batch(arr, len(items), _stream(stream)))

    @staticmethod
    def scale(block_size: int) -> float:
        return float(lib.mfa_hadamard_scale(block_size))


def mla_forward(base: AttentionDescriptor, kv_latent, w_k, w_v, query, output, B, H, S_q, S_kv,
                head_dim, latent_dim, precision: Precision, k_buf=None, v_buf=None,
                logsumexp=None, stream=None):
    d = MLADescriptor()
    d.base = base
    d.batch_size, d.num_heads = B, H
    d.sequence_length_q, d.sequence_length_kv = S_q, S_kv
    d.head_dim, d.kv_latent_dim = head_dim, latent_dim
    d.precision = int(precision)
    check(lib.mfa_mla_forward(ctypes.byref(d), _ptr(kv_latent), _ptr(w_k), _ptr(w_v), _ptr(query),
                              _ptr(k_buf), _ptr(v_buf), _ptr(output), _ptr(logsumexp),
                              _stream(stream)))


def mla_forward_absorbed(base: AttentionDescriptor, kv_latent, w_k, w_v, query, output, B, H,
                         S_q, S_kv, head_dim, latent_dim, precision: Precision, workspace=None,
                         logsumexp=None, stream=None):
    """Absorbed MLA (attention in the latent space; K/V never materialised)."""
    d = MLADescriptor()
    d.base = base
    d.batch_size, d.num_heads = B, H
    d.sequence_length_q, d.sequence_length_kv = S_q, S_kv
    d.head_dim, d.kv_latent_dim = head_dim, latent_dim
    d.precision = int(precision)
    check(lib.mfa_mla_forward_absorbed(ctypes.byref(d), _ptr(kv_latent), _ptr(w_k), _ptr(w_v),
                                       _ptr(query), _ptr(workspace), _ptr(output),
                                       _ptr(logsumexp), _stream(stream)))


def attention_flops(B, H, R, C, D, causal=False, kind="forward") -> float:
    """Algorithmic FLOPs: forward 4·D per unmasked pair, backward 10·D."""
    if causal:
        # pairs (i, j) with j <= i, i < R, j < C
        if R <= C:
            pairs = R * (R + 1) // 2
        else:
            pairs = C * (C + 1) // 2 + (R - C) * C
    else:
        pairs = R * C
    per = {"forward": 4, "backward": 10, "backward7": 14}[kind]
    return float(per) * D * pairs * B * H
