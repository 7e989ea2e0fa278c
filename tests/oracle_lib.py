"""numpy front-end to the CPU oracle (oracle/libmfa_oracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this module, and
only as the checker.  See oracle/mfa_oracle.c for the reference files each routine restates.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(_REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "libmfa_oracle.so")
# MFA_ORACLE_LIB: another build of the same source, e.g. the sanitizer build
# (oracle/_asan/libmfa_oracle.so, tools/asan_check.sh).
_ALT = os.environ.get("MFA_ORACLE_LIB")


def _load():
    if _ALT:
        return ctypes.CDLL(_ALT)
    src = os.path.join(ORACLE_DIR, "mfa_oracle.c")
    if not os.path.exists(ORACLE_LIB) or os.path.getmtime(ORACLE_LIB) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", ORACLE_DIR])
    return ctypes.CDLL(ORACLE_LIB)


olib = _load()

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(dtype=np.uint8, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


class AttnArgs(ctypes.Structure):
    _fields_ = [
        ("B", ctypes.c_int32), ("H", ctypes.c_int32), ("Hkv", ctypes.c_int32),
        ("R", ctypes.c_int32), ("C", ctypes.c_int32), ("D", ctypes.c_int32),
        ("scale", ctypes.c_float),
        ("causal", ctypes.c_int32), ("window", ctypes.c_int32), ("window_size", ctypes.c_uint32),
        ("amask", ctypes.c_void_p), ("ranges", ctypes.c_void_p),
        ("Q", ctypes.c_void_p), ("K", ctypes.c_void_p), ("V", ctypes.c_void_p),
    ]


olib.mfa_oracle_lcg_fill.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_float, _f32p]
olib.mfa_oracle_lcg_stream.argtypes = [ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint64,
                                       ctypes.c_float, ctypes.c_float, _f32p]
olib.mfa_oracle_f32_to_f16.restype = ctypes.c_uint16
olib.mfa_oracle_f32_to_f16.argtypes = [ctypes.c_float]
olib.mfa_oracle_f16_to_f32.restype = ctypes.c_float
olib.mfa_oracle_f16_to_f32.argtypes = [ctypes.c_uint16]
olib.mfa_oracle_f32_to_bf16_rne.restype = ctypes.c_uint16
olib.mfa_oracle_f32_to_bf16_rne.argtypes = [ctypes.c_float]
olib.mfa_oracle_f32_to_bf16_trunc.restype = ctypes.c_uint16
olib.mfa_oracle_f32_to_bf16_trunc.argtypes = [ctypes.c_float]
olib.mfa_oracle_round16.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_int, _f32p]
olib.mfa_oracle_attention_forward.argtypes = [ctypes.POINTER(AttnArgs), _f32p, ctypes.c_void_p]
olib.mfa_oracle_attention_backward.argtypes = [ctypes.POINTER(AttnArgs), _f32p, _f32p, _f32p,
                                               _f32p, _f32p]
olib.mfa_oracle_quant_scale_tensor.restype = ctypes.c_float
olib.mfa_oracle_quant_scale_tensor.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_int]
olib.mfa_oracle_quant_scales_block.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_uint32,
                                               ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                               _f32p]
olib.mfa_oracle_quant_scales_row.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_int, _f32p]
olib.mfa_oracle_quantize.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_int, ctypes.c_float,
                                     ctypes.c_int32, _u8p]
olib.mfa_oracle_quantize_block.argtypes = [_f32p, ctypes.c_uint64, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_int, _f32p,
                                           ctypes.c_void_p, _u8p]
olib.mfa_oracle_dequantize.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_int, ctypes.c_float,
                                       ctypes.c_int32, _f32p]
olib.mfa_oracle_dequantize_block.argtypes = [_u8p, ctypes.c_uint64, ctypes.c_uint32,
                                             ctypes.c_uint32, ctypes.c_int, _f32p,
                                             ctypes.c_void_p, _f32p]
olib.mfa_oracle_gemm.argtypes = [_f32p, _f32p, _f32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int]
olib.mfa_oracle_set_threads.restype = ctypes.c_int
olib.mfa_oracle_set_threads.argtypes = [ctypes.c_int]

INT8, INT4 = 3, 4


def lcg(seed: int, count: int, scale: float = 0.25) -> np.ndarray:
    """KernelRegressionTests.deterministicData (KernelRegressionTests.swift:41-50)."""
    out = np.empty(count, dtype=np.float32)
    olib.mfa_oracle_lcg_fill(seed, count, scale, out)
    return out


class LCGStream:
    """QuantizedAttentionTest.nextRandom (QuantizedAttentionTest.swift:446-450)."""

    def __init__(self, seed: int):
        self.state = ctypes.c_uint64(seed)

    def draw(self, count: int, mul: float = 2.0, add: float = -1.0) -> np.ndarray:
        out = np.empty(count, dtype=np.float32)
        olib.mfa_oracle_lcg_stream(ctypes.byref(self.state), count, mul, add, out)
        return out


def round16(x: np.ndarray, kind: str) -> np.ndarray:
    """Values after storage in fp16 ('fp16'), bf16 RNE ('bf16') or bf16 truncation."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty_like(x)
    olib.mfa_oracle_round16(x.reshape(-1), x.size,
                            {"fp16": 1, "bf16": 2, "bf16_trunc": 3}[kind], out.reshape(-1))
    return out


def attention(Q, K, V, *, scale=None, causal=False, window=None, amask=None, ranges=None,
              dO=None):
    """Forward (and backward when dO is given) on contiguous BHSD float32 arrays.
    Returns dict with O, L (log2 units) and, for backward, D (scale·rowsum), dQ, dK, dV."""
    Q = np.ascontiguousarray(Q, dtype=np.float32)
    K = np.ascontiguousarray(K, dtype=np.float32)
    V = np.ascontiguousarray(V, dtype=np.float32)
    B, H, R, D = Q.shape
    Hkv, C = K.shape[1], K.shape[2]
    a = AttnArgs()
    a.B, a.H, a.Hkv, a.R, a.C, a.D = B, H, Hkv, R, C, D
    a.scale = -1.0 if scale is None else scale
    a.causal = int(causal)
    a.window = int(window is not None)
    a.window_size = 0 if window is None else window
    keep = [Q, K, V]
    if amask is not None:
        amask = np.ascontiguousarray(amask, dtype=np.float32)
        keep.append(amask)
        a.amask = amask.ctypes.data
    if ranges is not None:
        ranges = np.ascontiguousarray(ranges, dtype=np.uint32)
        keep.append(ranges)
        a.ranges = ranges.ctypes.data
    a.Q, a.K, a.V = Q.ctypes.data, K.ctypes.data, V.ctypes.data
    O = np.empty((B, H, R, D), dtype=np.float32)
    L = np.empty((B, H, R), dtype=np.float32)
    olib.mfa_oracle_attention_forward(ctypes.byref(a), O, L.ctypes.data)
    out = {"O": O, "L": L}
    if dO is not None:
        dO = np.ascontiguousarray(dO, dtype=np.float32)
        Dt = np.empty((B, H, R), dtype=np.float32)
        dQ = np.empty_like(Q)
        dK = np.empty_like(K)
        dV = np.empty_like(V)
        olib.mfa_oracle_attention_backward(ctypes.byref(a), dO, Dt, dQ, dK, dV)
        out.update(D=Dt, dQ=dQ, dK=dK, dV=dV)
    return out


def quant_scale_tensor(x: np.ndarray, prec: int) -> float:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    return float(olib.mfa_oracle_quant_scale_tensor(x, x.size, prec))


def quant_scales_block(x: np.ndarray, rows: int, cols: int, bs: int, prec: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    nb = ((rows + bs - 1) // bs) * ((cols + bs - 1) // bs)
    out = np.empty(nb, dtype=np.float32)
    olib.mfa_oracle_quant_scales_block(x, x.size, rows, cols, bs, prec, out)
    return out


def quant_scales_row(x: np.ndarray, rows: int, cols: int, prec: int) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    out = np.empty(rows, dtype=np.float32)
    olib.mfa_oracle_quant_scales_row(x, x.size, rows, cols, prec, out)
    return out


def quantize(x: np.ndarray, prec: int, scale: float, zp: int = 0) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    out = np.empty(x.size if prec == INT8 else (x.size + 1) // 2, dtype=np.uint8)
    olib.mfa_oracle_quantize(x, x.size, prec, scale, zp, out)
    return out


def quantize_block(x: np.ndarray, cols: int, bs: int, prec: int, scales: np.ndarray,
                   zps: np.ndarray | None = None) -> np.ndarray:
    x = np.ascontiguousarray(x, dtype=np.float32).reshape(-1)
    scales = np.ascontiguousarray(scales, dtype=np.float32)
    out = np.empty(x.size if prec == INT8 else (x.size + 1) // 2, dtype=np.uint8)
    z = None if zps is None else np.ascontiguousarray(zps, dtype=np.int32)
    olib.mfa_oracle_quantize_block(x, x.size, cols, bs, prec, scales,
                                   None if z is None else z.ctypes.data, out)
    return out


def dequantize(q: np.ndarray, count: int, prec: int, scale: float, zp: int = 0) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.uint8)
    out = np.empty(count, dtype=np.float32)
    olib.mfa_oracle_dequantize(q, count, prec, scale, zp, out)
    return out


def dequantize_block(q: np.ndarray, count: int, cols: int, bs: int, prec: int,
                     scales: np.ndarray, zps: np.ndarray | None = None) -> np.ndarray:
    q = np.ascontiguousarray(q, dtype=np.uint8)
    scales = np.ascontiguousarray(scales, dtype=np.float32)
    z = None if zps is None else np.ascontiguousarray(zps, dtype=np.int32)
    out = np.empty(count, dtype=np.float32)
    olib.mfa_oracle_dequantize_block(q, count, cols, bs, prec, scales,
                                     None if z is None else z.ctypes.data, out)
    return out


def gemm(A: np.ndarray, B: np.ndarray, prev: np.ndarray | None = None) -> np.ndarray:
    """C = A·B (+ prev, loadPreviousC) with double accumulation, one fp32 rounding."""
    A = np.ascontiguousarray(A, dtype=np.float32)
    B = np.ascontiguousarray(B, dtype=np.float32)
    M, K = A.shape
    N = B.shape[1]
    if prev is None:
        C = np.zeros((M, N), dtype=np.float32)
    else:
        C = np.array(prev, dtype=np.float32, copy=True, order="C")
    olib.mfa_oracle_gemm(A, B, C, M, N, K, 0 if prev is None else 1)
    return C


def set_threads(n: int) -> int:
    return int(olib.mfa_oracle_set_threads(n))


olib.mfa_oracle_hadamard.argtypes = [_f32p, ctypes.c_int, ctypes.c_int64, ctypes.c_float]
olib.mfa_oracle_hadamard.restype = None


def hadamard(x: np.ndarray, block_size: int, scale: float) -> np.ndarray:
    """HadamardRotation.rotate on a copy of the flat FP32 buffer x (oracle/mfa_oracle.c)."""
    y = np.array(x, dtype=np.float32, copy=True, order="C").ravel()
    olib.mfa_oracle_hadamard(y, block_size, y.size // block_size, scale)
    return y.reshape(np.shape(x))
