"""Shared helpers for the GPU parity tests (device tensors <-> oracle arrays)."""
from __future__ import annotations

import numpy as np
import torch

import mfa_amd as mfa
import oracle_lib as ol

TORCH_DTYPE = {mfa.Precision.FP32: torch.float32, mfa.Precision.FP16: torch.float16,
               mfa.Precision.BF16: torch.bfloat16}
ROUND = {mfa.Precision.FP16: "fp16", mfa.Precision.BF16: "bf16"}


def to_device(x: np.ndarray, prec: mfa.Precision, dev="cuda:0") -> torch.Tensor:
    """Store x in `prec` on the device (RNE); returns the device tensor."""
    return torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(dev).to(TORCH_DTYPE[prec])


def seen(x: np.ndarray, prec: mfa.Precision) -> np.ndarray:
    """The values the kernel actually sees after storage in `prec`."""
    if prec == mfa.Precision.FP32:
        return np.asarray(x, dtype=np.float32)
    return ol.round16(x, ROUND[prec])


def maxerr(a, b) -> float:
    a = a.detach().float().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    if a.size == 0:
        return 0.0
    return float(np.max(np.abs(a.astype(np.float64) - b.astype(np.float64))))


def relerr(a, b) -> float:
    a = a.detach().float().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().float().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    d = np.linalg.norm((a.astype(np.float64) - b.astype(np.float64)).ravel())
    return float(d / (np.linalg.norm(b.astype(np.float64).ravel()) + 1e-8))


def run_forward(Qn, Kn, Vn, prec=mfa.Precision.FP32, causal=False, window=None, scale=None,
                amask=None, ranges=None, low_precision_intermediates=None, q_strides=None,
                layout=None, dev="cuda:0"):
    """Forward through the C ABI on BHSD numpy inputs; returns (O, L) torch tensors."""
    B, H, R, D = Qn.shape
    Hkv, C = Kn.shape[1], Kn.shape[2]
    lp = prec != mfa.Precision.FP32
    base = mfa.AttentionDescriptor.make(
        low_precision=lp, precision=prec if lp else None, causal=causal, window=window,
        scale=scale, low_precision_intermediates=low_precision_intermediates,
        sparse_mask=(mfa.MaskType.sparseRanges if ranges is not None else None))
    desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D, Hkv=Hkv, C=C)
    q, k, v = to_device(Qn, prec, dev), to_device(Kn, prec, dev), to_device(Vn, prec, dev)
    o = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device=dev)
    l_dtype = torch.float16 if base.low_precision_intermediates else torch.float32
    l = torch.full((B, H, R), float("nan"), dtype=l_dtype, device=dev)
    mask = None
    if amask is not None:
        mask = torch.from_numpy(np.ascontiguousarray(amask, dtype=np.float32)).to(dev)
    if ranges is not None:
        mask = torch.from_numpy(np.ascontiguousarray(ranges, dtype=np.uint32).view(np.int32)).to(dev)
    mfa.MultiHeadAttention().forward(desc, q, k, v, o, l, mask=mask)
    torch.cuda.synchronize()
    return o, l
