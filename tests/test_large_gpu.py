"""GPU parity at the maximum-size edge: tensors past 2^31 elements (O and the gradients past
8 GiB), so every head / batch offset needs 64-bit arithmetic.  The shapes are many short heads
(B1024 H64 S256 D128 fp16, the tuned kernels' grids at their largest), and the oracle checks
heads at the start, the middle and the very end of the tensors.  Reference addressing:
MultiHeadAttention.swift's per-(batch, head) buffer offsets."""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr

pytestmark = pytest.mark.gpu
FP16 = mfa.Precision.FP16
DEV = "cuda:0"
B, H, S, D = 1024, 64, 256, 128  # 2^31 elements per Q/K/V/dO tensor
HEADS = ((0, 0), (511, 37), (B - 1, H - 1))


def need_memory(gib):
    free, _ = torch.cuda.mem_get_info(0)
    if free < gib * 2**30:
        pytest.skip(f"needs {gib} GiB of free device memory, {free / 2**30:.0f} GiB free")


def uniform16(seed):
    g = torch.Generator(device=DEV)
    g.manual_seed(seed)
    x = torch.rand((B, H, S, D), generator=g, device=DEV, dtype=torch.float16)
    return x.sub_(0.5)


def host(t, b, h):
    return t[b:b + 1, h:h + 1].float().cpu().numpy()


@pytest.mark.parametrize("causal", [False, True])
def test_forward_past_2g_elements(gpu, causal):
    need_memory(24)
    q, k, v = (uniform16(90 + i) for i in range(3))
    o = torch.full((B, H, S, D), float("nan"), device=DEV)
    l = torch.full((B, H, S), float("nan"), dtype=torch.float16, device=DEV)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, causal=causal)
    mfa.MultiHeadAttention().forward(mfa.MultiHeadDescriptor.make(base, B, H, S, D),
                                     q, k, v, o, l)
    torch.cuda.synchronize()
    assert o.numel() >= 2**31  # last O element at byte offset 8 GiB - 4
    for b, h in HEADS:
        ref = ol.attention(host(q, b, h), host(k, b, h), host(v, b, h), causal=causal)
        assert maxerr(o[b, h], ref["O"][0, 0]) <= 5e-3, (b, h)
        assert maxerr(l[b, h], ref["L"][0, 0]) <= 2e-2, (b, h)
    assert torch.isfinite(o).all() and torch.isfinite(l).all()  # every NaN-filled row written
    del q, k, v, o, l
    torch.cuda.empty_cache()


def test_backward_past_2g_elements(gpu):
    need_memory(56)
    q, k, v, do = (uniform16(95 + i) for i in range(4))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), device=DEV)
    l = torch.empty((B, H, S), dtype=torch.float16, device=DEV)
    dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=DEV)
    dq, dk, dv = (torch.full((B, H, S, D), float("nan"), device=DEV) for _ in range(3))
    mha = mfa.MultiHeadAttention()
    mha.forward(desc, q, k, v, o, l)
    mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf)
    torch.cuda.synchronize()
    for b, h in HEADS:
        ref = ol.attention(host(q, b, h), host(k, b, h), host(v, b, h), dO=host(do, b, h))
        for name, got in (("dQ", dq), ("dK", dk), ("dV", dv)):
            e = maxerr(got[b, h], ref[name][0, 0])
            assert e <= 5e-2, (name, b, h, e)
        assert maxerr(dbuf[b, h], ref["D"][0, 0]) <= 1e-1, (b, h)
    for g in (dq, dk, dv):
        assert torch.isfinite(g).all()  # NaN-filled: every gradient row was written
    del q, k, v, do, o, l, dbuf, dq, dk, dv
    torch.cuda.empty_cache()
