"""GPU: the per-rank forward and backward (mfa_shard.forward_shard / backward_shard) through
the C ABI reproduce the unsharded call when every rank's slices are run (ranks simulated in
one process; each slice is independent, so the results are bit-identical whenever the same
kernel instantiation runs)."""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import mfa_shard as sh

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,H,Hkv,world,prec", [(2, 8, 8, 3, mfa.Precision.FP32),
                                                (3, 8, 2, 2, mfa.Precision.FP32),
                                                (2, 16, 16, 8, mfa.Precision.FP16)])
def test_sharded_forward_equals_full(gpu, B, H, Hkv, world, prec):
    S, D = 200, 64
    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(3)
    dt = torch.float32 if prec == mfa.Precision.FP32 else torch.float16
    q = torch.randn((B, H, S, D), generator=g, device=dev).to(dt)
    k = torch.randn((B, Hkv, S, D), generator=g, device=dev).to(dt)
    v = torch.randn((B, Hkv, S, D), generator=g, device=dev).to(dt)
    lp = prec != mfa.Precision.FP32
    base = mfa.AttentionDescriptor.make(low_precision=lp, precision=prec if lp else None,
                                        causal=True)
    o_full = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l_full = torch.empty((B, H, S), dtype=torch.float16 if lp else torch.float32, device=dev)
    mfa.MultiHeadAttention().forward(mfa.MultiHeadDescriptor.make(base, B, H, S, D, Hkv=Hkv),
                                     q, k, v, o_full, l_full)
    o = torch.full_like(o_full, float("nan"))
    l = torch.full_like(l_full, float("nan"))
    n = sum(sh.forward_shard(mfa, base, q, k, v, o, l, world, r) for r in range(world))
    torch.cuda.synchronize()
    assert n == B * H
    if prec == mfa.Precision.FP32:
        assert torch.equal(o, o_full) and torch.equal(l, l_full)
    else:
        assert float((o - o_full).abs().max()) < 2e-3
        assert float((l.float() - l_full.float()).abs().max()) < 1e-2


@pytest.mark.parametrize("B,H,Hkv,world,prec", [(2, 8, 8, 3, mfa.Precision.FP16),
                                                (3, 8, 2, 2, mfa.Precision.FP16),
                                                (2, 4, 1, 2, mfa.Precision.BF16),
                                                (2, 4, 4, 4, mfa.Precision.FP32)])
def test_sharded_backward_equals_full(gpu, B, H, Hkv, world, prec):
    S, D = 192, 128
    dev = "cuda:0"
    g = torch.Generator(device=dev)
    g.manual_seed(5)
    lp = prec != mfa.Precision.FP32
    dt = {mfa.Precision.FP32: torch.float32, mfa.Precision.FP16: torch.float16,
          mfa.Precision.BF16: torch.bfloat16}[prec]
    q, do = ((torch.rand((B, H, S, D), generator=g, device=dev) - 0.5).to(dt) for _ in range(2))
    k, v = ((torch.rand((B, Hkv, S, D), generator=g, device=dev) - 0.5).to(dt) for _ in range(2))
    base = mfa.AttentionDescriptor.make(low_precision=lp, precision=prec if lp else None,
                                        causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D, Hkv=Hkv)
    mha = mfa.MultiHeadAttention()
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16 if lp else torch.float32, device=dev)
    mha.forward(desc, q, k, v, o, l)
    dd = torch.bfloat16 if lp else torch.float32
    full = [torch.empty_like(o), torch.empty((B, Hkv, S, D), dtype=torch.float32, device=dev),
            torch.empty((B, Hkv, S, D), dtype=torch.float32, device=dev),
            torch.empty((B, H, S), dtype=dd, device=dev)]
    mha.backward(desc, q, k, v, o, do, l, *full)
    shard = [torch.full_like(t, float("nan")) for t in full]
    n = sum(sh.backward_shard(mfa, base, q, k, v, o, do, l, *shard, world, r)
            for r in range(world))
    torch.cuda.synchronize()
    assert n == B * H
    for a, b in zip(shard, full):
        assert torch.equal(a, b)
