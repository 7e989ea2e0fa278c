"""GPU parity of the tuned backward kernels (attention_bwd_fast.hip) against the CPU oracle and
against the generic backward kernels (MFA_DISABLE_FAST=1) on the same inputs.

Shapes cover what the fast path claims: fp16/bf16, D in {64, 128, 256} (and D = 72, 136 that
pad to those), no mask / causal / sliding window, ragged R and C, cross attention (R != C),
GQA/MQA group sums.  Tolerances are the reference's mixed-precision ones
(SquareAttentionTest.swift:557-571: grads 5e-2, D 1e-1), scaled with sequence length as in
test_backward_gpu.py.
"""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, seen
from test_backward_gpu import check_backward, run_backward

pytestmark = pytest.mark.gpu

FP16, BF16 = mfa.Precision.FP16, mfa.Precision.BF16


def gaussian(shape, seed, s=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * s).astype(np.float32)


CASES = [
    # B, H, Hkv, R, C, D, mask
    (1, 2, 2, 256, 256, 64, None),
    (1, 2, 2, 300, 300, 128, "causal"),
    (2, 2, 2, 130, 130, 256, "causal"),
    (1, 2, 2, 200, 200, 128, ("window", 40)),
    (1, 3, 3, 100, 260, 64, None),
    (1, 2, 2, 260, 100, 128, "causal"),
    (1, 4, 2, 190, 190, 128, "causal"),
    (2, 4, 1, 96, 96, 256, None),
    (1, 2, 2, 77, 77, 72, "causal"),
    (1, 1, 1, 161, 161, 136, None),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("prec", [FP16, BF16])
def test_fast_backward_vs_oracle(gpu, case, prec):
    B, H, Hkv, R, C, D, mask = case
    seed = R + C + D
    Q, dO = gaussian((B, H, R, D), seed, 0.5), gaussian((B, H, R, D), seed + 1, 0.5)
    K, V = gaussian((B, Hkv, C, D), seed + 2, 0.5), gaussian((B, Hkv, C, D), seed + 3, 0.5)
    kw = {}
    if mask == "causal":
        kw["causal"] = True
    elif mask:
        kw["window"] = mask[1]
    tol = 5e-2 if prec == FP16 else 1e-1
    check_backward(Q, K, V, dO, prec, tol, 1e-1, **kw)


@pytest.mark.parametrize("D", [64, 128, 256])
@pytest.mark.parametrize("causal", [False, True])
def test_fast_matches_generic(gpu, D, causal):
    B, H, S = 1, 2, 192
    Q, K, V, dO = (gaussian((B, H, S, D), 70 + i, 0.5) for i in range(4))
    fast = run_backward(Q, K, V, dO, FP16, causal=causal)
    os.environ["MFA_DISABLE_FAST"] = "1"
    try:
        gen = run_backward(Q, K, V, dO, FP16, causal=causal)
    finally:
        os.environ.pop("MFA_DISABLE_FAST", None)
    for name in ("dQ", "dK", "dV"):
        a, b = fast[name].cpu().numpy(), gen[name].cpu().numpy()
        scale = max(1.0, float(np.abs(b).max()))
        assert np.abs(a - b).max() <= 2e-3 * scale, name
    # D is computed from the same values in the same precision; it may differ in summation
    # order only.
    assert np.abs(fast["D"].float().cpu().numpy() - gen["D"].float().cpu().numpy()).max() <= 2e-2


def test_fast_backward_c5_slice_full_length(gpu):
    # BASELINE configs[4] (fp16, S=4096, D=256) on 2 heads at full sequence length, checked
    # against a float64 torch restatement of the same math on the GPU (the C oracle is too
    # slow at this size), plus the exact identity sum_k dV[k] = sum_q dO[q] (rows of P sum to 1).
    B, H, S, D = 1, 2, 4096, 256
    g = torch.Generator(device="cuda:0").manual_seed(5)
    dev = "cuda:0"
    q, k, v, do = ((torch.rand((B, H, S, D), generator=g, device=dev) - 0.5).half()
                   for _ in range(4))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    dq, dk, dv = (torch.empty((B, H, S, D), dtype=torch.float32, device=dev) for _ in range(3))
    dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
    mha = mfa.MultiHeadAttention()
    mha.forward(desc, q, k, v, o, l)
    mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf)
    torch.cuda.synchronize()
    sc = 1.0 / np.sqrt(D)
    Q, K, V, dO = (t.double() for t in (q, k, v, do))
    P = torch.softmax((Q @ K.transpose(-1, -2)) * sc, dim=-1)
    O = P @ V
    dP = dO @ V.transpose(-1, -2)
    Dr = (dO * O).sum(-1, keepdim=True)
    dS = P * (dP - Dr)
    ref = {"dQ": (dS @ K) * sc, "dK": (dS.transpose(-1, -2) @ Q) * sc, "dV": P.transpose(-1, -2) @ dO}
    for name, got in (("dQ", dq), ("dK", dk), ("dV", dv)):
        r = ref[name]
        err = (got.double() - r).abs().max().item()
        assert err <= 5e-2 * max(1.0, r.abs().max().item()), f"{name}: {err}"
    sum_dv = dv.double().sum(dim=2)
    sum_do = do.double().sum(dim=2)
    assert (sum_dv - sum_do).abs().max().item() <= 1e-2 * max(1.0, sum_do.abs().max().item())


def test_c5_full_shard_slice_invariance(gpu):
    # BASELINE configs[4] at its full per-GPU shard (B8 H32 S4096 D256 fp16, 256 slices):
    # a size-independent property — every (batch, head) slice is independent, so the slices
    # of the full launch must equal, bit for bit, the same slices run alone (whose numerics
    # test_fast_backward_c5_slice_full_length pins).  Plus the dV column-sum identity on the
    # whole shard.
    B, H, S, D = 8, 32, 4096, 256
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(11)
    q, k, v, do = ((torch.rand((B, H, S, D), generator=g, device=dev) - 0.5).half()
                   for _ in range(4))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16)
    mha = mfa.MultiHeadAttention()

    def run(qq, kk, vv, dd):
        b, h = qq.shape[0], qq.shape[1]
        desc = mfa.MultiHeadDescriptor.make(base, b, h, S, D)
        o = torch.empty((b, h, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((b, h, S), dtype=torch.float16, device=dev)
        dq, dk, dv = (torch.empty((b, h, S, D), dtype=torch.float32, device=dev) for _ in range(3))
        dbuf = torch.empty((b, h, S), dtype=torch.bfloat16, device=dev)
        mha.forward(desc, qq, kk, vv, o, l)
        mha.backward(desc, qq, kk, vv, o, dd, l, dq, dk, dv, dbuf)
        torch.cuda.synchronize()
        return o, l, dq, dk, dv

    full = run(q, k, v, do)
    for (bi, hi) in [(0, 0), (3, 17), (7, 31)]:
        sl = lambda t: t[bi:bi + 1, hi:hi + 1].contiguous()
        one = run(sl(q), sl(k), sl(v), sl(do))
        for name, a, b1 in zip(("O", "L", "dQ", "dK", "dV"), full, one):
            assert torch.equal(a[bi:bi + 1, hi:hi + 1], b1), f"{name} slice ({bi},{hi})"
    dv = full[4]
    sum_dv = dv.double().sum(dim=2)
    sum_do = do.double().sum(dim=2)
    assert (sum_dv - sum_do).abs().max().item() <= 1e-2 * max(1.0, sum_do.abs().max().item())
    assert all(torch.isfinite(t).all() for t in full)


@pytest.mark.parametrize("prec", [FP16, BF16])
def test_config5_full_size_forward_backward(gpu, prec):
    """BASELINE.json configs[4] per-GPU shard (B8 H32 S4096 D256, non-causal) through the C
    ABI, forward then backward: one (b, h) slice against the C oracle at full length, and on
    every slice the size-independent identities of the backward (rows of P sum to one, so
    sum_k dV_k = sum_r dO_r; rows of dS sum to zero, so sum_k dK_k = 0)."""
    B, H, S, D = 8, 32, 4096, 256
    dt = torch.float16 if prec == FP16 else torch.bfloat16
    g = torch.Generator(device=gpu)
    g.manual_seed(55)
    q, k, v, do = ((torch.rand((B, H, S, D), generator=g, device=gpu) * 2 - 1).to(dt)
                   for _ in range(4))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=gpu)
    l = torch.empty((B, H, S), dtype=torch.float16, device=gpu)
    dq, dk, dv = (torch.full_like(o, float("nan")) for _ in range(3))
    dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=gpu)
    mha = mfa.MultiHeadAttention()
    mha.forward(desc, q, k, v, o, l)
    mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf)
    torch.cuda.synchronize()
    for t in (o, dq, dk, dv):
        assert torch.isfinite(t).all()
    # Identities on every slice (fp32 sums on the GPU).
    # Bounds relative to the sums of magnitudes: P and dS are rounded to the 16-bit MFMA
    # operand type, so each identity holds to that type's relative precision.
    eps = 2e-3 if prec == FP16 else 1.6e-2
    sdv, sdo = dv.sum(dim=2), do.float().sum(dim=2)
    assert ((sdv - sdo).abs() <= eps * do.float().abs().sum(dim=2) + 1e-3).all()
    assert (dk.sum(dim=2).abs() <= eps * dk.abs().sum(dim=2) + 1e-3).all()
    # One slice against the oracle (the inputs the kernel saw, already rounded).
    b, h = 3, 17
    sl = lambda t: t[b:b + 1, h:h + 1].float().cpu().numpy()
    ref = ol.attention(sl(q), sl(k), sl(v), dO=sl(do))
    assert maxerr(sl(o), ref["O"]) <= (5e-3 if prec == FP16 else 1e-2)
    tol = 5e-2 if prec == FP16 else 1e-1
    for name, t in (("dQ", dq), ("dK", dk), ("dV", dv)):
        e = maxerr(sl(t), ref[name])
        assert e <= tol, f"{name} max error {e} > {tol}"
    assert maxerr(dbuf[b:b + 1, h:h + 1].float().cpu().numpy(), ref["D"]) <= 1e-1
