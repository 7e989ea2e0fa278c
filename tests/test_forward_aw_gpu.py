"""GPU parity of the one-wave-per-SIMD forward with two query sub-blocks per wave and O in
kernel-owned AGPRs (attention_fwd_aw.hip), against the CPU oracle at the same tolerances as
the v2 kernels (tests/test_forward_v2_gpu.py: O 5e-3 fp16 / 1e-2 bf16, L 7e-3 + half an fp16
ulp).

The kernel is selected with MFA_FWD_AW=1 where it is not the default; every case asserts that
the launch was the aw kernel.  Cases cover both schedules (unmasked 256-row blocks; causal
mirrored pairs with the phase-2 split of B's keys and the in-register merge), odd block counts,
R and C off the tile grid, R != C, GQA, batches, and the speculative softmax pass's rescale
branch (a spike at the first, a middle and the last tile; a ramp that rescales every tile).
"""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
from test_forward_v2_gpu import BF16, FP16, check, gaussian

pytestmark = pytest.mark.gpu


@pytest.fixture
def aw(monkeypatch):
    monkeypatch.setenv("MFA_FWD_AW", "1")
    mfa.last_launches()
    yield
    names = [r["name"] for r in mfa.last_launches()]
    assert names and all(n.startswith("mfa_fwd_aw_kernel<") for n in names), names


CASES = [
    # B, H, Hkv, R, C, causal
    (1, 2, 2, 256, 256, False),
    (1, 2, 2, 256, 256, True),
    (1, 2, 2, 300, 300, True),      # 3 blocks: the middle pair is B only
    (1, 2, 2, 1024, 1024, True),    # 8 blocks: long phase 2
    (1, 2, 2, 1000, 1000, True),    # partial last block
    (1, 3, 3, 100, 260, False),     # one 128-row block (X1's rows past R)
    (1, 2, 2, 384, 300, False),
    (1, 2, 2, 260, 100, True),      # R > C: both blocks end at the last key (no phase 2)
    (1, 2, 2, 129, 1000, True),     # R < C
    (1, 4, 2, 640, 640, True),      # GQA
    (2, 4, 1, 512, 512, False),     # MQA, batch
    (2, 2, 2, 1536, 1536, True),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("prec", [FP16, BF16])
def test_aw_vs_oracle(gpu, aw, case, prec):
    B, H, Hkv, R, C, causal = case
    seed = R + 3 * C + 7 * B
    Q = gaussian((B, H, R, 128), seed)
    K, V = gaussian((B, Hkv, C, 128), seed + 1), gaussian((B, Hkv, C, 128), seed + 2)
    check(Q, K, V, prec, causal=causal)


@pytest.mark.parametrize("spike_key", [0, 70, 200, 511])
@pytest.mark.parametrize("prec", [FP16, BF16])
@pytest.mark.parametrize("causal", [False, True])
def test_aw_forced_rescale(gpu, aw, spike_key, prec, causal):
    # One key aligned with every query: the tile holding it raises the running max by ~20 in
    # log2 units, so the speculative pass is redone with the new offset there.
    B, H, S, D = 1, 2, 512, 128
    Q = gaussian((B, H, S, D), 7, 0.3)
    K = gaussian((B, H, S, D), 8, 0.3)
    V = gaussian((B, H, S, D), 9)
    direction = np.ones(D, dtype=np.float32) / np.sqrt(D)
    Q += 2.0 * direction
    K[:, :, spike_key] = 20.0 * direction
    check(Q, K, V, prec, causal=causal)


@pytest.mark.parametrize("prec", [FP16, BF16])
@pytest.mark.parametrize("causal", [False, True])
def test_aw_rescale_every_tile(gpu, aw, prec, causal):
    # Scores grow with the key index (S·c from ~19 to ~32 in log2 units), so the running max
    # moves past the threshold every few tiles, and the first tile's speculative P (computed
    # against offset 0) overflows fp16 before the rescale recomputes it.  (Larger scores would
    # only test the fp16 rounding of Q·scale·log2e, which the v2 kernels share.)
    B, H, S, D = 1, 1, 768, 128
    Q = np.zeros((B, H, S, D), dtype=np.float32)
    Q[..., 0] = 1.0
    K = gaussian((B, H, S, D), 11, 0.05)
    K[..., 0] = np.linspace(150.0, 250.0, S, dtype=np.float32)
    V = gaussian((B, H, S, D), 12)
    check(Q, K, V, prec, tol_l=2e-2, causal=causal)


@pytest.mark.parametrize("prec", [FP16, BF16])
def test_aw_config2_shape_heads(gpu, aw, prec):
    # BASELINE configs[1] (H16 S4096 D128 causal): every mirrored pair class; heads 0, 7, 15
    # against a float64 torch restatement of the reference forward.
    B, H, S, D = 1, 16, 4096, 128
    g = torch.Generator(device="cuda:0").manual_seed(3)
    dt = torch.float16 if prec == FP16 else torch.bfloat16
    q, k, v = ((torch.rand((B, H, S, D), generator=g, device="cuda:0") * 2 - 1).to(dt)
               for _ in range(3))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec, causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    l = torch.empty((B, H, S), dtype=torch.float16, device="cuda:0")
    mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
    torch.cuda.synchronize()
    for hh in (0, 7, 15):
        Qd, Kd, Vd = (t[0, hh].double() for t in (q, k, v))
        s = (Qd @ Kd.T) / np.sqrt(D)
        s = s + torch.triu(torch.full_like(s, float("-inf")), diagonal=1)
        m = s.max(dim=1, keepdim=True).values
        p = torch.exp(s - m)
        ref_o = (p @ Vd) / p.sum(dim=1, keepdim=True)
        ref_l = (m.squeeze(1) + torch.log(p.sum(dim=1))) / np.log(2)
        assert (o[0, hh].double() - ref_o).abs().max().item() <= 5e-3
        assert (l[0, hh].double() - ref_l).abs().max().item() <= 7e-3
