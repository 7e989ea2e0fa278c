#!/usr/bin/env python3
"""v3 forward vs the v2 kernels on identical inputs: rows / heads that differ (development)."""
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import torch  # noqa: E402
import mfa_amd as mfa  # noqa: E402


def run(B, H, R, C, D, causal, prec=mfa.Precision.FP16, seed=0):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(seed)
    dt = torch.float16 if prec == mfa.Precision.FP16 else torch.bfloat16
    q = torch.randn((B, H, R, D), generator=g, device=dev).to(dt)
    k = torch.randn((B, H, C, D), generator=g, device=dev).to(dt)
    v = torch.randn((B, H, C, D), generator=g, device=dev).to(dt)
    base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=prec, causal=causal)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D, C=C)
    outs = []
    for var in ("1", "0"):
        os.environ["MFA_FWD3"] = var
        o = torch.zeros((B, H, R, D), dtype=torch.float32, device=dev)
        l = torch.zeros((B, H, R), dtype=torch.float16, device=dev)
        mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
        torch.cuda.synchronize()
        outs.append((o, l))
    (o3, l3), (o2, l2) = outs
    err = (o3 - o2).abs().amax(dim=-1)  # [B, H, R]
    bad = (err > 5e-3).nonzero().tolist()
    print(f"B{B} H{H} R{R} C{C} D{D} causal={causal}: max O err {err.max().item():.3g}, "
          f"L err {(l3.float() - l2.float()).abs().max().item():.3g}, bad rows {len(bad)}")
    if bad:
        rows = sorted({r for _, _, r in bad})
        print("   bad rows:", rows[:40], "..." if len(rows) > 40 else "")


if __name__ == "__main__":
    for args in [(1, 2, 300, 300, 128, True), (1, 2, 256, 256, 128, True), (1, 2, 512, 512, 128, True),
                 (1, 2, 384, 384, 128, True), (1, 2, 300, 300, 128, False), (1, 2, 512, 512, 128, False),
                 (1, 1, 1024, 1024, 128, True), (1, 2, 640, 640, 128, True)]:
        run(*args)
