#!/usr/bin/env python3
"""Uniform-attention probe of the v3 causal forward: Q = K = 0 so every visible key has P = 1,
V[k, d] = k + d/1000, so O[r, d] = mean of the visible keys' indices (development)."""
import os
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import torch  # noqa: E402
import mfa_amd as mfa  # noqa: E402

dev = torch.device("cuda:0")
B, H, R, D = 1, 1, int(sys.argv[1]) if len(sys.argv) > 1 else 256, 128
q = torch.zeros((B, H, R, D), device=dev, dtype=torch.float16)
k = torch.zeros_like(q)
v = (torch.arange(R, device=dev, dtype=torch.float32)[:, None] / 8 +
     torch.arange(D, device=dev, dtype=torch.float32)[None, :] / 1024).to(torch.float16)[None, None].contiguous()
base = mfa.AttentionDescriptor.make(R, R, D, low_precision=True, precision=mfa.Precision.FP16, causal=True)
desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D)
o = torch.zeros((B, H, R, D), dtype=torch.float32, device=dev)
l = torch.zeros((B, H, R), dtype=torch.float16, device=dev)
os.environ["MFA_FWD3"] = "1"
mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
torch.cuda.synchronize()
vf = v.float()[0, 0]
exp = torch.stack([vf[: r + 1].mean(0) for r in range(R)])
err = (o[0, 0] - exp).abs().amax(-1)
for r in range(R):
    if err[r] > 1e-2:
        # implied sum of included key indices (times 1/8) vs expected
        print(f"row {r}: O[0]={o[0,0,r,0].item():.4f} exp {exp[r,0].item():.4f}  L={l[0,0,r].item():.3f} "
              f"log2(r+1)={torch.log2(torch.tensor(r + 1.0)).item():.3f}  O[32]={o[0,0,r,32].item():.4f} O[64]={o[0,0,r,64].item():.4f} O[96]={o[0,0,r,96].item():.4f}")
print("bad rows", int((err > 1e-2).sum()))
