#!/usr/bin/env python3
"""Debug: stream-split causal forward vs the mirrored kernel, error per 128-row group."""
import os, sys
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import numpy as np
import torch
import mfa_amd as mfa

def run(q, k, v, env):
    old = {kk: os.environ.get(kk) for kk in env}
    os.environ.update({kk: str(vv) for kk, vv in env.items()})
    B, H, R, D = q.shape
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16, causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D, Hkv=k.shape[1], C=k.shape[2])
    o = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device="cuda:0")
    l = torch.full((B, H, R), float("nan"), dtype=torch.float16, device="cuda:0")
    mfa.last_launches()
    mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
    torch.cuda.synchronize()
    names = [r["name"] for r in mfa.last_launches()]
    for kk, vv in old.items():
        if vv is None: os.environ.pop(kk, None)
        else: os.environ[kk] = vv
    return o, l, names

g = torch.Generator(device="cuda:0").manual_seed(1)
for (B, H, R, D) in [(1, 1, 256, 128), (1, 2, 1024, 128)]:
    q, k, v = (torch.randn((B, H, R, D), generator=g, device="cuda:0").half() for _ in range(3))
    o0, l0, n0 = run(q, k, v, {"MFA_FWD_STREAM": 0})
    for W in (2, 3, 5):
        for slow in (0, 1):
            o1, l1, n1 = run(q, k, v, {"MFA_FWD_STREAM": 1, "MFA_FWD_STREAM_WGS": W, "MFA_FWD_STREAM_SLOW": slow})
            e = (o1 - o0).abs().amax(dim=-1)  # [B,H,R]
            el = (l1.float() - l0.float()).abs()
            per = e.view(B, H, R // 128 if R >= 128 else 1, -1).amax(dim=-1)
            print(f"B{B} H{H} R{R} W{W} slow{slow} {n1} maxO {e.max().item():.3g} maxL {el.max().item():.3g}")
            print("   per 128-row group:", np.array2string(per.cpu().numpy(), precision=3, max_line_width=200))
