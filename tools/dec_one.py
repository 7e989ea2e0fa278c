#!/usr/bin/env python3
"""Runs one decode shape 50 times (a short program for rocprofv3 kernel stats).
Usage: python tools/dec_one.py B H Hkv R C D {8,4}"""
import os
import sys

import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision
B, H, Hkv, R, C, D, bits = (int(x) for x in sys.argv[1:8])
kv = P.INT8 if bits == 8 else P.INT4
nb = D if bits == 8 else D // 2
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(5)
q = ((torch.rand((B, H, R, D), generator=g, device=dev) * 2 - 1)).half()
k = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
v = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
o = torch.empty((B, H, R, D), dtype=torch.float32, device=dev)
l = torch.empty((B, H, R), dtype=torch.float16, device=dev)
base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=P.FP16)
desc = mfa.quantized_descriptor(base, P.FP16, kv, kv, B=B, H=H, Hkv=Hkv)
tq, tk, tv = mfa.quantized_tensor(q, P.FP16), mfa.quantized_tensor(k, kv, scale=0.01), mfa.quantized_tensor(v, kv, scale=0.01)
qa = mfa.QuantizedAttention()
for _ in range(50):
    qa.forward(desc, tq, tk, tv, o, l)
torch.cuda.synchronize()
print([r["name"] for r in mfa.quantized_plan(desc, mfa.KernelType.forward, tq, tk, tv)])
