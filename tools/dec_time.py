#!/usr/bin/env python3
"""Per-call times of the quantised decode forward at a few shapes (best of 5 rounds of 20
calls, HIP events on one stream), one line per shape; MFA_LIB selects the library.
Development tool: TAG=x python tools/dec_time.py"""
import os
import sys

import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision
dev = torch.device("cuda:0")
st = torch.cuda.Stream()
g = torch.Generator(device=dev).manual_seed(5)
cases = [(8, 32, 4, 1, 16384, 256, 8), (8, 32, 8, 1, 16384, 128, 4), (4, 32, 8, 1, 32768, 128, 8),
         (1, 32, 8, 4, 65536, 128, 8), (32, 16, 16, 1, 8192, 128, 8)]
if os.environ.get("DEC_SET") == "rows":  # more than 16 rows per kv head (the 32-row kernel)
    cases = [(8, 32, 4, 4, 16384, 128, 8), (8, 32, 4, 4, 16384, 128, 4), (8, 64, 8, 4, 16384, 128, 8),
             (8, 32, 4, 8, 16384, 128, 8), (32, 32, 8, 4, 4096, 128, 8)]
out = []
for B, H, Hkv, R, C, D, bits in cases:
    kv = P.INT8 if bits == 8 else P.INT4
    nb = D if bits == 8 else D // 2
    q = ((torch.rand((B, H, R, D), generator=g, device=dev) * 2 - 1)).half()
    k = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
    v = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
    o = torch.empty((B, H, R, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, R), dtype=torch.float16, device=dev)
    base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=P.FP16)
    desc = mfa.quantized_descriptor(base, P.FP16, kv, kv, B=B, H=H, Hkv=Hkv)
    tq, tk, tv = (mfa.quantized_tensor(q, P.FP16), mfa.quantized_tensor(k, kv, scale=0.01),
                  mfa.quantized_tensor(v, kv, scale=0.01))
    qa = mfa.QuantizedAttention()
    best = 1e9
    with torch.cuda.stream(st):
        for _ in range(5):
            qa.forward(desc, tq, tk, tv, o, l, stream=st)
        torch.cuda.synchronize()
        for _ in range(5):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(20):
                qa.forward(desc, tq, tk, tv, o, l, stream=st)
            e1.record(st)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / 20)
    byts = 2.0 * B * Hkv * C * nb
    out.append(f"B{B} H{H}/{Hkv} R{R} C{C} D{D} INT{bits}: {best * 1e3:6.1f} us {byts / best / 1e6:5.0f} GB/s")
    del q, k, v, o, l
print(os.environ.get("TAG", "lib"), " | ".join(out))
