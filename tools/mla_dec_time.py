#!/usr/bin/env python3
"""Times the absorbed-MLA decode call of bench.py's next_rows row (B32 H16 S_q 1 S_kv 4096,
latent 512, bf16): best of 5 rounds of 50 calls, HIP events on one stream.  Prints one line.
Development tool (MFA_LIB selects the library): python tools/mla_dec_time.py"""
import os
import sys

import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
u = lambda shape, dt: ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25).to(dt)
B, H, Sq, Skv, D, LAT = 32, 16, 1, 4096, 128, 512
lat = u((B * Skv, LAT), torch.bfloat16)
wk = (u((LAT, H * D), torch.float32) * 0.7).to(torch.bfloat16)
wv = (u((LAT, H * D), torch.float32) * 0.7).to(torch.bfloat16)
q = u((B, H, Sq, D), torch.bfloat16)
o = torch.empty((B, H, Sq, D), dtype=torch.float32, device=dev)
base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)
st = torch.cuda.Stream()
best = 1e9
with torch.cuda.stream(st):
    for _ in range(20):
        mfa.mla_forward_absorbed(base, lat, wk, wv, q, o, B, H, Sq, Skv, D, LAT, mfa.Precision.BF16, stream=st)
    torch.cuda.synchronize()
    for _ in range(5):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(50):
            mfa.mla_forward_absorbed(base, lat, wk, wv, q, o, B, H, Sq, Skv, D, LAT, mfa.Precision.BF16, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 50)
print(f"{os.environ.get('TAG', 'lib')} mla_absorbed_decode {best * 1e3:.1f} us  o[0,0,0,:2]={o[0, 0, 0, :2].tolist()}")
