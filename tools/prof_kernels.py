#!/usr/bin/env python3
"""Runs one hot-path configuration a few times (a short program for rocprofv3 PMC passes).
Usage: python tools/prof_kernels.py {c2,c3,c3i8,c5f,c5q,c5kv,mla_dec,quant,dec4,dec8} [reps]"""
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import torch  # noqa: E402
import mfa_amd as mfa  # noqa: E402

which = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(1)
u = lambda shape, dt: ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25).to(dt)
mha = mfa.MultiHeadAttention()
if which in ("c2", "c3"):
    S, causal = (4096, True) if which == "c2" else (8192, False)
    B, H, D = 1, 16, 128
    q, k, v = (u((B, H, S, D), torch.float16) for _ in range(3))
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16, causal=causal)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    for _ in range(reps):
        mha.forward(desc, q, k, v, o, l)
elif which == "quant":
    # Runtime quantiser at the C3 K size (16.8 M FP32 elements): tensor-wise and row-wise INT8.
    x = u((16 * 8192 * 128,), torch.float32)
    for _ in range(reps):
        mfa.quantize(x, mfa.Precision.INT8)
        mfa.quantize(x, mfa.Precision.INT8, rows=16 * 8192, cols=128)
elif which == "mla_dec":
    # Absorbed MLA decode, as bench.py's next_rows entry (B32 H16 S_q 1 S_kv 4096, latent 512).
    B, H, Sq, Skv, D, LAT = 32, 16, 1, 4096, 128, 512
    lat = u((B * Skv, LAT), torch.bfloat16)
    wk = (u((LAT, H * D), torch.float32) * 0.7).to(torch.bfloat16)
    wv = (u((LAT, H * D), torch.float32) * 0.7).to(torch.bfloat16)
    q = u((B, H, Sq, D), torch.bfloat16)
    o = torch.empty((B, H, Sq, D), dtype=torch.float32, device=dev)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)
    for _ in range(reps):
        mfa.mla_forward_absorbed(base, lat, wk, wv, q, o, B, H, Sq, Skv, D, LAT, mfa.Precision.BF16)
elif which in ("dec4", "dec8"):
    # Split-KV decode as bench.py's int8_decode row (B32 H16 S_kv 8192 D128, S_q 1), INT4 / INT8.
    B, H, C, D = 32, 16, 8192, 128
    kv = mfa.Precision.INT4 if which == "dec4" else mfa.Precision.INT8
    nb = D // 2 if which == "dec4" else D
    q = u((B, H, 1, D), torch.float16)
    k = torch.randint(0, 256, (B, H, C, nb), generator=g, device=dev, dtype=torch.uint8)
    v = torch.randint(0, 256, (B, H, C, nb), generator=g, device=dev, dtype=torch.uint8)
    o = torch.empty((B, H, 1, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, 1), dtype=torch.float16, device=dev)
    base = mfa.AttentionDescriptor.make(1, C, D, low_precision=True, precision=mfa.Precision.FP16)
    qd = mfa.quantized_descriptor(base, mfa.Precision.FP16, kv, kv, B=B, H=H)
    tq = mfa.quantized_tensor(q, mfa.Precision.FP16)
    tk = mfa.quantized_tensor(k, kv, scale=0.01)
    tv = mfa.quantized_tensor(v, kv, scale=0.01)
    for _ in range(reps):
        mfa.QuantizedAttention().forward(qd, tq, tk, tv, o, l)
elif which == "c3i8":
    B, H, S, D = 1, 16, 8192, 128
    qf = u((B, H, S, D), torch.float16)
    kf, vf = u((B, H, S, D), torch.float32), u((B, H, S, D), torch.float32)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    kq, ks, _, _ = mfa.quantize(kf, mfa.Precision.INT8, rows=B * H * S, cols=D)
    vq, vs, _, _ = mfa.quantize(vf, mfa.Precision.INT8, rows=B * H * S, cols=D)
    base = mfa.AttentionDescriptor.make(S, S, D, low_precision=True, precision=mfa.Precision.FP16)
    qd = mfa.quantized_descriptor(base, mfa.Precision.FP16, mfa.Precision.INT8, mfa.Precision.INT8,
                                  B=B, H=H, integer_matmul=True)
    tq = mfa.quantized_tensor(qf, mfa.Precision.FP16)
    tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=float(ks.item()))
    tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=float(vs.item()))
    for _ in range(reps):
        mfa.QuantizedAttention().forward(qd, tq, tk, tv, o, l)
else:
    B, H, S, D = 2, 32, 4096, 256
    q, k, v, do = (u((B, H, S, D), torch.float16) for _ in range(4))
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    dq, dk, dv = (torch.empty((B, H, S, D), dtype=torch.float32, device=dev) for _ in range(3))
    dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    mha.forward(desc, q, k, v, o, l)
    for _ in range(reps):
        if which == "c5f":
            mha.forward(desc, q, k, v, o, l)
        elif which == "c5q":
            mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf, phase="query")
        else:
            mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf, phase="keyValue")
torch.cuda.synchronize()
