#!/usr/bin/env python3
"""Interleaved A/B of forward-kernel variants selected by environment knobs, in one process
(development tool).  Usage: python tools/ab_fwd.py VAR=val1,val2 [--cfg C2|C3] [--rounds N]"""
import argparse
import json
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import statistics
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knob")
    ap.add_argument("--cfg", default="C2")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--nocheck", action="store_true", help="timing-only variants (ablations)")
    a = ap.parse_args()
    var, vals = a.knob.split("=")
    vals = vals.split(",")
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(7)
    causal = a.cfg == "C2"
    B, H, S, D = (1, 16, 4096, 128) if a.cfg in ("C2", "C2Q8") else (1, 16, 8192, 128)
    if a.cfg == "C2D64":
        B, H, S, D = 1, 32, 4096, 64
        causal = True
    if a.cfg == "C2B4":  # C2 with 4x the batch (2048 causal blocks)
        B, H, S, D = 4, 16, 4096, 128
        causal = True
    if a.cfg == "C2S8":  # causal S8192 (1024 blocks)
        B, H, S, D = 1, 16, 8192, 128
        causal = True
    if a.cfg.startswith("x"):  # xB,H,S,D,causal (0/1)
        B, H, S, D, cz = (int(t) for t in a.cfg[1:].split(","))
        causal = bool(cz)
    if a.cfg in ("C4A", "C4AF"):  # C4's attention (bf16), and the same shape in fp16
        B, H, S, D = 1, 16, 4096, 128
        causal = False
    if a.cfg == "C5F":  # C5's forward on a 2-batch slice
        B, H, S, D = 2, 32, 4096, 256
        causal = False
    dt = torch.bfloat16 if a.cfg == "C4A" else torch.float16
    q, k, v = (((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1) * 0.25).to(dt)
               for _ in range(3))
    i8 = a.cfg == "C3I8"
    q8c = a.cfg == "C2Q8"  # QuantizedAttention, per-tensor INT8 K/V, dequant-exact, causal C2
    if q8c:
        causal = True
        kq, ks, _, _ = mfa.quantize(k.float().view(-1), mfa.Precision.INT8)
        vq, vs, _, _ = mfa.quantize(v.float().view(-1), mfa.Precision.INT8)
        torch.cuda.synchronize()
        qdesc = mfa.quantized_descriptor(
            mfa.AttentionDescriptor.make(S, S, D, causal=True, low_precision=True,
                                         precision=mfa.Precision.FP16),
            mfa.Precision.FP16, mfa.Precision.INT8, mfa.Precision.INT8, B=B, H=H)
        tq = mfa.quantized_tensor(q, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=ks.item())
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=vs.item())
    if i8:
        causal = False
        kq, ks, _, _ = mfa.quantize(k.float().view(-1), mfa.Precision.INT8)
        vq, vs, _, _ = mfa.quantize(v.float().view(-1), mfa.Precision.INT8)
        torch.cuda.synchronize()
        qdesc = mfa.quantized_descriptor(mfa.AttentionDescriptor.make(S, S, D), mfa.Precision.FP16,
                                         mfa.Precision.INT8, mfa.Precision.INT8, B=B, H=H,
                                         integer_matmul=True)
        tq = mfa.quantized_tensor(q, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=ks.item())
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=vs.item())
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    base = mfa.AttentionDescriptor.make(
        low_precision=True, precision=mfa.Precision.BF16 if a.cfg == "C4A" else mfa.Precision.FP16,
        causal=causal)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    mha = mfa.MultiHeadAttention()
    if i8 or q8c:
        qa = mfa.QuantizedAttention()
        run = lambda: qa.forward(qdesc, tq, tk, tv, o)
    else:
        run = lambda: mha.forward(desc, q, k, v, o, l)
    flop = 4 * D * (S * (S + 1) / 2 if causal else S * S) * B * H
    ref = None
    res = {x: [] for x in vals}
    rel = {}
    for r in range(a.rounds):
        for x in vals:
            os.environ[var] = x
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = o.clone()
            elif i8:
                rel[x] = float((o - ref).norm() / ref.norm())
            elif not a.nocheck:
                assert torch.allclose(o, ref, atol=2e-3), f"{var}={x} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[x].append(e0.elapsed_time(e1) / a.reps)
    out = {x: {"ms_med": round(statistics.median(t), 4), "tflops": round(flop / statistics.median(t) / 1e9, 1)}
           for x, t in res.items()}
    print(json.dumps({"cfg": a.cfg, "knob": var, **out, "relL2_vs_first": rel}))


if __name__ == "__main__":
    main()
