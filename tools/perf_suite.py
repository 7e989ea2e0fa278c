#!/usr/bin/env python3
"""Per-configuration timing of every hot-path entry point on one MI355X (development tool).

Times, with HIP events on the launch stream, each BASELINE.json config that fits one GPU:
  C2  fp16 forward, H16 S4096 D128, causal
  C3  INT8 K/V forward (integer-MFMA and dequant-exact) and fp16 at the same shape
  C4  mlaCompressed bf16 forward (latent 512 -> 16 heads x 128), S4096
  C5  fp16 fwd + bwd, D256, one GPU's shard (B=8 of 64, H=32, S=4096)
Prints one JSON object per config.  Usage: python tools/perf_suite.py [--only C2,C5] [--reps N]
"""
from __future__ import annotations

import argparse
import json
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))

PEAK = 256 * 4 * 1024 * 2.4e9 / 1e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="C2,C3,C4,C5,BWD128")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--c5-batch", type=int, default=8)
    args = ap.parse_args()
    only = set(args.only.split(","))
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    g = torch.Generator(device=dev)
    g.manual_seed(7)

    def uni(shape, dt):
        return ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25).to(dt)

    def time_it(fn, reps):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    def emit(name, **kw):
        print(json.dumps({"config": name, **kw}), flush=True)

    mha = mfa.MultiHeadAttention()
    if "C2" in only:
        B, H, S, D = 1, 16, 4096, 128
        q, k, v = (uni((B, H, S, D), torch.float16) for _ in range(3))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                            causal=True)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        for rnd in range(2):
            for var, stg in (("pair", "4"), ("pair", "2"), ("single", "0")):
                os.environ["MFA_FWD_VARIANT"] = var
                os.environ["MFA_FWD_PAIR"] = stg
                ms = time_it(lambda: mha.forward(desc, q, k, v, o, l, stream=stream),
                             args.reps * 5)
                f = mfa.attention_flops(B, H, S, S, D, causal=True)
                emit("C2", variant=var, pair_waves=stg, round=rnd, ms=round(ms, 4),
                     tflops=round(f / ms / 1e9, 1), frac=round(f / ms / 1e9 / PEAK, 4))
        os.environ.pop("MFA_FWD_VARIANT", None)
        os.environ.pop("MFA_FWD_PAIR", None)
        base_nc = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc_nc = mfa.MultiHeadDescriptor.make(base_nc, B, H, S, D)
        ms = time_it(lambda: mha.forward(desc_nc, q, k, v, o, l, stream=stream), args.reps * 5)
        f = mfa.attention_flops(B, H, S, S, D)
        emit("C2-noncausal", ms=round(ms, 4), tflops=round(f / ms / 1e9, 1))
        del q, k, v, o, l

    if "TUNE" in only:
        # A/B of attention_fwd_v2.hip scheduling knobs (MFA_FWD2_TUNE), interleaved rounds.
        B, H, S, D = 1, 16, 8192, 128
        q, k, v = (uni((B, H, S, D), torch.float16) for _ in range(3))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        f = mfa.attention_flops(B, H, S, S, D)
        res = {}
        for rnd in range(3):
            for tv in "012345":
                os.environ["MFA_FWD2_TUNE"] = tv
                ms = time_it(lambda: mha.forward(desc, q, k, v, o, l, stream=stream), args.reps)
                res.setdefault(tv, []).append(round(f / ms / 1e9, 1))
        os.environ.pop("MFA_FWD2_TUNE", None)
        for tv, r in res.items():
            emit("TUNE", variant=tv, tflops=r)
        del q, k, v, o, l

    if "C3" in only:
        B, H, S, D = 1, 16, 8192, 128
        qf = uni((B, H, S, D), torch.float16)
        kf, vf = uni((B, H, S, D), torch.float32), uni((B, H, S, D), torch.float32)
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        kq, ks, _, _ = mfa.quantize(kf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        vq, vs, _, _ = mfa.quantize(vf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        base = mfa.AttentionDescriptor.make(S, S, D, low_precision=True,
                                            precision=mfa.Precision.FP16)
        qa = mfa.QuantizedAttention()
        tq = mfa.quantized_tensor(qf, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=float(ks.item()))
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=float(vs.item()))
        f = mfa.attention_flops(B, H, S, S, D)
        for im in (True, False):
            qd = mfa.quantized_descriptor(base, mfa.Precision.FP16, mfa.Precision.INT8,
                                          mfa.Precision.INT8, B=B, H=H, integer_matmul=im)
            ms = time_it(lambda: qa.forward(qd, tq, tk, tv, o, l, stream=stream), args.reps)
            emit("C3", path="int8-mfma" if im else "int8-dequant-exact", ms=round(ms, 4),
                 tops=round(f / ms / 1e9, 1))
        kh, vh = kf.half(), vf.half()
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        ms = time_it(lambda: mha.forward(desc, qf, kh, vh, o, l, stream=stream), args.reps)
        emit("C3", path="fp16", ms=round(ms, 4), tflops=round(f / ms / 1e9, 1),
             frac=round(f / ms / 1e9 / PEAK, 4))
        del qf, kf, vf, o, l, kq, vq, kh, vh

    if "C4" in only:
        B, H, S, D, LAT = 1, 16, 4096, 128, 512
        lat = uni((B * S, LAT), torch.bfloat16)
        wk = (uni((LAT, H * D), torch.float32) * 0.176).to(torch.bfloat16)
        wv = (uni((LAT, H * D), torch.float32) * 0.176).to(torch.bfloat16)
        q = uni((B, H, S, D), torch.bfloat16)
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        kb = torch.empty((B * S, H * D), dtype=torch.bfloat16, device=dev)
        vb = torch.empty_like(kb)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)
        fn = lambda: mfa.mla_forward(base, lat, wk, wv, q, o, B, H, S, S, D, LAT,
                                     mfa.Precision.BF16, k_buf=kb, v_buf=vb, stream=stream)
        ms = time_it(fn, args.reps)
        f = 2 * (2 * B * S * LAT * H * D) + mfa.attention_flops(B, H, S, S, D)
        emit("C4", ms=round(ms, 4), tflops=round(f / ms / 1e9, 1),
             frac=round(f / ms / 1e9 / PEAK, 4))
        del lat, wk, wv, q, o, kb, vb

    for tag, D5 in (("C5", 256), ("BWD128", 128)):
      if tag not in only:
        continue
      if True:
        B, H, S, D = args.c5_batch, 32, 4096, D5
        q, k, v, do = (uni((B, H, S, D), torch.float16) for _ in range(4))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        dq, dk, dv = (torch.empty((B, H, S, D), dtype=torch.float32, device=dev) for _ in range(3))
        dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        ff = mfa.attention_flops(B, H, S, S, D)
        fb = mfa.attention_flops(B, H, S, S, D, kind="backward")
        reps = max(2, args.reps // 4)
        ms_f = time_it(lambda: mha.forward(desc, q, k, v, o, l, stream=stream), reps)
        ms_q = time_it(lambda: mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf,
                                            stream=stream, phase="query"), reps)
        ms_kv = time_it(lambda: mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf,
                                             stream=stream, phase="keyValue"), reps)
        emit(tag, batch=B, fwd_ms=round(ms_f, 3), fwd_tflops=round(ff / ms_f / 1e9, 1),
             bwdq_ms=round(ms_q, 3), bwdkv_ms=round(ms_kv, 3),
             bwd_tflops=round(fb / (ms_q + ms_kv) / 1e9, 1),
             fwdbwd_tflops=round((ff + fb) / (ms_f + ms_q + ms_kv) / 1e9, 1),
             frac=round((ff + fb) / (ms_f + ms_q + ms_kv) / 1e9 / PEAK, 4))


if __name__ == "__main__":
    main()
