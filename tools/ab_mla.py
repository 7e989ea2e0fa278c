#!/usr/bin/env python3
"""Interleaved one-process A/B of an environment knob on the C4 MLA forward (decompression
GEMMs + attention), checked against the first arm at bf16 tolerance (development tool).
Usage: python tools/ab_mla.py VAR=a,b [--rounds N]"""
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
    ap.add_argument("--rounds", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    var, vals = a.knob.split("=")
    vals = vals.split(",")
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(3)
    u = lambda shape: ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25)
    B, H, S, D, LAT = 1, 16, 4096, 128, 512
    lat = u((B * S, LAT)).bfloat16()
    wk = (u((LAT, H * D)) * 0.176).bfloat16()
    wv = (u((LAT, H * D)) * 0.176).bfloat16()
    q = u((B, H, S, D)).bfloat16()
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    kb = torch.empty((B * S, H * D), dtype=torch.bfloat16, device=dev)
    vb = torch.empty_like(kb)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)
    run = lambda: mfa.mla_forward(base, lat, wk, wv, q, o, B, H, S, S, D, LAT, mfa.Precision.BF16,
                                  k_buf=kb, v_buf=vb)
    res = {x: [] for x in vals}
    ref = None
    for _ in range(a.rounds):
        for x in vals:
            os.environ[var] = x
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = (o.clone(), kb.clone(), vb.clone())
            else:
                for got, want in ((kb, ref[1]), (vb, ref[2]), (o, ref[0])):
                    assert torch.allclose(got.float(), want.float(), rtol=1e-2, atol=1e-3), \
                        f"{var}={x}: result differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[x].append(e0.elapsed_time(e1) / a.reps)
    print(json.dumps({"cfg": "C4", "knob": var,
                      **{x: {"ms_med": round(statistics.median(t), 4)} for x, t in res.items()}}))


if __name__ == "__main__":
    main()
