#!/usr/bin/env python3
"""One-process A/B of backward-kernel knobs (development tool): times MultiHeadAttention.backward
(backwardQuery + backwardKeyValue) on a C5 slice for each value of an environment knob,
interleaved, and checks dQ/dK/dV bit-identical to the first value.
Usage: python tools/ab_bwd.py VAR=a,b [--shape B,H,S,D] [--rounds N]"""
import argparse
import json
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "metal-flash-attention-plus_amd", "python"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("knob")
    ap.add_argument("--shape", default="2,32,4096,256")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    var, vals = a.knob.split("=")
    vals = vals.split(",")
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    B, H, S, D = (int(x) for x in a.shape.split(","))
    g = torch.Generator(device=dev).manual_seed(5)
    q, k, v, do = (((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1) * 0.25).half()
                   for _ in range(4))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    mha = mfa.MultiHeadAttention()
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    mha.forward(desc, q, k, v, o, l)
    dq, dk, dv = (torch.empty((B, H, S, D), dtype=torch.float32, device=dev) for _ in range(3))
    dd = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
    run = lambda: mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dd)
    flop = 14 * D * S * S * B * H
    ref = None
    res = {x: [] for x in vals}
    for _ in range(a.rounds):
        for x in vals:
            os.environ[var] = x
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = (dq.clone(), dk.clone(), dv.clone())
            else:
                assert all(torch.equal(t, r) for t, r in zip((dq, dk, dv), ref)), f"{var}={x} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[x].append(e0.elapsed_time(e1) / a.reps)
    out = {x: {"ms_med": round(statistics.median(t), 4),
               "tflops_14D": round(flop / statistics.median(t) / 1e9, 1)} for x, t in res.items()}
    print(json.dumps({"shape": a.shape, "knob": var, **out}))


if __name__ == "__main__":
    main()
