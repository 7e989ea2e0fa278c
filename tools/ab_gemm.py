#!/usr/bin/env python3
"""One-process A/B of a GEMM environment knob (development tool): times mfa.gemm on an
M x N x K 16-bit NN problem for each value, interleaved, and checks bit-identity with the first.
Usage: python tools/ab_gemm.py VAR=a,b [--mnk M,N,K] [--bf16]"""
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
    ap.add_argument("--mnk", default="4096,4096,4096")
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    var, vals = a.knob.split("=")
    vals = vals.split(",")
    import torch
    import mfa_amd as mfa
    P = mfa.Precision
    M, N, K = (int(x) for x in a.mnk.split(","))
    dt, pr = (torch.bfloat16, P.BF16) if a.bf16 else (torch.float16, P.FP16)
    g = torch.Generator(device="cuda").manual_seed(3)
    x = (torch.rand((M, K), generator=g, device="cuda") - 0.5).to(dt)
    w = (torch.rand((K, N), generator=g, device="cuda") - 0.5).to(dt)
    c = torch.empty((M, N), device="cuda", dtype=dt)
    run = lambda: mfa.gemm(x, w, c, M, N, K, pr, pr)
    ref = None
    res = {v: [] for v in vals}
    for _ in range(a.rounds):
        for v in vals:
            os.environ[var] = v
            run()
            torch.cuda.synchronize()
            if ref is None:
                ref = c.clone()
            else:
                assert torch.equal(c, ref), f"{var}={v} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.reps)
    flop = 2.0 * M * N * K
    print(json.dumps({"mnk": a.mnk, "knob": var, **{v: {"ms_med": round(statistics.median(t), 4),
                      "tflops": round(flop / statistics.median(t) / 1e9, 1)} for v, t in res.items()}}))


if __name__ == "__main__":
    main()
