#!/usr/bin/env python3
"""Interleaved one-process A/B of an environment knob on the Hadamard rotation of a 1 GiB fp32
buffer, block 128 (the bench's row), with a bit-identity check (development tool).
Usage: python tools/ab_had.py VAR=a,b [--rounds N]"""
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
    ap.add_argument("--rounds", type=int, default=8)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--n", type=int, default=128)
    a = ap.parse_args()
    var, vals = a.knob.split("=")
    vals = vals.split(",")
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    x0 = torch.rand((1 << 28,), device=dev) - 0.5
    x = x0.clone()
    rot = mfa.HadamardRotation()
    res = {v: [] for v in vals}
    ref = None
    for _ in range(a.rounds):
        for v in vals:
            os.environ[var] = v
            x.copy_(x0)
            rot.rotate(x, a.n, (1 << 28) // a.n)
            torch.cuda.synchronize()
            if ref is None:
                ref = x.clone()
            else:
                assert torch.equal(x, ref), f"{var}={v} differs"
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                rot.rotate(x, a.n, (1 << 28) // a.n)
            e1.record()
            torch.cuda.synchronize()
            res[v].append(e0.elapsed_time(e1) / a.reps)
    print(json.dumps({"cfg": f"hadamard 1GiB n{a.n}", "knob": var,
                      **{v: {"ms_med": round(statistics.median(t), 4),
                             "GBps": round(8 * (1 << 28) / statistics.median(t) / 1e6, 1)}
                         for v, t in res.items()}}))


if __name__ == "__main__":
    main()
