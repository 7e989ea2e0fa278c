#!/usr/bin/env python3
"""Timings of the §8(f) kernels on one GPU (HIP events on the launch stream): the general GEMM
(transposed / mixed-precision GEMMDescriptor cases) and the Hadamard rotation."""
import json
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision
DT = {P.FP32: torch.float32, P.FP16: torch.float16, P.BF16: torch.bfloat16}


def timeit(fn, iters=20, warm=5):
    for _ in range(warm):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    out = {}
    n = 4096
    for pa, pb, ta, tb in [(P.FP16, P.FP16, 0, 0), (P.FP16, P.FP16, 0, 1), (P.FP16, P.FP16, 1, 0),
                           (P.BF16, P.BF16, 1, 1), (P.FP32, P.FP32, 0, 0), (P.FP16, P.FP32, 0, 0)]:
        a = torch.randn(n, n, device="cuda").to(DT[pa])
        b = torch.randn(n, n, device="cuda").to(DT[pb])
        c = torch.empty(n, n, device="cuda", dtype=torch.float32)
        ms = timeit(lambda: mfa.gemm(a, b, c, n, n, n, pa, P.FP32, prec_b=pb, transpose_a=ta,
                                     transpose_b=tb))
        key = f"gemm_{pa.name}x{pb.name}_{'T' if ta else 'N'}{'T' if tb else 'N'}_{n}"
        out[key] = {"ms": round(ms, 4), "tflops": round(2 * n ** 3 / ms / 1e9, 1)}
    # MLA: decompress path vs absorbed (latent-space) path, C4 prefill and a decode shape.
    for (B, H, Sq, Skv) in [(1, 16, 4096, 4096), (32, 16, 1, 4096), (8, 16, 16, 8192)]:
        D, lat = 128, 512
        bf = torch.bfloat16
        latent = torch.randn(B * Skv, lat, device="cuda").to(bf)
        wk = (torch.randn(lat, H * D, device="cuda") * lat ** -0.5).to(bf)
        wv = (torch.randn(lat, H * D, device="cuda") * lat ** -0.5).to(bf)
        q = torch.randn(B, H, Sq, D, device="cuda").to(bf)
        o = torch.empty(B, H, Sq, D, device="cuda")
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.BF16)
        args = (base, latent, wk, wv, q, o, B, H, Sq, Skv, D, lat, P.BF16)
        t_dec = timeit(lambda: mfa.mla_forward(*args))
        t_abs = timeit(lambda: mfa.mla_forward_absorbed(*args))
        out[f"mla_B{B}_H{H}_Sq{Sq}_Skv{Skv}"] = {"decompress_ms": round(t_dec, 4),
                                                 "absorbed_ms": round(t_abs, 4)}
    nb, bs = 1 << 18, 1024
    x = torch.randn(nb, bs, device="cuda")
    hr = mfa.HadamardRotation()
    for bs_ in (16, 128, 1024):
        ms = timeit(lambda: hr.rotate(x, bs_, nb * bs // bs_))
        out[f"hadamard_bs{bs_}_1GiB"] = {"ms": round(ms, 4), "GB/s": round(8 * nb * bs / ms / 1e6, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
