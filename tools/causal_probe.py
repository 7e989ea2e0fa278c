#!/usr/bin/env python3
"""Where the causal C2 forward loses against non-causal (development tool).

Times the fp16 D128 forward over shapes and variants in interleaved rounds and prints the
per-shape TFLOP/s.  Usage: python tools/causal_probe.py
"""
import json
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))


def main():
    import torch
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream(dev).cuda_stream
    mha = mfa.MultiHeadAttention()
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    shapes = [(1, 16, 4096), (1, 16, 8192), (1, 64, 4096), (4, 16, 4096), (1, 16, 2048)]
    bufs = {}
    for B, H, S in shapes:
        D = 128
        q, k, v = (((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1) * 0.25).half()
                   for _ in range(3))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        bufs[(B, H, S)] = (q, k, v, o, l)
    res = {}
    for rnd in range(3):
        for (B, H, S), (q, k, v, o, l) in bufs.items():
            for causal in (True, False):
                for var in ("pair", "single"):
                    os.environ["MFA_FWD_VARIANT"] = var
                    base = mfa.AttentionDescriptor.make(low_precision=True,
                                                        precision=mfa.Precision.FP16,
                                                        causal=causal)
                    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, 128)
                    fn = lambda: mha.forward(desc, q, k, v, o, l, stream=stream)
                    for _ in range(20):
                        fn()
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    n = 40
                    e0.record()
                    for _ in range(n):
                        fn()
                    e1.record()
                    torch.cuda.synchronize()
                    ms = e0.elapsed_time(e1) / n
                    f = mfa.attention_flops(B, H, S, S, 128, causal=causal)
                    res.setdefault((B, H, S, causal, var), []).append(
                        (round(ms * 1e3, 1), round(f / ms / 1e9, 1)))
    os.environ.pop("MFA_FWD_VARIANT", None)
    for key, r in res.items():
        B, H, S, causal, var = key
        print(json.dumps({"B": B, "H": H, "S": S, "causal": causal, "variant": var,
                          "us": [x[0] for x in r], "tflops": [x[1] for x in r]}), flush=True)


if __name__ == "__main__":
    main()
