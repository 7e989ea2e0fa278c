#!/usr/bin/env python3
"""A/B of the split-KV decode kernels at decode shapes: the default routing against an
MFA_DECODE16 setting (argv[1], e.g. 2 = the 32-row kernel at D = 256, 0 = everywhere).
Per-call times from HIP events on one stream, best of 5 interleaved rounds of 20 calls, and
the K/V HBM rate.  Development tool: python tools/dec_ab.py 2"""
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision


def main():
    alt = sys.argv[1] if len(sys.argv) > 1 else "0"
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream()
    g = torch.Generator(device=dev).manual_seed(5)
    cases = [("B32 H16 R1 C8192 D256", 32, 16, 16, 1, 8192, 256),
             ("B8 H32/4 R1 C16384 D256", 8, 32, 4, 1, 16384, 256),
             ("B16 H16 R4 C8192 D256", 16, 16, 16, 4, 8192, 256),
             ("B32 H16 R1 C8192 D128", 32, 16, 16, 1, 8192, 128)]
    for kv in (P.INT8, P.INT4):
        for name, B, H, Hkv, R, C, D in cases:
            nb = D if kv == P.INT8 else D // 2
            q = ((torch.rand((B, H, R, D), generator=g, device=dev) * 2 - 1)).half()
            k = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
            v = torch.randint(0, 256, (B, Hkv, C, nb), generator=g, device=dev, dtype=torch.uint8)
            o = torch.empty((B, H, R, D), dtype=torch.float32, device=dev)
            l = torch.empty((B, H, R), dtype=torch.float16, device=dev)
            base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=P.FP16)
            desc = mfa.quantized_descriptor(base, P.FP16, kv, kv, B=B, H=H, Hkv=Hkv)
            tq = mfa.quantized_tensor(q, P.FP16)
            tk = mfa.quantized_tensor(k, kv, scale=0.01)
            tv = mfa.quantized_tensor(v, kv, scale=0.01)
            qa = mfa.QuantizedAttention()
            byts = 2.0 * B * Hkv * C * nb

            def setv(a):
                if a:
                    os.environ["MFA_DECODE16"] = alt
                else:
                    os.environ.pop("MFA_DECODE16", None)

            res = {False: [], True: []}
            plans = {}
            with torch.cuda.stream(st):
                for a in (False, True):
                    setv(a)
                    plans[a] = [r["name"] for r in mfa.quantized_plan(desc, mfa.KernelType.forward, tq, tk, tv)]
                    for _ in range(5):
                        qa.forward(desc, tq, tk, tv, o, l, stream=st)
                torch.cuda.synchronize()
                for _ in range(5):
                    for a in (False, True):
                        setv(a)
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        for _ in range(20):
                            qa.forward(desc, tq, tk, tv, o, l, stream=st)
                        e1.record(st)
                        torch.cuda.synchronize()
                        res[a].append(e0.elapsed_time(e1) / 20)
            setv(False)
            x, y = min(res[False]), min(res[True])
            print(f"{'INT8' if kv == P.INT8 else 'INT4'} {name:24s} default {x * 1e3:7.1f} us "
                  f"({byts / x / 1e6:6.0f} GB/s)  alt {y * 1e3:7.1f} us ({byts / y / 1e6:6.0f} GB/s)  "
                  f"ratio {y / x:.3f}  {plans[False][0]} | {plans[True][0]}", flush=True)
            del q, k, v, o, l


if __name__ == "__main__":
    main()
