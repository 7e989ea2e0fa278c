#!/usr/bin/env python3
"""A/B of the on-load quantised forward (attention_fwd_kv8.hip; causal: the mirrored shared-tile
kernel's on-load instantiation) against the dequantisation pass
+ 16-bit kernel path (MFA_KV8=0), per-tensor INT8 / INT4 K/V, at the C3 shape (FP16 and BF16
Q), D = 64 and the C5 shape (D = 256).  Prints per-launch-sequence times from HIP events on one
stream, best of 5 rounds, interleaved.  Development tool: python tools/kv8_ab.py"""
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

import numpy as np
import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision


def main():
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream()
    g = torch.Generator(device=dev).manual_seed(3)
    cases = [("C3 fp16", 1, 16, 8192, 128, P.FP16, False), ("C3 bf16", 1, 16, 8192, 128, P.BF16, False),
             ("D64 fp16", 1, 32, 8192, 64, P.FP16, False), ("C5 fp16", 2, 32, 4096, 256, P.FP16, False),
             ("C5 bf16", 2, 32, 4096, 256, P.BF16, False),
             ("C2c fp16", 1, 16, 4096, 128, P.FP16, True), ("C2c bf16", 1, 16, 4096, 128, P.BF16, True),
             ("S8kc fp16", 1, 16, 8192, 128, P.FP16, True),
             ("D64c fp16", 1, 32, 8192, 64, P.FP16, True), ("C5c fp16", 2, 32, 4096, 256, P.FP16, True),
             ("C5c bf16", 2, 32, 4096, 256, P.BF16, True), ("B4c fp16", 4, 32, 4096, 128, P.FP16, True),
             ("S8kw fp16", 1, 16, 8192, 128, P.FP16, False, 1024),
             ("C5w bf16", 2, 32, 4096, 256, P.BF16, False, 512)]
    # --bw BS: block-wise K/V scales of block size BS (round 6), on load vs the pass (MFA_KV8_BW).
    bw = 0
    if "--bw" in sys.argv:
        i = sys.argv.index("--bw")
        bw = int(sys.argv[i + 1])
        del sys.argv[i:i + 2]
    knob = "MFA_KV8_BW" if bw else "MFA_KV8"
    if len(sys.argv) > 1:
        cases = [c for c in cases if any(c[0].startswith(x) for x in sys.argv[1].split(","))]
    for kv in (P.INT8, P.INT4):
        for name, B, H, S, D, qp, causal, *win in cases:
            win = win[0] if win else None
            tdt = torch.float16 if qp == P.FP16 else torch.bfloat16
            q = ((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1)).to(tdt)
            nb = D if kv == P.INT8 else D // 2
            k = torch.randint(0, 256, (B, H, S, nb), generator=g, device=dev, dtype=torch.uint8)
            v = torch.randint(0, 256, (B, H, S, nb), generator=g, device=dev, dtype=torch.uint8)
            o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
            l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
            base = mfa.AttentionDescriptor.make(S, S, D, causal=causal, window=win, low_precision=True,
                                                precision=qp)
            desc = mfa.quantized_descriptor(base, qp, kv, kv, B=B, H=H)
            tq = mfa.quantized_tensor(q, qp)
            tk = mfa.quantized_tensor(k, kv, scale=0.01)
            tv = mfa.quantized_tensor(v, kv, scale=0.01)
            if bw:
                nbl = ((B * H * S + bw - 1) // bw) * ((D + bw - 1) // bw)
                scs = [torch.rand(nbl, generator=g, device=dev) * 0.01 + 0.005 for _ in range(2)]
                for t, sc in ((tk, scs[0]), (tv, scs[1])):
                    t.block_scales, t.block_size = sc.data_ptr(), bw
            qa = mfa.QuantizedAttention()
            r = np.arange(S)
            lo = np.maximum(0, r - win) if win is not None else np.zeros(S, dtype=np.int64)
            hi = np.minimum(S - 1, r) if causal else np.full(S, S - 1)
            fl = 4.0 * B * H * D * float(np.maximum(hi - lo + 1, 0).sum())

            def run(onload):
                if onload and bw:
                    os.environ[knob] = "1"  # (block-wise: on load only when forced at these sizes)
                elif onload:
                    os.environ.pop(knob, None)
                else:
                    os.environ[knob] = "0"
                qa.forward(desc, tq, tk, tv, o, l, stream=st)

            res = {True: [], False: []}
            plans = {}
            with torch.cuda.stream(st):
                for onload in (True, False):
                    for _ in range(3):
                        run(onload)
                    if onload and bw:
                        os.environ[knob] = "1"
                    elif onload:
                        os.environ.pop(knob, None)
                    else:
                        os.environ[knob] = "0"
                    plans[onload] = [r["name"] for r in mfa.quantized_plan(desc, mfa.KernelType.forward,
                                                                           tq, tk, tv)]
                torch.cuda.synchronize()
                n = 10
                for _ in range(5):
                    for onload in (True, False):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        run(onload)
                        e0.record(st)
                        for _ in range(n):
                            run(onload)
                        e1.record(st)
                        torch.cuda.synchronize()
                        res[onload].append(e0.elapsed_time(e1) / n)
            os.environ.pop(knob, None)
            a, b = min(res[True]), min(res[False])
            print(f"{'INT8' if kv == P.INT8 else 'INT4'} {name:9s} on-load {a * 1e3:8.1f} us "
                  f"({fl / a / 1e9:7.1f} TF)  pass {b * 1e3:8.1f} us ({fl / b / 1e9:7.1f} TF)  "
                  f"ratio {b / a:.3f}  on-load plan {plans[True]}  pass plan {plans[False]}",
                  flush=True)
            del q, k, v, o, l


if __name__ == "__main__":
    main()
