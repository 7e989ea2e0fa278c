#!/usr/bin/env python3
"""A/B of the quantised backwardQuery: the tuned kernel on the stored K/V bytes (LDS byte ring,
kv_bytes.h) against the dequantisation pass + the same kernel on the dense copy
(MFA_BWDQ_BYTES=0), per-tensor INT8 / INT4 K/V, FP16 Q/dO, non-causal, at D = 256 (the C5-like
int8_fwd_bwd_d256 shape) and D = 128.  Best of 5 interleaved rounds of HIP-event timing on one
stream.  Development tool: python tools/qbwd_ab.py"""
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402

P = mfa.Precision


def main():
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream()
    g = torch.Generator(device=dev).manual_seed(4)
    for kv in (P.INT8, P.INT4):
        for B, H, S, D in ((2, 32, 4096, 256), (4, 32, 4096, 128)):
            u = lambda: ((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1) * 0.5).half()
            q, do = u(), u()
            nb = D if kv == P.INT8 else D // 2
            k = torch.randint(0, 256, (B, H, S, nb), generator=g, device=dev, dtype=torch.uint8)
            v = torch.randint(0, 256, (B, H, S, nb), generator=g, device=dev, dtype=torch.uint8)
            o = u().float()
            l = torch.full((B, H, S), 8.0, dtype=torch.float16, device=dev)
            dq = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
            dv_ = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
            base = mfa.AttentionDescriptor.make(S, S, D, low_precision=True, precision=P.FP16)
            desc = mfa.quantized_descriptor(base, P.FP16, kv, kv, B=B, H=H)
            tq = mfa.quantized_tensor(q, P.FP16)
            tk = mfa.quantized_tensor(k, kv, scale=0.01)
            tv = mfa.quantized_tensor(v, kv, scale=0.01)
            qa = mfa.QuantizedAttention()
            fl = 6.0 * B * H * S * S * D  # the phase's 3 GEMMs

            modes = {True: {"MFA_BWDQ_BYTES": "1"}, False: {"MFA_BWDQ_BYTES": "0"}}

            def setmode(onload):
                os.environ.update(modes[onload])

            def run():
                qa.backwardQuery(desc, tq, tk, tv, o, do, l, dq, dv_, stream=st)

            res = {m: [] for m in modes}
            plans = {}
            with torch.cuda.stream(st):
                for onload in modes:
                    setmode(onload)
                    for _ in range(3):
                        run()
                    plans[onload] = [r["name"] for r in mfa.quantized_plan(
                        desc, mfa.KernelType.backwardQuery, tq, tk, tv)]
                torch.cuda.synchronize()
                n = 5
                for _ in range(5):
                    for onload in modes:
                        setmode(onload)
                        run()
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(st)
                        for _ in range(n):
                            run()
                        e1.record(st)
                        torch.cuda.synchronize()
                        res[onload].append(e0.elapsed_time(e1) / n)
            os.environ.pop("MFA_BWDQ_BYTES", None)
            a, b = min(res[True]), min(res[False])
            print(f"{'INT8' if kv == P.INT8 else 'INT4'} B{B} H{H} S{S} D{D}: on-load {a * 1e3:8.1f} us "
                  f"({fl / a / 1e9:7.1f} TF)  pass {b * 1e3:8.1f} us ({fl / b / 1e9:7.1f} TF)  "
                  f"pass/on-load {b / a:.3f}  {plans[True]} | {plans[False]}", flush=True)
            del q, do, k, v, o, l, dq, dv_


if __name__ == "__main__":
    main()
