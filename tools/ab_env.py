"""One-process A/B of library environment knobs on a bench workload (development tool).

Usage: python tools/ab_env.py WORKLOAD VAR=a,b,c [VAR2=x,y] — times each setting by HIP
events (median of 5 rounds of 20 launches), interleaving settings round by round.
WORKLOAD: c3_int8_exact | c3_fp16 | c2 | sparse (the bench's block-sparse row) |
bwd256[_amask] | bwd128[_amask] (backwardKeyValue with or without an additive mask).  A value "-"
unsets the variable (the library default).
"""
import itertools
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import statistics
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402


def workload(name, dev="cuda:0"):
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    u = lambda shape, dt: ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25).to(dt)
    stream = torch.cuda.current_stream().cuda_stream
    if name.startswith("c3"):
        B, H, S, D = 1, 16, 8192, 128
        q = u((B, H, S, D), torch.float16)
        kf, vf = u((B, H, S, D), torch.float32), u((B, H, S, D), torch.float32)
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        base = mfa.AttentionDescriptor.make(S, S, D, low_precision=True, precision=mfa.Precision.FP16)
        flops = mfa.attention_flops(B, H, S, S, D)
        if name == "c3_fp16":
            desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
            kh, vh = kf.half(), vf.half()
            return (lambda: mfa.MultiHeadAttention().forward(desc, q, kh, vh, o, l, stream=stream)), flops
        kq, ks, _, _ = mfa.quantize(kf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        vq, vs, _, _ = mfa.quantize(vf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        qd = mfa.quantized_descriptor(base, mfa.Precision.FP16, mfa.Precision.INT8, mfa.Precision.INT8, B=B, H=H)
        tq = mfa.quantized_tensor(q, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=float(ks.item()))
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=float(vs.item()))
        qa = mfa.QuantizedAttention()
        return (lambda: qa.forward(qd, tq, tk, tv, o, l, stream=stream)), flops
    if name == "c2":
        B, H, S, D = 1, 16, 4096, 128
        q, k, v = (u((B, H, S, D), torch.float16) for _ in range(3))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16, causal=True)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        return (lambda: mfa.MultiHeadAttention().forward(desc, q, k, v, o, l, stream=stream)), \
            mfa.attention_flops(B, H, S, S, D, causal=True)
    if name == "sparse":
        import numpy as np
        B, H, S, D, blk, band = 1, 16, 4096, 128, 128, 8
        nb = S // blk
        pat = np.zeros((nb, nb), dtype=np.uint8)
        for i in range(nb):
            c0 = min(max(0, i - band // 2), nb - band)
            pat[i, c0:c0 + band] = 1
        rb = np.zeros((nb, 2), dtype=np.uint32)
        mfa.lib.mfa_sparse_build_block_sparse(pat.ctypes.data, nb, nb, blk, rb.ctypes.data)
        rows = np.ascontiguousarray(np.broadcast_to(np.repeat(rb, blk, axis=0), (B, H, S, 2)))
        mask = torch.from_numpy(rows.view(np.int32)).to(dev)
        q, k, v = (u((B, H, S, D), torch.float16) for _ in range(3))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                            sparse_mask=mfa.MaskType.sparseRanges)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        pairs = int((rows[0, 0, :, 1].astype(np.int64) - rows[0, 0, :, 0]).sum()) * B * H
        return (lambda: mfa.MultiHeadAttention().forward(desc, q, k, v, o, l, mask=mask,
                                                         stream=stream)), 4.0 * D * pairs
    if name.startswith("bwd256") or name.startswith("bwd128"):
        # backwardKeyValue at D = 256 / 128 with an additive mask (bwd*_amask) or none: 4 GEMMs
        # per tile.
        B, H, S, D = 1, 16, 2048, int(name[3:6])
        q, k, v, do = (u((B, H, S, D), torch.float16) for _ in range(4))
        name_ = name[:-2] if name.endswith("_q") else name
        mask = u((B, H, S, S), torch.float32) if name_.endswith("_amask") else None
        if name_.endswith("_ranges"):  # every key in range: the mask path with no amask traffic
            import numpy as np
            rows = np.zeros((B, H, S, 2), dtype=np.uint32)
            rows[..., 1] = S
            mask = torch.from_numpy(rows.view(np.int32)).to(dev)
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        dbuf = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
        dq, dk, dv = (torch.empty((B, H, S, D), dtype=torch.float32, device=dev) for _ in range(3))
        base = mfa.AttentionDescriptor.make(
            low_precision=True, precision=mfa.Precision.FP16,
            sparse_mask=mfa.MaskType.sparseRanges if name_.endswith("_ranges") else None)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        mha = mfa.MultiHeadAttention()
        mha.forward(desc, q, k, v, o, l, mask=mask, stream=stream)
        mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf, mask=mask, phase="query",
                     stream=stream)
        ph = "query" if name.endswith("_q") else "keyValue"  # *_q: the query phase (3 GEMMs)
        return (lambda: mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf, mask=mask,
                                     phase=ph, stream=stream)), \
            (6.0 if ph == "query" else 8.0) * B * H * S * S * D
    if name in ("qbwdq256", "qbwdq128"):
        # QuantizedAttention.backwardQuery, INT8 K/V per-tensor + fp16 Q/dO, B2 H32 S4096.
        B, H, S, D = 2, 32, 4096, int(name[5:])
        q, do = (u((B, H, S, D), torch.float16) for _ in range(2))
        kf, vf = u((B, H, S, D), torch.float32), u((B, H, S, D), torch.float32)
        kq, ks, _, _ = mfa.quantize(kf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        vq, vs, _, _ = mfa.quantize(vf, mfa.Precision.INT8, rows=B * H * S, cols=D)
        base = mfa.AttentionDescriptor.make(S, S, D, low_precision=True, precision=mfa.Precision.FP16)
        qd = mfa.quantized_descriptor(base, mfa.Precision.FP16, mfa.Precision.INT8, mfa.Precision.INT8, B=B, H=H)
        tq = mfa.quantized_tensor(q, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=float(ks.item()))
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=float(vs.item()))
        o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
        dq = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
        dvals = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
        qa = mfa.QuantizedAttention()
        qa.forward(qd, tq, tk, tv, o, l, stream=stream)
        return (lambda: qa.backwardQuery(qd, tq, tk, tv, o, do, l, dq, dvals, stream=stream)), \
            6.0 * B * H * S * S * D
    raise SystemExit(f"unknown workload {name}")


def main():
    name = sys.argv[1]
    axes = []
    for a in sys.argv[2:]:
        k, vals = a.split("=", 1)
        axes.append([(k, v) for v in vals.split(",")])
    settings = list(itertools.product(*axes)) or [()]
    fn, flops = workload(name)
    times = {s: [] for s in settings}
    for _ in range(60):
        fn()
    torch.cuda.synchronize()
    for _ in range(5):
        for s in settings:
            for k, v in s:
                if v == "-":
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            for _ in range(5):
                fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            e1.synchronize()
            times[s].append(e0.elapsed_time(e1) / 20)
    for s in settings:
        ms = statistics.median(times[s])
        print(f"{name} {' '.join(f'{k}={v}' for k, v in s) or '(default)'}: {ms * 1e3:.1f} us "
              f"{flops / ms / 1e9:.1f} TFLOPS", flush=True)


if __name__ == "__main__":
    main()
