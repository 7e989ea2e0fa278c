#!/usr/bin/env python3
"""Block-sparse backward cost model (development tool): times both backward phases on the
bench's banded buildBlockSparse ranges (B1 H16 S4096 D128, 128x128 blocks) at several band
widths, plus the dense (no-mask) phases, so the time per phase splits into a fixed part and a
part per kept block.  Usage: python tools/sparse_bwd_probe.py [bands, e.g. 2,4,8,16,32]"""
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
import sys

import numpy as np
import torch

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
import mfa_amd as mfa  # noqa: E402


def main():
    bands = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "2,4,8,16,32").split(",")]
    dev = torch.device("cuda:0")
    B, H, S, D, blk = 1, 16, 4096, 128, 128
    nb = S // blk
    g = torch.Generator(device=dev).manual_seed(5)
    u = lambda: ((torch.rand((B, H, S, D), generator=g, device=dev) * 2 - 1) * 0.25).half()
    q, k, v, do = u(), u(), u(), u()
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    dq, dk, dv = (torch.empty_like(o) for _ in range(3))
    db = torch.empty((B, H, S), dtype=torch.bfloat16, device=dev)
    mha = mfa.MultiHeadAttention()
    st = torch.cuda.Stream()

    def ev(fn, n=30):
        for _ in range(5):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(3):
            e0.record(st)
            for _ in range(n):
                fn()
            e1.record(st)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / n)
        return best * 1e3  # us

    with torch.cuda.stream(st):
        base_d = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc_d = mfa.MultiHeadDescriptor.make(base_d, B, H, S, D)
        mha.forward(desc_d, q, k, v, o, l, stream=st)
        for ph in ("query", "keyValue"):
            t = ev(lambda: mha.backward(desc_d, q, k, v, o, do, l, dq, dk, dv, db, stream=st, phase=ph))
            mfa.last_launches()
            mha.backward(desc_d, q, k, v, o, do, l, dq, dk, dv, db, stream=st, phase=ph)
            print(f"dense {ph:9s} {t:8.1f} us  {[r['name'] for r in mfa.last_launches()]}")
        for band in bands:
            pat = np.zeros((nb, nb), dtype=np.uint8)
            for i in range(nb):
                c0 = min(max(0, i - band // 2), nb - band)
                pat[i, c0:c0 + band] = 1
            rb = np.zeros((nb, 2), dtype=np.uint32)
            mfa.lib.mfa_sparse_build_block_sparse(pat.ctypes.data, nb, nb, blk, rb.ctypes.data)
            rows = np.ascontiguousarray(np.broadcast_to(np.repeat(rb, blk, axis=0), (B, H, S, 2)))
            mask = torch.from_numpy(rows.view(np.int32)).to(dev)
            base_s = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                                  sparse_mask=mfa.MaskType.sparseRanges)
            desc_s = mfa.MultiHeadDescriptor.make(base_s, B, H, S, D)
            mha.forward(desc_s, q, k, v, o, l, mask=mask, stream=st)
            res = []
            for ph in ("query", "keyValue"):
                t = ev(lambda: mha.backward(desc_s, q, k, v, o, do, l, dq, dk, dv, db, mask=mask,
                                            stream=st, phase=ph))
                res.append(t)
            print(f"band {band:2d} (density {band / nb:.3f}): query {res[0]:8.1f} us  "
                  f"keyValue {res[1]:8.1f} us  sum {sum(res):8.1f}")


if __name__ == "__main__":
    main()
