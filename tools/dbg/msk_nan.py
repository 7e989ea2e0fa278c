"""Debug: where the masked tuned backward leaves non-finite dK/dV on fully masked rows."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, "metal-flash-attention-plus_amd/python")
sys.path.insert(0, "tests")
import mfa_amd as mfa
from harness import to_device
FP16 = mfa.Precision.FP16
B, H, R, C, D = 1, 2, 130, 190, 128
g = lambda shape, s: np.random.default_rng(s).standard_normal(shape).astype(np.float32) * 0.5
Q, dO, K, V = g((B, H, R, D), 80), g((B, H, R, D), 81), g((B, H, C, D), 82), g((B, H, C, D), 83)
lo = (np.arange(R) % C).astype(np.uint32)
hi = np.minimum(lo + 50, C).astype(np.uint32)
if os.environ.get("EMPTY", "1") == "1":
    hi[5::9] = lo[5::9]
ranges = np.ascontiguousarray(np.broadcast_to(np.stack([lo, hi], -1), (B, H, R, 2)))
lpi = os.environ.get("LPI", "0") == "1"
base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, low_precision_intermediates=lpi,
                                    sparse_mask=mfa.MaskType.sparseRanges)
desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D, C=C)
dev = "cuda:0"
q, k, v, do = (to_device(x, FP16) for x in (Q, K, V, dO))
mask = torch.from_numpy(ranges.view(np.int32)).to(dev)
o = torch.empty((B, H, R, D), dtype=torch.float32, device=dev)
l = torch.empty((B, H, R), dtype=torch.float16 if lpi else torch.float32, device=dev)
dbuf = torch.full((B, H, R), float("nan"), dtype=torch.bfloat16 if lpi else torch.float32, device=dev)
dq, dk, dv = (torch.full((B, H, n, D), float("nan"), dtype=torch.float32, device=dev) for n in (R, C, C))
mha = mfa.MultiHeadAttention()
mha.forward(desc, q, k, v, o, l, mask=mask)
torch.cuda.synchronize()
print("L empty rows", l[0, :, 5::9].float().cpu().numpy()[:, :4], "O finite", bool(torch.isfinite(o).all()))
mfa.last_launches()
mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf, mask=mask)
torch.cuda.synchronize()
print([x["name"] for x in mfa.last_launches()])
print("D finite", bool(torch.isfinite(dbuf.float()).all()))
for n, t in (("dQ", dq), ("dK", dk), ("dV", dv)):
    a = t.cpu().numpy()
    bad = ~np.isfinite(a).all(axis=-1)
    print(n, "nonfinite rows per head:", [np.nonzero(bad[0, h])[0].tolist()[:20] for h in range(H)],
          "count", int(bad.sum()))
