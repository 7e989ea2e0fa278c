"""Per-row-group error of the AGPR-owning forward against the oracle (development tool)."""
import os
import sys

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_R, "tests"), os.path.join(_R, "metal-flash-attention-plus_amd", "python"), _R]
os.environ["MFA_FWD_AW"] = "1"
from test_forward_v2_gpu import FP16, gaussian  # noqa: E402
from harness import run_forward, seen  # noqa: E402
import oracle_lib as ol  # noqa: E402

for (B, H, R, C, causal) in [(1, 1, 512, 512, True), (1, 1, 512, 440, True), (1, 1, 512, 400, True)]:
    seed = R + 3 * C + 7 * B
    Q = gaussian((B, H, R, 128), seed)
    K, V = gaussian((B, H, C, 128), seed + 1), gaussian((B, H, C, 128), seed + 2)
    o, l = run_forward(Q, K, V, prec=FP16, causal=causal)
    ref = ol.attention(seen(Q, FP16), seen(K, FP16), seen(V, FP16), causal=causal)
    err = np.abs(o.cpu().numpy() - ref["O"]).max(axis=-1)[0, 0]
    el = np.abs(l.float().cpu().numpy() - ref["L"])[0, 0]
    print(f"R={R} C={C}")
    print("  O: " + " ".join(f"{x:.0e}" if x > 5e-3 else "." for x in err.reshape(-1, 16).max(axis=1)))
    print("  L: " + " ".join(f"{x:.0e}" if x > 1e-2 else "." for x in el.reshape(-1, 16).max(axis=1)))
    # Ratio test: is the wrong O a scaled version of the right one?
    rows = np.where(err > 5e-3)[0]
    if len(rows):
        r = rows[0]
        a, b_ = o.cpu().numpy()[0, 0, r], ref["O"][0, 0, r]
        print(f"  row {r}: o/ref median {np.median(a / b_):.4f} corr {np.corrcoef(a, b_)[0, 1]:.4f}")
