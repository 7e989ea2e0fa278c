#!/usr/bin/env python3
"""Debug the pp forward on a tiny case: per-row L and O error against the oracle (development)."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "metal-flash-attention-plus_amd", "python"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
import mfa_amd as mfa
import oracle_lib as ol
from harness import run_forward, seen

os.environ["MFA_FWD_PP"] = "1"
B, H, S, D = 1, 1, int(sys.argv[1]) if len(sys.argv) > 1 else 256, 128
causal = len(sys.argv) > 2 and sys.argv[2] == "1"
rng = np.random.default_rng(1)
Q, K, V = (rng.standard_normal((B, H, S, D)).astype(np.float32) for _ in range(3))
P = mfa.Precision.FP16
o, l = run_forward(Q, K, V, prec=P, causal=causal)
print([r["name"] for r in mfa.last_launches()])
ref = ol.attention(seen(Q, P), seen(K, P), seen(V, P), causal=causal)
on, ln = o.cpu().numpy()[0, 0], l.float().cpu().numpy()[0, 0]
ro, rl = ref["O"][0, 0], ref["L"][0, 0]
for r in list(range(0, S, 16)) + [S - 1]:
    print(f"row {r:4d} L {ln[r]:10.3f} ref {rl[r]:10.3f}  O err {np.abs(on[r] - ro[r]).max():.3e}  O[0:3] {on[r, :3]} ref {ro[r, :3]}")
