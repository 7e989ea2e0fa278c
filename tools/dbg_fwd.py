"""Debug: forward L/O error vs oracle for each kernel variant (development tool)."""
import os, sys
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import conftest  # noqa: F401
import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, run_forward, seen

def g(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)
for (R, C, D, causal) in [(200, 200, 128, False), (256, 256, 128, False), (300, 300, 128, True), (200, 200, 64, False)]:
    Q = g((1, 2, R, D), R); K = g((1, 2, C, D), C); V = g((1, 2, C, D), C + 1)
    P = mfa.Precision.FP16
    ref = ol.attention(seen(Q, P), seen(K, P), seen(V, P), causal=causal)
    out = []
    for var, env in (("pair", {"MFA_FWD_VARIANT": "pair"}), ("single", {"MFA_FWD_VARIANT": "single"}),
                     ("gen1", {"MFA_FWD_GEN": "1"})):
        for k, v in env.items():
            os.environ[k] = v
        o, l = run_forward(Q, K, V, prec=P, causal=causal)
        for k in env:
            os.environ.pop(k)
        lf = l.float().cpu().numpy()
        out.append(f"{var}: O {maxerr(o, ref['O']):.2e} L {maxerr(lf, ref['L']):.2e} Lraw-vs-ref-rounded {np.abs(lf - ref['L'].astype(np.float16).astype(np.float32)).max():.2e}")
    print((R, C, D, causal), " | ".join(out), flush=True)
