"""Debug: fast vs generic backward error table (development tool)."""
import os, sys
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import conftest  # noqa: F401  (sys.path setup)
import mfa_amd as mfa
from test_backward_gpu import run_backward

def g(shape, seed):
    return (np.random.default_rng(seed).standard_normal(shape) * 0.5).astype(np.float32)

for (B, H, Hkv, R, C, D, causal) in [(1,1,1,64,64,64,False),(1,1,1,128,128,64,False),(1,1,1,64,128,64,False),
                                      (1,1,1,128,64,64,False),(1,1,1,256,256,128,False),(1,1,1,64,64,256,False),(1,1,1,64,64,128,True)]:
    Q, dO = g((B,H,R,D), 1), g((B,H,R,D), 2)
    K, V = g((B,Hkv,C,D), 3), g((B,Hkv,C,D), 4)
    fast = run_backward(Q, K, V, dO, mfa.Precision.FP16, causal=causal)
    os.environ["MFA_DISABLE_FAST"] = "1"
    gen = run_backward(Q, K, V, dO, mfa.Precision.FP16, causal=causal)
    os.environ.pop("MFA_DISABLE_FAST")
    out = []
    for n in ("dQ", "dK", "dV", "D"):
        a = fast[n].float().cpu().numpy(); b = gen[n].float().cpu().numpy()
        out.append(f"{n}: {np.abs(a-b).max():.3g}/{np.abs(b).max():.3g}")
    print((R, C, D, causal), "  ".join(out), flush=True)
    if (R, C, D) == (64, 64, 64):
        a = fast["dV"].cpu().numpy()[0,0]; b = gen["dV"].cpu().numpy()[0,0]
        bad = np.argwhere(np.abs(a-b) > 1e-2)
        print("bad dV idx (key, d) first 20:", bad[:20].tolist(), "count", len(bad))
