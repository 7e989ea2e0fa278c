"""Which tile's P·V does the AGPR-owning forward get wrong? (development tool)"""
import os
import sys

import numpy as np

_R = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(_R, "tests"), os.path.join(_R, "metal-flash-attention-plus_amd", "python"), _R]
os.environ["MFA_FWD_AW"] = "1"
from test_forward_v2_gpu import FP16, gaussian  # noqa: E402
from harness import run_forward, seen  # noqa: E402

B, H, R, C = 1, 1, 512, 512
seed = R + 3 * C + 7 * B
Q = gaussian((B, H, R, 128), seed)
K, V = gaussian((B, H, C, 128), seed + 1), gaussian((B, H, C, 128), seed + 2)
o, l = run_forward(Q, K, V, prec=FP16, causal=True)
o = o.cpu().numpy()[0, 0].astype(np.float64)
q, k, v = (seen(x, FP16)[0, 0].astype(np.float64) for x in (Q, K, V))
s = q @ k.T / np.sqrt(128)
s[np.triu_indices(R, 1)] = -np.inf
p = np.exp(s - s.max(axis=1, keepdims=True))
lsum = p.sum(axis=1)
T = C // 64
def blk(t, q):
    return slice(64 * t + 16 * q, 64 * t + 16 * q + 16)
kk = k
for row in (384, 400, 430, 448, 500):
    r = o[row] * lsum[row] - p[row] @ v
    names, basis = [], []
    for q in range(4):
        for t in range(T):
            for q2 in range(4):
                for nm, src in (("V", v), ("K", kk)):
                    if nm == "K" and not (t == 3 or t == 2 or t == 4 or t == 5):
                        continue
                    names.append(f"P3q{q}{nm}{t}q{q2}"); basis.append(p[row, blk(3, q)] @ src[blk(t, q2)])
    B_ = np.stack(basis, axis=1)
    # sparse guess: greedy matching pursuit with 8 atoms
    res = r.copy(); chosen = []
    for it in range(8):
        sc = [abs(np.dot(res, b)) / np.linalg.norm(b) for b in basis]
        j = int(np.argmax(sc)); chosen.append(j)
        Bc = B_[:, chosen]
        al, *_ = np.linalg.lstsq(Bc, r, rcond=None)
        res = r - Bc @ al
    print(f"row {row}: unexplained {np.linalg.norm(res) / np.linalg.norm(r):.3f}; " + ", ".join(f"{names[j]} {a:+.2f}" for j, a in zip(chosen, al)))
