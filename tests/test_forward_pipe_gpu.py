"""GPU parity of the software-pipelined fp16 forward (attention_fwd_pipe.hip, hand-placed blocks
from tools/gen_fwd_pipe.py): against the CPU oracle at the reference's mixed tolerances (O 5e-3
on unit gaussians, L 7e-3 + half an fp16 ulp; SquareAttentionTest.swift:557-571), and against
the compiler-scheduled shared-tile kernel on identical inputs.  The pipeline carries S(t+1)
across the step boundary and rescales it there, so the lazy-rescale branch gets the same forced
inputs as the v2 kernel's tests: a spike at the first, a middle and the last tile, and a ramp
that rescales on every tile.  Every case asserts that the pipelined kernel is what ran."""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
from harness import maxerr, run_forward
from test_forward_v2_gpu import check, gaussian

pytestmark = pytest.mark.gpu
FP16 = mfa.Precision.FP16


class env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def launched():
    return [r["name"] for r in mfa.last_launches()]


PIPE = dict(MFA_FWD_PIPE=1, MFA_FWD_SHARE=1)


def check_pipe(Q, K, V, **kw):
    with env(**PIPE):
        mfa.last_launches()
        o, l = check(Q, K, V, FP16, **kw)
        assert launched()[-1].startswith("mfa_fwd_pipe_kernel"), launched()
    return o, l


CASES = [
    # B, H, Hkv, R, C, D
    (1, 2, 2, 256, 256, 128),
    (1, 2, 2, 384, 300, 128),    # odd block count (group 1 of the last pair has no rows)
    (1, 2, 2, 200, 333, 128),    # C off the tile grid: the last tile is edge-masked
    (1, 2, 2, 256, 64, 128),     # one key tile (no steady step)
    (1, 2, 2, 256, 128, 128),    # two key tiles
    (1, 2, 2, 256, 192, 128),    # three (an odd tile count)
    (2, 4, 2, 512, 512, 128),    # GQA, B = 2
    (1, 2, 2, 256, 256, 96),     # D below the padded width
    (1, 3, 3, 129, 1000, 128),
]


@pytest.mark.parametrize("case", CASES)
def test_pipe_vs_oracle(gpu, case):
    B, H, Hkv, R, C, D = case
    seed = R + 3 * C + D
    Q = gaussian((B, H, R, D), seed)
    K, V = gaussian((B, Hkv, C, D), seed + 1), gaussian((B, Hkv, C, D), seed + 2)
    check_pipe(Q, K, V)


@pytest.mark.parametrize("spike_key", [0, 70, 200, 255])
def test_pipe_forced_rescale(gpu, spike_key):
    B, H, S, D = 1, 2, 256, 128
    Q = gaussian((B, H, S, D), 7, 0.3)
    K = gaussian((B, H, S, D), 8, 0.3)
    V = gaussian((B, H, S, D), 9)
    direction = np.ones(D, dtype=np.float32) / np.sqrt(D)
    Q += 2.0 * direction
    K[:, :, spike_key] = 20.0 * direction
    check_pipe(Q, K, V, tol_o=5e-3)


def test_pipe_rescale_every_tile(gpu):
    B, H, S, D = 1, 1, 512, 128
    Q = np.zeros((B, H, S, D), dtype=np.float32)
    Q[..., 0] = 1.0
    K = gaussian((B, H, S, D), 11, 0.05)
    K[..., 0] = np.linspace(0.0, 120.0, S, dtype=np.float32)
    V = gaussian((B, H, S, D), 12)
    check_pipe(Q, K, V, tol_o=5e-3, tol_l=2e-2)


@pytest.mark.parametrize("spike_key", [None, 0, 1000])
def test_pipe_matches_shared_tile_kernel(gpu, spike_key):
    # The same staged tiles, the same arithmetic per element and the row sums in the same order
    # (fwd2_exp's, split across the two blocks): bit-identical O and L to the compiler-scheduled
    # shared-tile kernel, also when a rescale recomputes the speculative exponentials.
    B, H, S, D = 1, 4, 2048, 128
    Q, K, V = (gaussian((B, H, S, D), 50 + i) for i in range(3))
    if spike_key is not None:
        direction = np.ones(D, dtype=np.float32) / np.sqrt(D)
        Q += 2.0 * direction
        K[:, :, spike_key] = 20.0 * direction
    with env(**PIPE):
        mfa.last_launches()
        o1, l1 = run_forward(Q, K, V, prec=FP16)
        assert launched()[-1].startswith("mfa_fwd_pipe_kernel")
    with env(MFA_FWD_SHARE=1, MFA_FWD_PIPE=0):
        mfa.last_launches()
        o0, l0 = run_forward(Q, K, V, prec=FP16)
        assert launched()[-1].startswith("mfa_fwd2_share_kernel")
    assert torch.equal(o1, o0) and torch.equal(l1, l0)


def test_pipe_c3_heads(gpu):
    # BASELINE configs[2]'s fp16 shape (H16 S8192 D128) against a float64 restatement.
    B, H, S, D = 1, 16, 8192, 128
    g = torch.Generator(device="cuda:0").manual_seed(9)
    q, k, v = ((torch.rand((B, H, S, D), generator=g, device="cuda:0") * 2 - 1).half()
               for _ in range(3))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    l = torch.empty((B, H, S), dtype=torch.float16, device="cuda:0")
    with env(MFA_FWD_PIPE=1):
        mfa.last_launches()
        mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
        torch.cuda.synchronize()
        assert launched()[-1].startswith("mfa_fwd_pipe_kernel")
    for hh in (0, 9):
        Qd, Kd, Vd = (t[0, hh].double() for t in (q, k, v))
        s = (Qd @ Kd.T) / np.sqrt(D)
        m = s.max(dim=1, keepdim=True).values
        p = torch.exp(s - m)
        ref_o = (p @ Vd) / p.sum(dim=1, keepdim=True)
        ref_l = (m.squeeze(1) + torch.log(p.sum(dim=1))) / np.log(2)
        assert (o[0, hh].double() - ref_o).abs().max().item() <= 5e-3
        assert (l[0, hh].double() - ref_l).abs().max().item() <= 7e-3 + 4e-3
