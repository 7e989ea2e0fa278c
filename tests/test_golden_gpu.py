"""GPU parity against the committed golden fixtures (tests/golden/, made by make_golden.py from
the CPU oracle on the reference's own input generators), through the C ABI.

Tolerances are the reference's (SquareAttentionTest.swift:558-570): FP32 O/L/D/dQ/dK/dV 2e-5
absolute; mixed FP16 O 5e-2, L 7e-3, D 1e-1, gradients 5e-2.  Quantiser outputs are bit-exact."""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
from harness import maxerr, run_forward, to_device
from test_backward_gpu import run_backward

pytestmark = pytest.mark.gpu
P = mfa.Precision
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.mark.parametrize("name,causal", [("c1_fp32_s128_d64.npz", False),
                                         ("causal_fp32_b2h2_s96_d32.npz", True)])
def test_fp32_forward_backward_matches_golden(gpu, name, causal):
    g = load(name)
    r = run_backward(g["Q"], g["K"], g["V"], g["dO"], P.FP32, causal=causal)
    for k in ("O", "L", "D", "dQ", "dK", "dV"):
        assert maxerr(r[k], g[k]) <= 2e-5, k


@pytest.mark.parametrize("prec", [P.FP16, P.BF16])
def test_mixed_forward_backward_matches_golden(gpu, prec):
    g = load("c1_fp32_s128_d64.npz")
    r = run_backward(g["Q"], g["K"], g["V"], g["dO"], prec)
    tol = {"O": 5e-2, "L": 7e-3, "D": 1e-1, "dQ": 5e-2, "dK": 5e-2, "dV": 5e-2}
    for k, t in tol.items():
        assert maxerr(r[k], g[k]) <= t, k


def test_window_cross_attention_matches_golden(gpu):
    g = load("window_fp32_r80_c112_d32_w24.npz")
    o, l = run_forward(g["Q"], g["K"], g["V"], P.FP32, window=24)
    assert maxerr(o, g["O"]) <= 2e-5 and maxerr(l, g["L"]) <= 2e-5


def test_runtime_quantizer_matches_golden_bytes(gpu):
    g = load("quant_stream_s32_d16.npz")
    for name in ("Q", "K", "V"):
        x = torch.from_numpy(g[name]).to("cuda:0")
        for prec, tag in ((P.INT8, "i8"), (P.INT4, "i4")):
            data, scale, _, _ = mfa.quantize(x, prec, rows=32, cols=16)
            torch.cuda.synchronize()
            assert scale.item() == g[f"{name}_{tag}_scale"][0]
            assert np.array_equal(data.cpu().numpy(), g[f"{name}_{tag}"])


def test_quantized_forward_matches_golden(gpu):
    g = load("quant_stream_s32_d16.npz")
    desc = mfa.quantized_descriptor(mfa.AttentionDescriptor.make(32, 32, 16), P.INT8, P.INT8,
                                    P.INT8)
    dev = "cuda:0"
    keep = []

    def qt(name):
        d = torch.from_numpy(g[f"{name}_i8"]).to(dev)
        keep.append(d)
        return mfa.quantized_tensor(d, P.INT8, scale=float(g[f"{name}_i8_scale"][0]))

    o = torch.full((1, 1, 32, 16), float("nan"), dtype=torch.float32, device=dev)
    mfa.QuantizedAttention().forward(desc, qt("Q"), qt("K"), qt("V"), o)
    torch.cuda.synchronize()
    assert maxerr(o, g["O_deq_i8"]) <= 2e-3  # dequant-exact
    err = np.linalg.norm(o.cpu().numpy() - g["O_fp32"]) / np.linalg.norm(g["O_fp32"])
    assert err < 0.25  # QuantizedAttentionTest.swift:519-520


def test_blockwise_quantizer_matches_golden(gpu):
    g = load("blockwise_i8_32x32_bs8.npz")
    x = torch.from_numpy(g["x"]).to("cuda:0")
    data, _, sc, _ = mfa.quantize(x, P.INT8, mfa.QuantMode.blockwise, 32, 32, 8)
    torch.cuda.synchronize()
    assert np.array_equal(sc.cpu().numpy(), g["scales"])
    assert np.array_equal(data.cpu().numpy(), g["q"])
