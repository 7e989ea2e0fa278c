"""CPU: the oracle reproduces the committed golden fixtures (tests/golden/make_golden.py), and an
independent float64 numpy restatement agrees with them — the fixtures are the frozen checker
values the GPU parity tests (test_golden_gpu.py) compare against."""
import os

import numpy as np
import pytest

import oracle_lib as ol

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
LOG2E = 1.4426950408889634


def load(name):
    with np.load(os.path.join(GOLD, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def numpy_attention(Q, K, V, causal=False, window=None, dO=None):
    """Float64 restatement of Network.swift's naive attention (L in log2 units, D scaled)."""
    Q, K, V = (x.astype(np.float64) for x in (Q, K, V))
    scale = 1.0 / np.sqrt(Q.shape[-1])
    S = np.einsum("bhrd,bhcd->bhrc", Q, K)
    R, C = S.shape[-2:]
    r = np.arange(R)[:, None]
    c = np.arange(C)[None, :]
    masked = np.zeros((R, C), dtype=bool)
    if causal:
        masked |= c > r
    if window is not None:
        masked |= r > c + window
    S = np.where(masked, -np.inf, S * scale)
    m = S.max(-1, keepdims=True)
    P = np.exp(S - m)
    l = P.sum(-1, keepdims=True)
    P /= l
    out = {"O": np.einsum("bhrc,bhcd->bhrd", P, V), "L": (m + np.log(l))[..., 0] * LOG2E}
    if dO is not None:
        dO = dO.astype(np.float64)
        Dn = (dO * out["O"]).sum(-1)
        dP = np.einsum("bhrd,bhcd->bhrc", dO, V)
        dS = P * (dP - Dn[..., None])
        out["D"] = Dn * scale
        out["dV"] = np.einsum("bhrc,bhrd->bhcd", P, dO)
        out["dQ"] = np.einsum("bhrc,bhcd->bhrd", dS, K) * scale
        out["dK"] = np.einsum("bhrc,bhrd->bhcd", dS, Q) * scale
    return out


@pytest.mark.parametrize("name,kw", [("c1_fp32_s128_d64.npz", {}),
                                     ("causal_fp32_b2h2_s96_d32.npz", {"causal": True})])
def test_oracle_reproduces_attention_fixtures(name, kw):
    g = load(name)
    r = ol.attention(g["Q"], g["K"], g["V"], dO=g["dO"], **kw)
    for k in ("O", "L", "D", "dQ", "dK", "dV"):
        assert np.array_equal(r[k], g[k]), k
    n = numpy_attention(g["Q"], g["K"], g["V"], dO=g["dO"], **kw)
    for k in ("O", "L", "D", "dQ", "dK", "dV"):
        assert np.max(np.abs(n[k] - g[k])) < 1e-6, k


def test_oracle_reproduces_window_fixture():
    g = load("window_fp32_r80_c112_d32_w24.npz")
    r = ol.attention(g["Q"], g["K"], g["V"], window=24)
    assert np.array_equal(r["O"], g["O"]) and np.array_equal(r["L"], g["L"])
    n = numpy_attention(g["Q"], g["K"], g["V"], window=24)
    assert np.max(np.abs(n["O"] - g["O"])) < 1e-6


def test_quant_stream_fixture():
    g = load("quant_stream_s32_d16.npz")
    s = ol.LCGStream(0x5EED5EED)
    for name in ("Q", "K", "V"):
        x = s.draw(32 * 16).reshape(1, 1, 32, 16)
        assert np.array_equal(x, g[name])
        for prec, tag in ((ol.INT8, "i8"), (ol.INT4, "i4")):
            sc = ol.quant_scale_tensor(x, prec)
            assert np.float32(sc) == g[f"{name}_{tag}_scale"][0]
            assert np.array_equal(ol.quantize(x, prec, sc), g[f"{name}_{tag}"])
    # The reference's INT8 gate (QuantizedAttentionTest.swift:519-520) holds on the fixture.
    err = np.linalg.norm(g["O_deq_i8"] - g["O_fp32"]) / np.linalg.norm(g["O_fp32"])
    assert err < 0.25


def test_blockwise_fixture():
    g = load("blockwise_i8_32x32_bs8.npz")
    sc = ol.quant_scales_block(g["x"], 32, 32, 8, ol.INT8)
    assert np.array_equal(sc, g["scales"])
    assert np.array_equal(ol.quantize_block(g["x"], 32, 8, ol.INT8, sc), g["q"])
