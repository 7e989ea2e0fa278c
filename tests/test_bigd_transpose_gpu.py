"""GPU parity for what the reference boundary accepts beyond D <= 256 and dense layouts.

* Head dimension > 256: the reference's parameter tables end at 384 and fall back to their
  last row for any larger D (AttentionDescriptor+Parameters.swift:44-69, :116, :142; README
  "infinite head dimension", :96-104).  Forward, backwardQuery and backwardKeyValue at
  D in {288, 320, 384, 512} against the oracle at the reference's tolerances
  (SquareAttentionTest.swift:557-571: FP32 2e-5; mixed O 5e-2, L 7e-3, D 1e-1, gradients 5e-2).
* Transposed operands: createTransposeState maps transposeState.O to O and dO, Q/K/V to
  dQ/dK/dV (AttentionDescriptor.swift:150-165); a transposed operand is column-major within a
  head (leadingDimension = sequence length, AttentionKernel.swift:299-313).
  RectangularAttentionTest.swift:5-29 draws random transpose states; here every state of the
  16 is run through forward + backward against the oracle.
"""
import itertools

import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, seen, to_device

pytestmark = pytest.mark.gpu
FP32, FP16, BF16 = mfa.Precision.FP32, mfa.Precision.FP16, mfa.Precision.BF16
DEV = "cuda:0"


def gaussian(shape, seed, amp=1.0):
    return (np.random.default_rng(seed).standard_normal(shape) * amp).astype(np.float32)


def colmajor(x):
    """[B, H, S, D] -> the transposed in-memory layout [B, H, D, S] (column-major per head)."""
    return np.ascontiguousarray(np.swapaxes(x, 2, 3))


def run(Q, K, V, dO, prec, tr=(False, False, False, False), causal=False, window=None):
    """Forward + backward through the C ABI with the operands laid out per `tr`
    (transpose Q, K, V, O); returns every output in BHSD order."""
    B, H, R, D = Q.shape
    Hkv, C = K.shape[1], K.shape[2]
    lp = prec != FP32
    base = mfa.AttentionDescriptor.make(low_precision=lp, precision=prec if lp else None,
                                        causal=causal, window=window, transpose=tr)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, R, D, Hkv=Hkv, C=C)
    lay = lambda x, t: to_device(colmajor(x) if t else x, prec)
    q, k, v = lay(Q, tr[0]), lay(K, tr[1]), lay(V, tr[2])
    do = lay(dO, tr[3])
    o = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device=DEV)
    l = torch.full((B, H, R), float("nan"), dtype=torch.float16 if lp else torch.float32,
                   device=DEV)
    dbuf = torch.full((B, H, R), float("nan"), dtype=torch.bfloat16 if lp else torch.float32,
                      device=DEV)
    dq = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device=DEV)
    dk = torch.full((B, Hkv, C, D), float("nan"), dtype=torch.float32, device=DEV)
    dv = torch.full((B, Hkv, C, D), float("nan"), dtype=torch.float32, device=DEV)
    mha = mfa.MultiHeadAttention()
    mha.forward(desc, q, k, v, o, l)
    mha.backward(desc, q, k, v, o, do, l, dq, dk, dv, dbuf)
    torch.cuda.synchronize()

    def back(t, transposed, S):
        a = t.cpu().numpy()
        if transposed:  # memory [B, H, D, S]
            a = np.swapaxes(a.reshape(a.shape[0], a.shape[1], D, S), 2, 3)
        return a

    return {"O": back(o, tr[3], R), "L": l.float().cpu().numpy(), "D": dbuf.float().cpu().numpy(),
            "dQ": back(dq, tr[0], R), "dK": back(dk, tr[1], C), "dV": back(dv, tr[2], C)}


def check(got, ref, prec, S):
    if prec == FP32:
        tol = {"O": 2e-5, "L": 2e-5, "D": 2e-5, "dQ": 2e-5, "dK": 2e-5, "dV": 2e-5}
        tol = {k: v * max(1.0, S / 64) for k, v in tol.items()}
    else:
        # L is stored in FP16: the reference's 7e-3 plus half an FP16 ulp of |L|.
        lt = 7e-3 + 2.0 ** -11 * float(np.abs(ref["L"]).max())
        tol = {"O": 5e-2, "L": lt, "D": 1e-1, "dQ": 5e-2, "dK": 5e-2, "dV": 5e-2}
    for name, t in tol.items():
        g = got[name]
        assert np.isfinite(g).all(), f"{name} has non-finite values"
        e = maxerr(g, ref[name])
        assert e <= t, f"{name} max error {e:.3e} > {t:.3e}"


@pytest.mark.parametrize("D", [288, 320, 384, 512])
@pytest.mark.parametrize("prec", [FP32, FP16, BF16])
def test_large_head_dimension_fwd_bwd(gpu, D, prec):
    B, H, S = 1, 2, 130
    amp = 1.0 if prec == FP32 else 0.5
    Q, K, V, dO = (gaussian((B, H, S, D), 700 + i, amp) for i in range(4))
    got = run(Q, K, V, dO, prec)
    ref = ol.attention(seen(Q, prec), seen(K, prec), seen(V, prec), dO=seen(dO, prec))
    check(got, ref, prec, S)


@pytest.mark.parametrize("prec", [FP32, FP16])
@pytest.mark.parametrize("R,C,Hkv,causal,window", [
    (200, 200, 2, True, None),     # causal, GQA group of 2
    (96, 300, 4, False, None),     # cross-attention
    (260, 260, 1, False, 70),      # MQA, sliding window
])
def test_large_head_dimension_masks_gqa(gpu, prec, R, C, Hkv, causal, window):
    B, H, D = 1, 4, 384
    Q, dO = gaussian((B, H, R, D), 710, 0.5), gaussian((B, H, R, D), 711, 0.5)
    K, V = gaussian((B, Hkv, C, D), 712, 0.5), gaussian((B, Hkv, C, D), 713, 0.5)
    got = run(Q, K, V, dO, prec, causal=causal, window=window)
    ref = ol.attention(seen(Q, prec), seen(K, prec), seen(V, prec), dO=seen(dO, prec),
                       causal=causal, window=window)
    check(got, ref, prec, max(R, C))


ALL_TRANSPOSES = list(itertools.product([False, True], repeat=4))


@pytest.mark.parametrize("tr", ALL_TRANSPOSES, ids=lambda t: "".join("T" if x else "N" for x in t))
def test_transposes_fwd_bwd_fp32(gpu, tr):
    # RectangularAttentionTest shapes are rectangular (R != C): Q/O/dO/dQ over R, K/V over C.
    B, H, R, C, D = 1, 2, 77, 131, 40
    Q, dO = gaussian((B, H, R, D), 720), gaussian((B, H, R, D), 721)
    K, V = gaussian((B, H, C, D), 722), gaussian((B, H, C, D), 723)
    got = run(Q, K, V, dO, FP32, tr=tr)
    ref = ol.attention(Q, K, V, dO=dO)
    check(got, ref, FP32, max(R, C))


@pytest.mark.parametrize("tr", [(True, True, True, True), (False, False, False, True),
                                (True, False, True, False)],
                         ids=lambda t: "".join("T" if x else "N" for x in t))
@pytest.mark.parametrize("prec,D", [(FP16, 128), (BF16, 64), (FP16, 256), (FP16, 320)])
def test_transposes_fwd_bwd_mixed(gpu, tr, prec, D):
    B, H, S = 1, 2, 200
    Q, K, V, dO = (gaussian((B, H, S, D), 730 + i, 0.5) for i in range(4))
    got = run(Q, K, V, dO, prec, tr=tr, causal=True)
    ref = ol.attention(seen(Q, prec), seen(K, prec), seen(V, prec), dO=seen(dO, prec), causal=True)
    check(got, ref, prec, S)


def test_transposed_equals_dense_bitwise(gpu):
    """The generic kernels read strided operands element-wise: the same values in the
    transposed layout give bit-identical O and gradients to the dense layout on the same
    kernels (dense operands at an unaligned head dimension keep both on the generic path)."""
    B, H, S, D = 1, 2, 150, 36
    Q, K, V, dO = (gaussian((B, H, S, D), 740 + i) for i in range(4))
    a = run(Q, K, V, dO, FP32)
    b = run(Q, K, V, dO, FP32, tr=(True, True, True, True))
    for name in ("O", "L", "D", "dQ", "dK", "dV"):
        assert np.array_equal(a[name], b[name]), name


def quantize_host(x, prec):
    s = ol.quant_scale_tensor(x, int(prec))
    q = ol.quantize(x, int(prec), s)
    return q, s, ol.dequantize(q, x.size, int(prec), s).reshape(x.shape)


@pytest.mark.parametrize("R", [1, 16, 300])
@pytest.mark.parametrize("kv", [mfa.Precision.INT8, mfa.Precision.INT4])
def test_large_head_dimension_quantized(gpu, R, kv):
    """QuantizedAttention forward + backward with INT8 / INT4 K/V at D = 384 (decode and
    prefill row counts): dequant-exact against the oracle on the dequantised values."""
    B, H, C, D = 1, 2, 257, 384
    Q, dO = gaussian((B, H, R, D), 750, 0.5), gaussian((B, H, R, D), 751, 0.5)
    K, V = gaussian((B, H, C, D), 752), gaussian((B, H, C, D), 753)
    kq, ks, kd = quantize_host(K, kv)
    vq, vs, vd = quantize_host(V, kv)
    Qd, dOd = seen(Q, FP16), seen(dO, FP16)
    ref = ol.attention(Qd, kd, vd, dO=dOd)
    base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=FP16)
    desc = mfa.quantized_descriptor(base, FP16, kv, kv, B=B, H=H)
    kt = torch.from_numpy(kq).to(DEV)
    vt = torch.from_numpy(vq).to(DEV)
    tq = mfa.quantized_tensor(to_device(Q, FP16), FP16)
    tk = mfa.quantized_tensor(kt, kv, scale=ks)
    tv = mfa.quantized_tensor(vt, kv, scale=vs)
    o = torch.full((B, H, R, D), float("nan"), dtype=torch.float32, device=DEV)
    l = torch.empty((B, H, R), dtype=torch.float16, device=DEV)
    qa = mfa.QuantizedAttention()
    qa.forward(desc, tq, tk, tv, o, l)
    do = to_device(dO, FP16)
    dq = torch.empty((B, H, R, D), dtype=torch.float32, device=DEV)
    dk, dv = (torch.empty((B, H, C, D), dtype=torch.float32, device=DEV) for _ in range(2))
    dvals = torch.empty((B, H, R), dtype=torch.bfloat16, device=DEV)
    qa.backwardQuery(desc, tq, tk, tv, o, do, l, dq, dvals)
    qa.backwardKeyValue(desc, tq, tk, tv, do, l, dvals, dk, dv)
    torch.cuda.synchronize()
    assert maxerr(o, ref["O"]) < 2e-2
    assert maxerr(l, ref["L"]) < 7e-3 + 2.0 ** -11 * float(np.abs(ref["L"]).max())
    for name, t in (("dQ", dq), ("dK", dk), ("dV", dv)):
        assert maxerr(t, ref[name]) < 5e-2, name
