"""GPU parity for the absorbed MLA path (mfa_mla_forward_absorbed: attention in the latent
space).  The reference has no absorbed kernel and no MLA test (parity
unpinned for MLA); the pins are
  * the oracle on the exact decompressed K = latent·W_k, V = latent·W_v (fp32, no rounding),
  * the decompress path mfa_mla_forward on the same inputs (the row it must match
    "within tolerance", §8f).
The two GPU paths round different intermediates to the 16-bit precision (Q̃ and Õ here, K and
V there), so they agree to that precision, not bit for bit.  Tolerances: the reference's mixed
precision O tolerance 5e-2 (SquareAttentionTest.swift:558-563) for FP16, 1e-1 for BF16 (8-bit
mantissa, as tests/test_mla_gpu.py)."""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, relerr, seen, to_device

pytestmark = pytest.mark.gpu
P = mfa.Precision
DEV = "cuda:0"


def make_inputs(B, H, Sq, Skv, D, latent, prec, seed):
    rng = np.random.default_rng(seed)
    lat = seen(rng.standard_normal((B * Skv, latent)).astype(np.float32), prec)
    s = np.sqrt(1.0 / latent)
    wk = seen((rng.standard_normal((latent, H * D)) * s).astype(np.float32), prec)
    wv = seen((rng.standard_normal((latent, H * D)) * s).astype(np.float32), prec)
    Q = seen(rng.standard_normal((B, H, Sq, D)).astype(np.float32), prec)
    return lat, wk, wv, Q


def run_both(B, H, Sq, Skv, D, latent, prec, causal, seed=0):
    lat, wk, wv, Q = make_inputs(B, H, Sq, Skv, D, latent, prec, seed)
    dl, dk, dv, dq = (to_device(x, prec) for x in (lat, wk, wv, Q))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec, causal=causal)
    outs = []
    for fn in (mfa.mla_forward_absorbed, mfa.mla_forward):
        o = torch.full((B, H, Sq, D), float("nan"), dtype=torch.float32, device=DEV)
        l = torch.full((B, H, Sq), float("nan"), dtype=torch.float16, device=DEV)
        fn(base, dl, dk, dv, dq, o, B, H, Sq, Skv, D, latent, prec, logsumexp=l)
        torch.cuda.synchronize()
        outs.append((o, l))
    return outs, (lat, wk, wv, Q)


def bhsd(x, B, S, H, D):
    return np.ascontiguousarray(x.reshape(B, S, H, D).transpose(0, 2, 1, 3))


@pytest.mark.parametrize("prec", [P.FP16, P.BF16])
@pytest.mark.parametrize("latent", [256, 512])
@pytest.mark.parametrize("causal", [False, True])
def test_absorbed_matches_oracle_and_decompress(gpu, prec, latent, causal):
    B, H, S, D = 2, 4, 200, 64
    ((oa, la), (od, ld)), (lat, wk, wv, Q) = run_both(B, H, S, S, D, latent, prec, causal)
    K = bhsd(ol.gemm(lat, wk), B, S, H, D)
    V = bhsd(ol.gemm(lat, wv), B, S, H, D)
    ref = ol.attention(Q, K, V, causal=causal)
    tol = 5e-2 if prec == P.FP16 else 1e-1
    assert torch.isfinite(oa).all()
    assert maxerr(oa, ref["O"]) < tol
    assert maxerr(oa, od) < tol
    # L (FP16 storage): the reference's 7e-3 plus the storage rounding and the 16-bit Q̃.
    assert maxerr(la, ref["L"]) < (3e-2 if prec == P.FP16 else 1e-1)


@pytest.mark.parametrize("Sq,Skv", [(1, 300), (5, 1000), (33, 70)])
def test_absorbed_decode_shapes(gpu, Sq, Skv):
    # Decode-shaped queries (the case absorption is for): few query rows, long latent cache.
    B, H, D, latent, prec = 2, 16, 128, 512, P.BF16
    ((oa, _), (od, _)), (lat, wk, wv, Q) = run_both(B, H, Sq, Skv, D, latent, prec, False, seed=9)
    K = bhsd(ol.gemm(lat, wk), B, Skv, H, D)
    V = bhsd(ol.gemm(lat, wv), B, Skv, H, D)
    ref = ol.attention(Q, K, V)
    assert maxerr(oa, ref["O"]) < 1e-1
    assert relerr(oa, od) < 2e-2


@pytest.mark.parametrize("B,D", [(6, 64), (5, 192), (9, 128)])
def test_absorbed_decode_batch_groups(gpu, B, D):
    # The split-KV merge combines 4 batch items per workgroup and projects through W_v in
    # 128-dim chunks: batch counts that are not multiples of 4, and D > 128.
    H, Sq, Skv, latent, prec = 4, 1, 1500, 512, P.BF16
    ((oa, _), (od, _)), (lat, wk, wv, Q) = run_both(B, H, Sq, Skv, D, latent, prec, False, seed=B)
    K = bhsd(ol.gemm(lat, wk), B, Skv, H, D)
    V = bhsd(ol.gemm(lat, wv), B, Skv, H, D)
    ref = ol.attention(Q, K, V)
    assert maxerr(oa, ref["O"]) < 1e-1
    assert relerr(oa, od) < 2e-2


def test_absorbed_config4(gpu):
    # BASELINE.json configs[3] shape (H16 assumed): both GPU paths agree; one head
    # against the oracle on the exact decompressed K/V.
    B, H, S, D, latent, prec = 1, 16, 4096, 128, 512, P.BF16
    ((oa, la), (od, ld)), (lat, wk, wv, Q) = run_both(B, H, S, S, D, latent, prec, False, seed=4)
    assert relerr(oa, od) < 2e-2
    assert maxerr(la, ld) < 5e-2
    h = 5
    K = bhsd(ol.gemm(lat, wk), B, S, H, D)[:, h:h + 1]
    V = bhsd(ol.gemm(lat, wv), B, S, H, D)[:, h:h + 1]
    ref = ol.attention(Q[:, h:h + 1], K, V)
    assert maxerr(oa[:, h:h + 1], ref["O"]) < 2e-2


def test_absorbed_rejects_unsupported(gpu):
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.FP16)
    x = torch.zeros(16, dtype=torch.float16, device=DEV)
    o = torch.zeros(16, dtype=torch.float32, device=DEV)
    with pytest.raises(mfa.MFAError, match="latent dimension"):
        mfa.mla_forward_absorbed(base, x, x, x, x, o, 1, 1, 1, 1, 8, 96, P.FP16)


@pytest.mark.parametrize("causal", [False, True])
def test_absorbed_split_kv_causal(gpu, causal):
    # Few query blocks (B1 H2 S1024 -> 64 blocks): the keys are split over 8 workgroups per
    # block and merged (flash-decoding); causal splits beyond a block's last key stay empty.
    B, H, S, D, latent, prec = 1, 2, 1024, 64, 256, P.FP16
    ((oa, la), (od, ld)), (lat, wk, wv, Q) = run_both(B, H, S, S, D, latent, prec, causal, seed=2)
    K = bhsd(ol.gemm(lat, wk), B, S, H, D)
    V = bhsd(ol.gemm(lat, wv), B, S, H, D)
    ref = ol.attention(Q, K, V, causal=causal)
    assert maxerr(oa, ref["O"]) < 5e-2
    assert maxerr(la, ref["L"]) < 3e-2
    assert maxerr(oa, od) < 5e-2
