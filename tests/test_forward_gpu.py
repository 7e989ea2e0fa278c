"""GPU parity: attention forward through the C ABI vs the CPU oracle.

Cases follow the reference's own tests (paths relative to the reference repo):
  - SquareAttentionTest.testCorrectness shape list, FP32 tol 2e-5 / mixed 5e-2 (O), 7e-3 (L)
    (Tests/FlashAttentionTests/Attention/SquareAttentionTest.swift:5-26, :557-571);
  - KernelRegressionTests: causal B1 H2 S96 D64 (tol 2e-3), pipeline-cache shapes S64/S80,
    strided BSHD == contiguous bit-exact, BF16 inputs 5e-3 (KernelRegressionTests.swift:238-512);
  - BASELINE.json config 1 (1 head fp32 S128 D64) and config 2 at full size on one head.
"""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, relerr, run_forward, seen, to_device

pytestmark = pytest.mark.gpu

FP32, FP16, BF16 = mfa.Precision.FP32, mfa.Precision.FP16, mfa.Precision.BF16


def gaussian(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def check_forward(Qn, Kn, Vn, prec, tol_o, tol_l, **kw):
    o, l = run_forward(Qn, Kn, Vn, prec=prec, **kw)
    ref = ol.attention(seen(Qn, prec), seen(Kn, prec), seen(Vn, prec),
                       scale=kw.get("scale"), causal=kw.get("causal", False),
                       window=kw.get("window"), amask=kw.get("amask"), ranges=kw.get("ranges"))
    eo, el = maxerr(o, ref["O"]), maxerr(l, ref["L"])
    assert np.isfinite(o.cpu().numpy()).all()
    assert eo <= tol_o, f"O max error {eo} > {tol_o}"
    assert el <= tol_l, f"L max error {el} > {tol_l}"
    return o, l, ref


def test_config1_fp32_s128_d64(gpu):
    # BASELINE.json configs[0]: 1 head fp32 forward, seq=128, d=64.
    S, D = 128, 64
    Q = ol.lcg(11, S * D).reshape(1, 1, S, D)
    K = ol.lcg(22, S * D).reshape(1, 1, S, D)
    V = ol.lcg(33, S * D).reshape(1, 1, S, D)
    check_forward(Q, K, V, FP32, 2e-5, 2e-5)


SQUARE_SHAPES = [(10, 3), (10, 80), (8, 2), (9, 2), (23, 2), (24, 2), (25, 2), (192, 77),
                 (192, 80), (93, 32), (99, 35), (64, 32), (64, 34), (64, 36), (64, 40), (32, 64),
                 (4, 1), (4, 2), (384, 95), (777, 199)]


@pytest.mark.parametrize("S,D", SQUARE_SHAPES)
def test_square_fp32(gpu, S, D):
    Q, K, V = (gaussian((1, 1, S, D), 100 + i) for i in range(3))
    check_forward(Q, K, V, FP32, 2e-5, 2e-5)


@pytest.mark.parametrize("S,D", [(10, 80), (192, 77), (93, 32), (64, 40), (384, 95), (777, 199),
                                 (4, 1)])
@pytest.mark.parametrize("prec", [FP16, BF16])
def test_square_mixed(gpu, S, D, prec):
    Q, K, V = (gaussian((1, 1, S, D), 200 + i) for i in range(3))
    # Mixed precision tolerances of SquareAttentionTest (O 5e-2, L 7e-3); L stored FP16.
    check_forward(Q, K, V, prec, 5e-2, 7e-3)


@pytest.mark.parametrize("prec,tol", [(FP32, 2e-3), (FP16, 2e-3), (BF16, 5e-3)])
def test_causal_regression_shape(gpu, prec, tol):
    B, H, S, D = 1, 2, 96, 64
    n = B * H * S * D
    Q = ol.lcg(11, n).reshape(B, H, S, D)
    K = ol.lcg(22, n).reshape(B, H, S, D)
    V = ol.lcg(33, n).reshape(B, H, S, D)
    check_forward(Q, K, V, prec, tol, 1e-2 if prec != FP32 else 2e-5, causal=True)


@pytest.mark.parametrize("S", [64, 80])
def test_pipeline_shapes_share_instance(gpu, S):
    B, H, D = 1, 2, 64
    n = B * H * S * D
    Q = ol.lcg(44, n).reshape(B, H, S, D)
    K = ol.lcg(55, n).reshape(B, H, S, D)
    V = ol.lcg(66, n).reshape(B, H, S, D)
    check_forward(Q, K, V, FP32, 2e-3, 2e-5, causal=True)


def test_bf16_inputs_match_reference(gpu):
    B, H, S, D = 1, 2, 96, 64
    n = B * H * S * D
    Q = ol.lcg(404, n).reshape(B, H, S, D)
    K = ol.lcg(505, n).reshape(B, H, S, D)
    V = ol.lcg(606, n).reshape(B, H, S, D)
    check_forward(Q, K, V, BF16, 5e-3, 1e-2)


@pytest.mark.parametrize("prec", [FP32, FP16])
def test_strided_bshd_matches_contiguous_bitexact(gpu, prec):
    # KernelRegressionTests.testStridedInputsMatchContiguous: BSHD storage presented through
    # BHSD element strides [S*H*D, D, H*D, 1] must equal the contiguous run exactly.
    B, H, S, D = 2, 3, 96, 64
    n = B * H * S * D
    Qn = ol.lcg(101, n).reshape(B, H, S, D)
    Kn = ol.lcg(202, n).reshape(B, H, S, D)
    Vn = ol.lcg(303, n).reshape(B, H, S, D)
    o_ref, _ = run_forward(Qn, Kn, Vn, prec=prec)
    base = mfa.AttentionDescriptor.make(low_precision=prec != FP32,
                                        precision=prec if prec != FP32 else None)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    to_bshd = lambda x: to_device(np.ascontiguousarray(x.transpose(0, 2, 1, 3)), prec)
    strides = [S * H * D, D, H * D, 1]
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    mfa.MultiHeadAttention().encodeForward(desc, to_bshd(Qn), to_bshd(Kn), to_bshd(Vn), o,
                                           query_strides=strides, key_strides=strides,
                                           value_strides=strides)
    torch.cuda.synchronize()
    assert torch.equal(o, o_ref)


@pytest.mark.parametrize("causal,share", [(False, "1"), (True, None)])
def test_strided_bshd_gqa_shared_tile_kernels(gpu, causal, share):
    # The shared-tile kernels (adjacent unmasked pairs, forced at this size; mirrored causal
    # pairs, the default) with BSHD strides, GQA (4 query heads per kv head) and B = 2: equal
    # to the contiguous BHSD run bit for bit, and to the oracle.
    B, H, Hkv, S, D = 2, 8, 2, 640, 128
    rng = np.random.default_rng(640)
    Qn = rng.standard_normal((B, H, S, D)).astype(np.float32)
    Kn = rng.standard_normal((B, Hkv, S, D)).astype(np.float32)
    Vn = rng.standard_normal((B, Hkv, S, D)).astype(np.float32)
    if share:
        os.environ["MFA_FWD_SHARE"] = share
    try:
        o_ref, _ = run_forward(Qn, Kn, Vn, prec=FP16, causal=causal)
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, causal=causal)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D, Hkv=Hkv)
        to_bshd = lambda x: to_device(np.ascontiguousarray(x.transpose(0, 2, 1, 3)), FP16)
        qs = [S * H * D, D, H * D, 1]
        ks = [S * Hkv * D, D, Hkv * D, 1]
        o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
        mfa.MultiHeadAttention().encodeForward(desc, to_bshd(Qn), to_bshd(Kn), to_bshd(Vn), o,
                                               query_strides=qs, key_strides=ks, value_strides=ks)
        torch.cuda.synchronize()
    finally:
        os.environ.pop("MFA_FWD_SHARE", None)
    assert torch.equal(o, o_ref)
    for b, hh in ((0, 0), (1, 5)):
        ref = ol.attention(seen(Qn[b:b + 1, hh:hh + 1], FP16), seen(Kn[b:b + 1, hh // 4:hh // 4 + 1], FP16),
                           seen(Vn[b:b + 1, hh // 4:hh // 4 + 1], FP16), causal=causal)
        assert np.abs(o[b, hh].cpu().numpy() - ref["O"][0, 0]).max() <= 5e-3


def test_forward_without_logsumexp_matches(gpu):
    # MultiHeadAttention.forward with logsumexp=nil uses a library scratch L (:296-319).
    B, H, S, D = 2, 3, 64, 32
    n = B * H * S * D
    Qn, Kn, Vn = (ol.lcg(77 + 11 * i, n).reshape(B, H, S, D) for i in range(3))
    o_ref, _ = run_forward(Qn, Kn, Vn)
    base = mfa.AttentionDescriptor.make()
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    mfa.MultiHeadAttention().forward(desc, to_device(Qn, FP32), to_device(Kn, FP32),
                                     to_device(Vn, FP32), o)
    torch.cuda.synchronize()
    assert torch.equal(o, o_ref)


@pytest.mark.parametrize("prec", [FP32, FP16, BF16])
@pytest.mark.parametrize("H,Hkv", [(8, 2), (4, 1), (6, 3)])
def test_gqa_mqa(gpu, prec, H, Hkv):
    B, S, D = 2, 130, 64
    Q = gaussian((B, H, S, D), 1)
    K = gaussian((B, Hkv, S, D), 2)
    V = gaussian((B, Hkv, S, D), 3)
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2)


@pytest.mark.parametrize("prec", [FP32, FP16])
@pytest.mark.parametrize("R,C", [(100, 300), (300, 100), (1, 257), (257, 1)])
def test_cross_attention(gpu, prec, R, C):
    B, H, D = 2, 2, 64
    Q = gaussian((B, H, R, D), 4)
    K = gaussian((B, H, C, D), 5)
    V = gaussian((B, H, C, D), 6)
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2)


@pytest.mark.parametrize("prec", [FP32, FP16, BF16])
@pytest.mark.parametrize("R,C", [(200, 200), (130, 300), (300, 130)])
def test_causal_ragged(gpu, prec, R, C):
    B, H, D = 1, 3, 80
    Q = gaussian((B, H, R, D), 7)
    K = gaussian((B, H, C, D), 8)
    V = gaussian((B, H, C, D), 9)
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2, causal=True)


@pytest.mark.parametrize("prec", [FP32, FP16])
@pytest.mark.parametrize("W", [0, 5, 64, 300])
def test_sliding_window(gpu, prec, W):
    # row > col + W is masked; not symmetric and not implicitly causal
    # (AttentionKernel+Softmax.swift:433-474).
    B, H, S, D = 1, 2, 257, 64
    Q, K, V = gaussian((B, H, S, D), 10), gaussian((B, H, S, D), 11), gaussian((B, H, S, D), 12)
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2, window=W)


def test_window_with_fully_masked_rows(gpu):
    # R > C + W: late rows are masked everywhere; the reference's finite mask value makes them
    # a uniform average, which requires no tile skipping.
    B, H, R, C, D = 1, 1, 200, 64, 32
    Q, K, V = gaussian((B, H, R, D), 13), gaussian((B, H, C, D), 14), gaussian((B, H, C, D), 15)
    check_forward(Q, K, V, FP32, 2e-5, 2e-3, window=16)


@pytest.mark.parametrize("prec", [FP32, FP16])
def test_sparse_ranges_sliding_builder(gpu, prec):
    # SparseMQABuilder.buildSlidingWindow ranges as the HAS_SPARSE_RANGES mask buffer,
    # indexed (b*H_kv + kv)*R + row (AttentionKernel+Softmax.swift:360-375).
    B, H, Hkv, S, D = 2, 4, 2, 150, 64
    rng_host = np.zeros((S, 2), dtype=np.uint32)
    mfa.lib.mfa_sparse_build_sliding_window(S, 40, rng_host.ctypes.data)
    ranges = np.ascontiguousarray(np.broadcast_to(rng_host, (B, Hkv, S, 2)))
    Q = gaussian((B, H, S, D), 16)
    K, V = gaussian((B, Hkv, S, D), 17), gaussian((B, Hkv, S, D), 18)
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2, ranges=ranges)


def test_sparse_ranges_with_empty_rows(gpu):
    B, H, S, D = 1, 1, 70, 32
    ranges = np.zeros((B, H, S, 2), dtype=np.uint32)
    ranges[..., 0] = np.arange(S) // 2
    ranges[..., 1] = np.minimum(S, np.arange(S) + 3)
    ranges[0, 0, ::7] = 0  # empty range: fully masked row -> uniform average
    Q, K, V = gaussian((B, H, S, D), 19), gaussian((B, H, S, D), 20), gaussian((B, H, S, D), 21)
    check_forward(Q, K, V, FP32, 2e-5, 2e-3, ranges=ranges)


@pytest.mark.parametrize("prec", [FP32, FP16])
def test_additive_mask(gpu, prec):
    # Dense fp32 mask [B, H, R, C] added to QK^T before scaling (:306-336).
    B, H, R, C, D = 2, 2, 90, 140, 64
    Q, K, V = gaussian((B, H, R, D), 22), gaussian((B, H, C, D), 23), gaussian((B, H, C, D), 24)
    amask = (np.random.default_rng(25).standard_normal((B, H, R, C)) * 3).astype(np.float32)
    amask[:, :, :, ::5] = -1e9
    tol = 2e-5 if prec == FP32 else 5e-2
    check_forward(Q, K, V, prec, tol, 2e-5 if prec == FP32 else 1e-2, amask=amask)


@pytest.mark.parametrize("scale", [0.5, 0.01])
def test_custom_softmax_scale(gpu, scale):
    B, H, S, D = 1, 2, 100, 64
    Q, K, V = gaussian((B, H, S, D), 26), gaussian((B, H, S, D), 27), gaussian((B, H, S, D), 28)
    check_forward(Q, K, V, FP32, 2e-5, 2e-5, scale=scale)


def test_transposed_query(gpu):
    # transposeState.Q: column-major within a head (AttentionKernelDescriptor.swift:34-47).
    B, H, S, D = 1, 2, 70, 48
    Q, K, V = gaussian((B, H, S, D), 29), gaussian((B, H, S, D), 30), gaussian((B, H, S, D), 31)
    base = mfa.AttentionDescriptor.make(transpose=(True, False, False, False))
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    qt = to_device(np.ascontiguousarray(Q.transpose(0, 1, 3, 2)), FP32)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    mfa.MultiHeadAttention().forward(desc, qt, to_device(K, FP32), to_device(V, FP32), o)
    torch.cuda.synchronize()
    ref = ol.attention(Q, K, V)
    assert maxerr(o, ref["O"]) <= 2e-5


@pytest.mark.parametrize("prec", [FP16, BF16])
def test_config2_full_size_one_head(gpu, prec):
    # BASELINE.json configs[1] shape (H16 S4096 D128 causal): all heads on the GPU, the oracle
    # on heads 0, 7 and 15; size-independent checks on every head (rows of P sum to one => O is a
    # convex combination of V rows: |O| <= max|V|).
    B, H, S, D = 1, 16, 4096, 128
    n = B * H * S * D
    Q = ol.lcg(11, n).reshape(B, H, S, D)
    K = ol.lcg(22, n).reshape(B, H, S, D)
    V = ol.lcg(33, n).reshape(B, H, S, D)
    o, l = run_forward(Q, K, V, prec=prec, causal=True)
    on = o.cpu().numpy()
    assert np.isfinite(on).all()
    assert np.abs(on).max() <= np.abs(V).max() * 1.01
    for h in (0, 7, 15):
        ref = ol.attention(seen(Q[:, h:h + 1], prec), seen(K[:, h:h + 1], prec),
                           seen(V[:, h:h + 1], prec), causal=True)
        assert maxerr(on[:, h:h + 1], ref["O"]) <= 5e-3
        assert maxerr(l[:, h:h + 1], ref["L"]) <= 7e-3


def test_single_element_edges(gpu):
    for (R, C, D) in [(1, 1, 1), (1, 2, 3), (33, 1, 7), (2, 65, 257 - 1)]:
        Q, K, V = gaussian((1, 1, R, D), R), gaussian((1, 1, C, D), C + 1), gaussian((1, 1, C, D), D)
        check_forward(Q, K, V, FP32, 2e-5, 2e-5)
