"""GPU parity for the general GEMM (GEMMDescriptor surface: mixed FP32/FP16/BF16 operands,
transposes, padded leading dimensions, loadPreviousC, batch) against the oracle GEMM.

Cases follow the reference's own GEMM tests:
  * LaplacianTest.swift: square FP32 problems of sizes 7..153 with transpose states
    (N,N), (N,T), (T,N); one operand is the periodic 1-D Laplacian (-2 on the diagonal, 1 on
    both wrapped off-diagonals), the other uniform [0, 1).  Threshold 1e-5 for FP32
    (createErrorThreshold).
  * AdversarialShapeTest.swift:7-64: 20 random problems — dims ⌊1000·u³⌋ (≥ 1), random
    precisions per operand, random transposes, leading dimensions padded by 0..63 half the
    time, random loadPreviousC; inputs uniform [0, 1) / √K; tolerance createTolerance
    (:317-372) restated below.  Seeded here (the reference draws unseeded).
The padding of every buffer is NaN, so a read outside the logical matrix shows up."""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import TORCH_DTYPE, seen

pytestmark = pytest.mark.gpu
P = mfa.Precision
DEV = "cuda:0"

LAPLACIAN_SIZES = [7, 8, 9, 10, 15, 16, 17, 18, 23, 24, 25, 31, 32, 33, 47, 48, 49, 63, 64, 65,
                   103, 104, 112, 126, 127, 128, 129, 130, 131, 135, 136, 137, 143, 144, 145,
                   151, 152, 153]


def buffer(logical: np.ndarray, ld: int, prec) -> tuple[torch.Tensor, np.ndarray]:
    """Row-major device buffer of `logical` with leading dimension ld (padding = NaN);
    returns (device tensor, the values the kernel sees)."""
    rows, cols = logical.shape
    full = np.full((rows, ld), np.nan, dtype=np.float32)
    full[:, :cols] = logical
    t = torch.from_numpy(full).to(DEV).to(TORCH_DTYPE[prec])
    return t, seen(logical, prec)


def read_back(c: torch.Tensor, M: int, N: int) -> np.ndarray:
    return c.float().cpu().numpy()[:M, :N]


def run(M, N, K, A_log, B_log, prec, ta, tb, pad=(0, 0, 0), prev=None):
    """A_log [M,K] and B_log [K,N] are the logical operands; they are stored transposed when
    ta / tb.  Returns (device result [M,N] as float, oracle)."""
    pa, pb, pc = prec
    a_mem = A_log.T if ta else A_log
    b_mem = B_log.T if tb else B_log
    lda, ldb, ldc = a_mem.shape[1] + pad[0], b_mem.shape[1] + pad[1], N + pad[2]
    a, a_seen = buffer(np.ascontiguousarray(a_mem), lda, pa)
    b, b_seen = buffer(np.ascontiguousarray(b_mem), ldb, pb)
    if prev is None:
        c = torch.full((M, ldc), float("nan"), dtype=TORCH_DTYPE[pc], device=DEV)
        prev_seen = None
    else:
        c, prev_seen = buffer(prev, ldc, pc)
    mfa.gemm(a, b, c, M, N, K, pa, pc, prec_b=pb, transpose_a=ta, transpose_b=tb,
             lda=lda, ldb=ldb, ldc=ldc, load_previous_c=prev is not None)
    torch.cuda.synchronize()
    A_s = a_seen.T if ta else a_seen
    B_s = b_seen.T if tb else b_seen
    ref = ol.gemm(A_s, B_s, prev_seen)
    got = read_back(c, M, N)
    if ldc > N and M > 0:
        pad_vals = c.float().cpu().numpy()[:, N:]
        assert np.all(np.isnan(pad_vals)), "store outside the logical C"
    return got, seen(ref, pc)


def laplacian(n: int) -> np.ndarray:
    L = np.zeros((n, n), dtype=np.float32)
    for i in range(n):
        L[i, i] = -2
        L[i, (i - 1) % n] = 1
        L[i, (i + 1) % n] = 1
    return L


@pytest.mark.parametrize("n", LAPLACIAN_SIZES)
@pytest.mark.parametrize("ta,tb", [(False, False), (False, True), (True, False)])
def test_laplacian_fp32(gpu, n, ta, tb):
    rng = np.random.default_rng(n)
    L, R = laplacian(n), rng.random((n, n), dtype=np.float32)
    # LaplacianTest swaps A and B when A is transposed (LaplacianTest.swift:131-133).
    A, B = (R, L) if ta else (L, R)
    got, ref = run(n, n, n, A, B, (P.FP32, P.FP32, P.FP32), ta, tb)
    assert np.max(np.abs(got - ref)) < 1e-5


@pytest.mark.parametrize("prec", [P.FP16, P.BF16])
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (True, True)])
def test_laplacian_16bit_transposed(gpu, prec, ta, tb):
    n = 137
    rng = np.random.default_rng(7)
    L, R = laplacian(n), rng.random((n, n), dtype=np.float32)
    A, B = (R, L) if ta else (L, R)
    got, ref = run(n, n, n, A, B, (prec, prec, prec), ta, tb)
    thr = {P.FP16: 5e-3, P.BF16: 5e-2}[prec]  # createErrorThreshold
    assert np.max(np.abs(got - ref)) < thr


def create_tolerance(pa, pb, pc, K) -> float:
    """AdversarialShapeTest.swift createTolerance (:317-372)."""
    noise = np.sqrt(K)
    tol = 3e-7
    if pa == P.FP16 or pb == P.FP16:
        tol = max(tol, 1e-5, 1e-3 / noise)
    if pc == P.FP16:
        tol = max(tol, 3e-4)
    if pa == pb == pc == P.FP16:
        tol = max(tol, 3e-3, 1e-5 * K)
    if P.BF16 in (pa, pb, pc):
        tol = max(tol, 2e-2 if K < 1000 else 5e-3)
    tol += {P.BF16: 2.0 ** -8, P.FP16: 2.0 ** -10}.get(pc, 2.0 ** -22)
    return tol


def adversarial_cases(n=20, seed=1234):
    rng = np.random.default_rng(seed)
    out = []
    for _ in range(n):
        u = rng.random(3, dtype=np.float32)
        dims = [max(1, int(x)) for x in (u * u * u) * 1000]
        precs = tuple(P(int(x)) for x in rng.integers(0, 3, 3))
        ta, tb, prev = (bool(x) for x in rng.integers(0, 2, 3))
        pad = tuple(int(x) for x in rng.integers(0, 64, 3)) if rng.integers(0, 2) else (0, 0, 0)
        out.append((tuple(dims), precs, ta, tb, pad, prev))
    return out


@pytest.mark.parametrize("case", adversarial_cases(), ids=lambda c: f"{c[0]}-{[int(p) for p in c[1]]}-{int(c[2])}{int(c[3])}")
def test_adversarial_shapes(gpu, case):
    (M, N, K), (pa, pb, pc), ta, tb, pad, use_prev = case
    rng = np.random.default_rng(M * 7 + N * 3 + K)
    s = 1 / np.sqrt(K)
    A = rng.random((M, K), dtype=np.float32) * s
    B = rng.random((K, N), dtype=np.float32) * s
    prev = rng.random((M, N), dtype=np.float32) * s if use_prev else None
    got, ref = run(M, N, K, A, B, (pa, pb, pc), ta, tb, pad, prev)
    assert np.max(np.abs(got - ref)) < create_tolerance(pa, pb, pc, K)


@pytest.mark.parametrize("ta,tb", [(False, True), (True, False), (True, True)])
@pytest.mark.parametrize("prec", [P.FP16, P.BF16, P.FP32])
def test_batched_transposed(gpu, prec, ta, tb):
    Bn, M, N, K = 3, 150, 200, 72
    rng = np.random.default_rng(5)
    A = rng.standard_normal((Bn, M, K)).astype(np.float32)
    Bm = rng.standard_normal((Bn, K, N)).astype(np.float32)
    a_mem = np.ascontiguousarray(A.transpose(0, 2, 1) if ta else A)
    b_mem = np.ascontiguousarray(Bm.transpose(0, 2, 1) if tb else Bm)
    a = torch.from_numpy(a_mem).to(DEV).to(TORCH_DTYPE[prec])
    b = torch.from_numpy(b_mem).to(DEV).to(TORCH_DTYPE[prec])
    c = torch.full((Bn, M, N), float("nan"), dtype=torch.float32, device=DEV)
    mfa.gemm(a, b, c, M, N, K, prec, P.FP32, transpose_a=ta, transpose_b=tb, batch=Bn,
             stride_a=M * K, stride_b=K * N, stride_c=M * N)
    torch.cuda.synchronize()
    As, Bs = seen(A, prec), seen(Bm, prec)
    ref = np.stack([ol.gemm(As[i], Bs[i]) for i in range(Bn)])
    tol = 1e-4 * np.sqrt(K) if prec == P.FP32 else 1e-3 * np.sqrt(K)
    assert np.max(np.abs(c.cpu().numpy() - ref)) < tol


@pytest.mark.parametrize("kern", ["gemm2", "gemm3"])
@pytest.mark.parametrize("ta,tb", [(False, True), (True, False)])
@pytest.mark.parametrize("prec,pc", [(P.FP16, P.FP32), (P.BF16, P.BF16), (P.BF16, P.FP16)])
def test_whole_tile_transposed_lds_dma(gpu, prec, pc, ta, tb, kern):
    # NT / TN with equal 16-bit operands and whole 128x128x64 tiles run mfa_gemm2_kernel (both
    # operands read by rows, or both transposed); whole 256x256 tiles the 8-wave
    # mfa_gemm3_kernel (forced here at a size below one round of the chip); C in its own
    # precision; batched, with padded leading dimensions (NaN padding catches any read outside
    # the logical matrices).
    Bn, M, N, K, pad = (2, 256, 384, 192, 8) if kern == "gemm2" else (2, 256, 512, 192, 8)
    rng = np.random.default_rng(11)
    A = rng.standard_normal((Bn, M, K)).astype(np.float32)
    Bm = rng.standard_normal((Bn, K, N)).astype(np.float32)
    a_log = A.transpose(0, 2, 1) if ta else A
    b_log = Bm.transpose(0, 2, 1) if tb else Bm
    lda, ldb = a_log.shape[2] + pad, b_log.shape[2] + pad
    a_full = np.full((Bn, a_log.shape[1], lda), np.nan, dtype=np.float32)
    a_full[:, :, :a_log.shape[2]] = a_log
    b_full = np.full((Bn, b_log.shape[1], ldb), np.nan, dtype=np.float32)
    b_full[:, :, :b_log.shape[2]] = b_log
    a = torch.from_numpy(a_full).to(DEV).to(TORCH_DTYPE[prec])
    b = torch.from_numpy(b_full).to(DEV).to(TORCH_DTYPE[prec])
    c = torch.full((Bn, M, N), float("nan"), dtype=torch.float32, device=DEV).to(TORCH_DTYPE[pc])
    os.environ["MFA_GEMM3"] = "1" if kern == "gemm3" else "0"
    try:
        mfa.last_launches()
        mfa.gemm(a, b, c, M, N, K, prec, pc, transpose_a=ta, transpose_b=tb, batch=Bn,
                 lda=lda, ldb=ldb, stride_a=a_full[0].size, stride_b=b_full[0].size, stride_c=M * N)
        launched = [r["name"] for r in mfa.last_launches()]
    finally:
        os.environ.pop("MFA_GEMM3", None)
    assert launched and launched[0].startswith(f"mfa_{kern}_kernel<"), launched
    torch.cuda.synchronize()
    As, Bs = seen(A, prec), seen(Bm, prec)
    ref = seen(np.stack([ol.gemm(As[i], Bs[i]) for i in range(Bn)]).astype(np.float32), pc)
    got = c.float().cpu().numpy()
    assert np.isfinite(got).all()
    tol = 1e-3 * np.sqrt(K) + (0 if pc == P.FP32 else 8e-3 * np.abs(ref).max())
    assert np.max(np.abs(got - ref)) < tol
    d = mfa.gemm_descriptor(M, N, K, prec, pc, transpose_a=ta, transpose_b=tb, batch=Bn,
                            lda=lda, ldb=ldb)
    assert b"mfa_gemm2_kernel" in mfa.gemm_kernel_descriptor(d).variant
    d = mfa.gemm_descriptor(4096, 4096, K, prec, pc, transpose_a=ta, transpose_b=tb)
    assert b"mfa_gemm3_kernel" in mfa.gemm_kernel_descriptor(d).variant


def test_zero_k_and_empty(gpu):
    # K = 0: C = 0 (or C itself with loadPreviousC); M = 0 / N = 0: nothing written.
    c = torch.full((5, 6), float("nan"), dtype=torch.float32, device=DEV)
    a = torch.zeros((5, 1), dtype=torch.float32, device=DEV)
    b = torch.zeros((1, 6), dtype=torch.float32, device=DEV)
    mfa.gemm(a, b, c, 5, 6, 0, P.FP32, P.FP32, prec_b=P.FP32, lda=1, ldb=6)
    torch.cuda.synchronize()
    assert torch.all(c == 0)
    c2 = torch.full((5, 6), 3.0, dtype=torch.float32, device=DEV)
    mfa.gemm(a, b, c2, 5, 6, 0, P.FP32, P.FP32, lda=1, ldb=6, load_previous_c=True)
    torch.cuda.synchronize()
    assert torch.all(c2 == 3.0)


@pytest.mark.parametrize("kern,img", [("gemm3", "1"), ("gemm2", "1"), ("gemm2", "0")])
@pytest.mark.parametrize("prec,pc", [(P.FP16, P.FP16), (P.BF16, P.BF16), (P.FP16, P.FP32)])
def test_whole_tile_c_image_padded_ldc(gpu, prec, pc, kern, img):
    # A 16-bit C leaves the whole-tile kernels through an LDS image as whole rows (default) or,
    # on mfa_gemm2_kernel, as per-lane pieces (MFA_GEMM_IMG=0); C has a padded leading dimension
    # whose padding, and the rows past M, must stay untouched (NaN sentinels).  256 x 256
    # problems run the 8-wave mfa_gemm3_kernel; MFA_GEMM3=0 keeps mfa_gemm2_kernel.
    Bn, M, N, K, cpad = 2, 256, 256, 128, 8
    rng = np.random.default_rng(12)
    A = rng.standard_normal((Bn, M, K)).astype(np.float32)
    Bm = rng.standard_normal((Bn, K, N)).astype(np.float32)
    a = torch.from_numpy(A).to(DEV).to(TORCH_DTYPE[prec])
    b = torch.from_numpy(Bm).to(DEV).to(TORCH_DTYPE[prec])
    ldc = N + cpad
    c = torch.full((Bn, M + 1, ldc), float("nan"), dtype=torch.float32, device=DEV).to(TORCH_DTYPE[pc])
    os.environ["MFA_GEMM_IMG"] = img
    os.environ["MFA_GEMM3"] = "1" if kern == "gemm3" else "0"
    try:
        mfa.last_launches()
        mfa.gemm(a, b, c, M, N, K, prec, pc, batch=Bn, ldc=ldc, stride_a=M * K, stride_b=K * N,
                 stride_c=(M + 1) * ldc)
        launched = [r["name"] for r in mfa.last_launches()]
    finally:
        os.environ.pop("MFA_GEMM_IMG", None)
        os.environ.pop("MFA_GEMM3", None)
    assert launched and launched[0].startswith(f"mfa_{kern}_kernel<"), launched
    torch.cuda.synchronize()
    got = c.float().cpu().numpy()
    assert np.isnan(got[:, :M, N:]).all() and np.isnan(got[:, M]).all()
    As, Bs = seen(A, prec), seen(Bm, prec)
    ref = seen(np.stack([ol.gemm(As[i], Bs[i]) for i in range(Bn)]).astype(np.float32), pc)
    tol = 1e-3 * np.sqrt(K) + (0 if pc == P.FP32 else 8e-3 * np.abs(ref).max())
    assert np.max(np.abs(got[:, :M, :N] - ref)) < tol
    # The plan names the 8-wave kernel once its 256 x 256 tiles fill a round of the chip.
    d = mfa.gemm_descriptor(M, N, K, prec, pc, batch=Bn, ldc=ldc)
    assert b"mfa_gemm3_kernel" not in mfa.gemm_kernel_descriptor(d).variant
    d = mfa.gemm_descriptor(4096, 4096, K, prec, pc)
    assert b"mfa_gemm3_kernel" in mfa.gemm_kernel_descriptor(d).variant
