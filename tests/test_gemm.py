"""GEMM plan (GEMMKernelDescriptor(descriptor:)) through the C ABI — no GPU needed.

Mirrors GEMMDescriptor.setFunctionConstants' leading-dimension rules
(GEMMDescriptor.swift:344-372) and the register-precision selection
(GEMMDescriptor.swift:204-219) with the gfx950 policy stated in include/mfa/mfa.h."""
import pytest

import mfa_amd as mfa

P = mfa.Precision


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_default_leading_dimensions(ta, tb):
    d = mfa.gemm_descriptor(70, 50, 30, P.FP32, P.FP32, transpose_a=ta, transpose_b=tb)
    k = mfa.gemm_kernel_descriptor(d)
    # expected leading = rows when transposed, columns otherwise (:348-355).
    assert k.lda == (70 if ta else 30)
    assert k.ldb == (30 if tb else 50)
    assert k.ldc == 50
    assert (k.grid_x, k.grid_y, k.grid_z) == (1, 1, 1)
    assert k.threadgroup_size == 256


def test_leading_dimension_too_small():
    d = mfa.gemm_descriptor(64, 64, 64, P.FP16, P.FP32, lda=63)
    with pytest.raises(mfa.MFAError, match="Leading block dimension was too small"):
        mfa.gemm_kernel_descriptor(d)
    d = mfa.gemm_descriptor(64, 64, 64, P.FP16, P.FP32, transpose_a=True, lda=64, ldb=64, ldc=80)
    k = mfa.gemm_kernel_descriptor(d)
    assert (k.lda, k.ldb, k.ldc) == (64, 64, 80)


def test_unsupported_precisions():
    d = mfa.gemm_descriptor(8, 8, 8, P.INT8, P.FP32)
    with pytest.raises(mfa.MFAError):
        mfa.gemm_kernel_descriptor(d)


@pytest.mark.parametrize("pa,pb,compute", [
    (P.FP16, P.FP16, P.FP16), (P.BF16, P.BF16, P.BF16), (P.FP32, P.FP32, P.FP32),
    (P.FP16, P.FP32, P.FP32), (P.FP16, P.BF16, P.FP32), (P.BF16, P.FP32, P.FP32)])
def test_register_precisions(pa, pb, compute):
    for ta in (0, 1):
        d = mfa.gemm_descriptor(300, 200, 100, pa, P.FP16, prec_b=pb, transpose_a=ta, batch=3)
        k = mfa.gemm_kernel_descriptor(d)
        assert list(k.register_precisions) == [compute, compute, P.FP32]
        assert list(k.memory_precisions) == [pa, pb, P.FP16]
        assert (k.grid_x, k.grid_y, k.grid_z) == (2, 3, 3)
        assert k.block_k == (16 if compute == P.FP32 else 32)
        tuned = compute != P.FP32 and not ta
        assert (b"mfa_gemm2_kernel" in k.variant) == tuned
        assert k.threadgroup_memory_allocation <= 160 * 1024
