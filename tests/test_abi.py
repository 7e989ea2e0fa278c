"""CPU tests of the C ABI (libmfa_amd.so): exports, host-side descriptor logic and the
reference host utilities.  No kernel is launched here."""
import ctypes

import numpy as np
import pytest

import mfa_amd as mfa


def test_library_exports_every_header_function():
    names = mfa.header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(mfa.lib, n)]
    assert not missing, missing


def test_version_and_abi():
    assert mfa.lib.mfa_abi_version() == 1
    assert b"gfx950" in mfa.lib.mfa_version()


def test_operand_buffer_bindings_match_reference_slots():
    # AttentionOperand.bufferBinding (AttentionOperand.swift:50-67)
    expect = {mfa.Operand.Q: 0, mfa.Operand.K: 1, mfa.Operand.V: 2, mfa.Operand.O: 3,
              mfa.Operand.L: 4, mfa.Operand.D: 5, mfa.Operand.dO: 6, mfa.Operand.dV: 7,
              mfa.Operand.dK: 8, mfa.Operand.dQ: 9, mfa.Operand.S: -1, mfa.Operand.P: -1,
              mfa.Operand.dP: -1, mfa.Operand.dS: -1}
    for op, slot in expect.items():
        assert mfa.lib.mfa_operand_buffer_binding(int(op)) == slot


def test_descriptor_defaults():
    d = mfa.AttentionDescriptor()
    mfa.lib.mfa_attention_descriptor_init(ctypes.byref(d))
    assert d.low_precision_inputs == 0 and d.low_precision_intermediates == 0
    assert d.input_memory_precision == -1 and d.sparsity_pattern == 0
    assert d.has_matrix_dimensions == 0 and d.has_softmax_scale == 0


def test_incomplete_descriptor_is_rejected():
    d = mfa.AttentionDescriptor()
    mfa.lib.mfa_attention_descriptor_init(ctypes.byref(d))
    out = mfa.KernelDescriptor()
    st = mfa.lib.mfa_attention_kernel_descriptor(ctypes.byref(d), 0, ctypes.byref(out))
    assert st == 1  # MFA_ERR_INVALID_DESCRIPTOR ("Descriptor was incomplete.")
    assert b"incomplete" in mfa.lib.mfa_last_error()


@pytest.mark.parametrize("lp,prec,expect_in", [(False, None, 0), (True, mfa.Precision.FP16, 1),
                                               (True, mfa.Precision.BF16, 2), (True, None, 1)])
def test_memory_precisions_follow_reference_policy(lp, prec, expect_in):
    # AttentionDescriptor+Precisions.swift:12-149
    d = mfa.AttentionDescriptor.make(128, 128, 64, low_precision=lp, precision=prec)
    k = mfa.kernel_descriptor(d, mfa.KernelType.forward)
    mp = list(k.memory_precisions)
    for op in (mfa.Operand.Q, mfa.Operand.K, mfa.Operand.V, mfa.Operand.dO):
        assert mp[op] == expect_in
    assert mp[mfa.Operand.L] == (1 if lp else 0)
    assert mp[mfa.Operand.D] == (2 if lp else 0)
    for op in (mfa.Operand.O, mfa.Operand.dV, mfa.Operand.dK, mfa.Operand.dQ):
        assert mp[op] == 0


@pytest.mark.parametrize("kind,cached", [
    (mfa.KernelType.forward, {mfa.Operand.Q, mfa.Operand.O}),
    (mfa.KernelType.backwardQuery, {mfa.Operand.Q, mfa.Operand.dO, mfa.Operand.dQ}),
    (mfa.KernelType.backwardKeyValue, {mfa.Operand.K, mfa.Operand.V, mfa.Operand.dK,
                                       mfa.Operand.dV})])
def test_kernel_plan_fields(kind, cached):
    d = mfa.AttentionDescriptor.make(4096, 4096, 128, low_precision=True,
                                     precision=mfa.Precision.FP16, causal=True)
    k = mfa.kernel_descriptor(d, kind)
    assert k.head_dimension == 128 and k.sequence_length == 4096
    assert {mfa.Operand(i) for i in range(14) if k.cache_state[i]} == cached
    kern = mfa.attention_kernel(k)
    assert kern.threadgroup_size % 64 == 0
    assert kern.block_parallelization == 128
    assert 0 < kern.threadgroup_memory_allocation <= 160 * 1024
    assert abs(kern.softmax_scale - 1 / np.sqrt(128)) < 1e-7
    assert kern.variant.startswith(b"mfa_")


def test_block_head_clamped_to_padded_head():
    # AttentionDescriptor.swift:90-105: head block <= roundup8(D)
    d = mfa.AttentionDescriptor.make(64, 64, 3)
    k = mfa.kernel_descriptor(d, mfa.KernelType.forward)
    assert k.block_head == 8


@pytest.mark.parametrize("D", [257, 300, 384, 512, 1000])
def test_large_head_dimension_descriptor(D):
    # The reference's tables fall back to their last row for any D
    # (AttentionDescriptor+Parameters.swift:44-69); here D > 256 runs the D-blocked kernels,
    # whose head block is the head-dimension chunk they stream.
    for prec, chunk in ((None, 64), (mfa.Precision.FP16, 128), (mfa.Precision.BF16, 128)):
        d = mfa.AttentionDescriptor.make(64, 64, D, low_precision=prec is not None, precision=prec)
        for kind in (mfa.KernelType.forward, mfa.KernelType.backwardQuery,
                     mfa.KernelType.backwardKeyValue):
            k = mfa.kernel_descriptor(d, kind)
            assert k.block_head == chunk and k.head_dimension == D
            kern = mfa.attention_kernel(k)
            assert b"bigd" in kern.variant, kern.variant


def test_broadcast_compatibility_rules():
    base = mfa.AttentionDescriptor.make()
    ok = mfa.MultiHeadDescriptor.make(base, 2, 8, 64, 32, Hkv=2)
    assert ok.broadcast_mode == mfa.Broadcast.groupedQuery
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(ok)) == 1
    bad = mfa.MultiHeadDescriptor.make(base, 2, 8, 64, 32, Hkv=3, mode=mfa.Broadcast.groupedQuery)
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(bad)) == 0
    mqa = mfa.MultiHeadDescriptor.make(base, 1, 8, 64, 32, Hkv=1)
    assert mqa.broadcast_mode == mfa.Broadcast.multiQuery
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(mqa)) == 1
    cross = mfa.MultiHeadDescriptor.make(base, 1, 8, 64, 32, C=100)
    assert cross.broadcast_mode == mfa.Broadcast.crossAttention
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(cross)) == 1


def test_incompatible_shapes_fail_before_launch():
    base = mfa.AttentionDescriptor.make()
    bad = mfa.MultiHeadDescriptor.make(base, 2, 8, 64, 32, Hkv=3, mode=mfa.Broadcast.groupedQuery)
    b = mfa.AttentionBuffers()
    b.Q = b.K = b.V = b.O = 16  # never dereferenced: validation fails first
    st = mfa.lib.mfa_multihead_forward(ctypes.byref(bad), ctypes.byref(b), None)
    assert st == 1
    b2 = mfa.AttentionBuffers()  # null operands: the descriptor is checked first, then them
    assert mfa.lib.mfa_multihead_forward(ctypes.byref(bad), ctypes.byref(b2), None) == 1
    good = mfa.MultiHeadDescriptor.make(base, 2, 8, 64, 32, Hkv=2)
    assert mfa.lib.mfa_multihead_forward(ctypes.byref(good), ctypes.byref(b2), None) == 4
    empty = mfa.MultiHeadDescriptor.make(base, 2, 8, 0, 32, C=64)  # no queries: nothing to read
    assert mfa.lib.mfa_multihead_forward(ctypes.byref(empty), ctypes.byref(b2), None) == 0


def test_masking_heuristic_known_answers():
    # MaskingStrategyHeuristic.sequenceBucket / defaultRule (:47-60, :111-136)
    bucket = mfa.lib.mfa_masking_sequence_bucket
    assert [bucket(s) for s in (1, 100, 200, 640, 900, 2000, 3500, 9999)] == \
        [64, 128, 256, 512, 1024, 2048, 3072, 4096]
    rule = mfa.lib.mfa_masking_default_rule
    assert rule(100, 192) == 1 and rule(8192, 192) == 1
    assert rule(4096, 64) == 0
    assert rule(2048, 64) == 1
    assert rule(256, 128) == 1 and rule(512, 128) == 0
    assert rule(200, 64) == 1
    assert rule(1024, 256) == 0 and rule(512, 256) == 1
    assert rule(700, 32) == 1


def test_sparse_builders_known_answers():
    # SparseMQABuilder.buildSlidingWindow: [max(0, i - w/2), min(n, i + w/2))
    out = np.zeros((10, 2), dtype=np.uint32)
    mfa.lib.mfa_sparse_build_sliding_window(10, 4, out.ctypes.data)
    assert out.tolist() == [[max(0, i - 2), min(10, i + 2)] for i in range(10)]
    out1 = np.zeros((3, 2), dtype=np.uint32)
    mfa.lib.mfa_sparse_build_sliding_window(3, 0, out1.ctypes.data)  # window capped at 1
    assert out1.tolist() == [[0, 0], [1, 1], [2, 2]]
    pat = np.array([[0, 1, 1, 0], [0, 0, 0, 0], [1, 0, 0, 1]], dtype=np.uint8)
    rng = np.zeros((3, 2), dtype=np.uint32)
    mfa.lib.mfa_sparse_build_block_sparse(pat.ctypes.data, 3, 4, 16, rng.ctypes.data)
    assert rng.tolist() == [[16, 48], [0, 0], [0, 64]]


def test_flop_accounting():
    # C2 = 68.73 GFLOP, C3 = 549.76 GOP
    assert abs(mfa.attention_flops(1, 16, 4096, 4096, 128, causal=True) / 1e9 - 68.73) < 0.01
    assert abs(mfa.attention_flops(1, 16, 8192, 8192, 128) / 1e9 - 549.76) < 0.01
