"""The reference's static tables through the C ABI: QuantizedKernelLayoutManifest
(QuantizedKernelLayoutManifest.swift:59-211) and the GLUON constants
(AttentionKernel+GluonOptimizations.swift:12-22).  Known answers are the reference's own
comments and tests (QuantizedAttentionTest.swift:380-398, MinimalGluonTests.swift:6-40)."""
import pytest

import mfa_amd as mfa

K = mfa.KernelType


def slot(kind, key):
    names = [mfa.lib.mfa_quantized_slot_name(k).decode() for k in range(mfa.QSLOT_COUNT)]
    return mfa.lib.mfa_quantized_slot(int(kind), names.index(key))


def test_key_names_in_declaration_order():
    names = [mfa.lib.mfa_quantized_slot_name(k).decode() for k in range(mfa.QSLOT_COUNT)]
    assert names[:5] == ["qData", "kData", "vData", "output", "gradOutput"]
    assert names[-2:] == ["scratch0", "scratch1"] and len(set(names)) == 39
    assert mfa.lib.mfa_quantized_slot_name(39) is None


def test_canonical_slots_follow_assignment_comments():
    # QuantizedKernelLayoutManifest.swift:73-113 (the `// n` comments).
    fwd = {"qData": 0, "kData": 1, "vData": 2, "output": 3, "logsumexp": 4, "qScale": 9,
           "qZeroPoint": 10, "kScale": 11, "kZeroPoint": 12, "vScale": 13, "vZeroPoint": 14,
           "qBlockScales": 17, "vBlockZeroPoints": 22, "qPrecomputedSums": 23,
           "vPrecomputedSums": 25, "qStrides": 26, "oStrides": 29, "maskBuffer": 30}
    for k, v in fwd.items():
        assert slot(K.forward, k) == v, k
    bq = {"gradOutput": 3, "gradQuery": 5, "dValues": 6, "dims": 15, "steClipRange": 16}
    for k, v in bq.items():
        assert slot(K.backwardQuery, k) == v, k
    bkv = {"gradOutput": 3, "dValues": 6, "gradKey": 7, "gradValue": 8}
    for k, v in bkv.items():
        assert slot(K.backwardKeyValue, k) == v, k


def test_backward_key_value_binds_o_strides_within_metal_limit():
    # QuantizedAttentionTest.swift:380-398
    s = mfa.quantized_layout(K.backwardKeyValue)["oStrides"]
    assert s != -1 and 0 <= s <= 30


@pytest.mark.parametrize("kind,unbound", [
    (K.forward, ["gradOutput", "gradQuery", "dValues", "gradKey", "gradValue", "dims",
                 "steClipRange", "maskMetadata"]),
    (K.backwardQuery, ["output", "gradKey", "gradValue", "maskBuffer", "qPrecomputedSums",
                       "numHeads", "scratch0"]),
    (K.backwardKeyValue, ["output", "gradQuery", "maskBuffer", "kPrecomputedSums"]),
    (K.mlaCompressed, ["kData", "vData", "logsumexp", "qScale", "maskBuffer"]),
])
def test_unlisted_keys_have_no_slot(kind, unbound):
    for k in unbound:
        assert slot(kind, k) == -1, (kind, k)


def test_every_bound_slot_is_unique_per_kernel_and_metal_range():
    for kind in (K.forward, K.backwardQuery, K.backwardKeyValue, K.mlaCompressed):
        lay = mfa.quantized_layout(kind)
        bound = [v for v in lay.values() if v >= 0]
        assert all(0 <= v <= 30 for v in bound)
        assert len(bound) == len(set(bound)), kind
    assert mfa.lib.mfa_quantized_slot_table(K.forward, None, 0) == 25
    assert mfa.lib.mfa_quantized_slot_table(K.mlaCompressed, None, 0) == 2
    assert mfa.lib.mfa_quantized_slot_table(7, None, 0) == -1


def test_metadata_keys_have_no_slot_anywhere():
    for kind in (K.forward, K.mlaCompressed):
        for k in ("numHeads", "headDimension", "sequenceLength", "scratch0", "scratch1"):
            assert slot(kind, k) == -1


def test_gluon_constants():
    # MinimalGluonTests.swift:6-40
    split, sync, sub = mfa.gluon_constants()
    assert (split, sync, sub) == (4, 2, 16)
    assert split & (split - 1) == 0 and sub % 8 == 0 and 2 <= sync <= 4


def test_gluon_never_enabled_for_library_plans():
    # shouldEnableGluonOptimizations (:314-320) on the block dimensions: the kernel plans cap
    # traversal at 128, so the predicate is false for every plan this library makes.
    assert mfa.lib.mfa_gluon_should_enable(512, 64) == 1
    assert mfa.lib.mfa_gluon_should_enable(511, 256) == 0
    for d in (32, 64, 128, 256):
        desc = mfa.AttentionDescriptor.make(4096, 4096, d, low_precision=True,
                                            precision=mfa.Precision.FP16)
        for kind in (K.forward, K.backwardQuery, K.backwardKeyValue):
            kd = mfa.kernel_descriptor(desc, kind)
            assert mfa.lib.mfa_gluon_should_enable(kd.block_traversal, kd.block_head) == 0
