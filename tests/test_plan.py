"""CPU tests of the plan query (mfa_multihead_plan / mfa_quantized_plan): the dispatcher run
with launches recorded, so no GPU is needed.  The GPU twin (test_plan_gpu.py) checks that the
launches a real call issues are exactly these."""
import ctypes

import pytest

import mfa_amd as mfa

P = mfa.Precision
K = mfa.KernelType


def mh(B, H, S, D, causal=False, prec=P.FP16, C=None, Hkv=None):
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec, causal=causal)
    return mfa.MultiHeadDescriptor.make(base, B, H, S, D, C=C, Hkv=Hkv)


def one(plan):
    assert len(plan) == 1, plan
    return plan[0]


# BASELINE.json configs: C2 (headline) fp16 causal H16 S4096 D128; C3 H16 S8192 non-causal;
# C5 B8 H32 S4096 D256 fwd + bwd.
def test_c2_headline_runs_shared_tile_pair_kernel():
    p = one(mfa.multihead_plan(mh(1, 16, 4096, 128, causal=True)))
    assert p["name"] == "mfa_fwd2_share_kernel<F16, 128, 64, true, true, true, true>"
    assert p["threads"] == 512 and p["lds_bytes"] == 160 * 1024  # two rings + Q staging
    # 32 query blocks of 128 rows per head, mirrored in pairs: 16 x 16 heads.
    assert p["workgroups"] == 16 * 16


def test_large_causal_runs_stream_split_kernel():
    # Past the mirrored kernel's range (2048 128-row blocks): the key tiles of all heads are
    # cut into one equal range per CU (256 when no GPU is visible to ask).
    p = one(mfa.multihead_plan(mh(4, 16, 4096, 128, causal=True)))
    assert p["name"] == "mfa_fwd2_stream_kernel<F16, 128, 64>"
    # Two-slot ring of 64-key K/V tiles, one O row image of 128 rows above it, decision word.
    assert p["threads"] == 512 and p["lds_bytes"] == 4 * 64 * 128 * 2 + 128 * (128 * 4 + 16) + 16
    assert p["workgroups"] == 256


def test_c3_runs_adjacent_shared_tile_kernel():
    # Unmasked with >= 256 block pairs: adjacent 128-row blocks share every K/V tile.
    p = one(mfa.multihead_plan(mh(1, 16, 8192, 128)))
    assert p["name"] == "mfa_fwd_pipe_kernel"
    assert p["threads"] == 512 and p["workgroups"] == 32 * 16


def test_small_unmasked_runs_single_block_kernel():
    # Fewer than 256 pairs would leave CUs idle: one 4-wave workgroup per 128-row block.
    p = one(mfa.multihead_plan(mh(1, 16, 2048, 128)))
    assert p["name"].startswith("mfa_fwd2_kernel<F16, 128, 64, 2")
    assert p["threads"] == 256 and p["workgroups"] == 16 * 16


def test_c5_forward_and_backward_phases():
    d = mh(8, 32, 4096, 256)
    f = one(mfa.multihead_plan(d))
    assert f["name"] == "mfa_fwd2_share_kernel<F16, 256, 32, false, false, false, false>"
    q = one(mfa.multihead_plan(d, K.backwardQuery))
    kv = one(mfa.multihead_plan(d, K.backwardKeyValue))
    assert q["name"] == "mfa_bwd_q_fast_kernel<F16, 256, 32, false, 0>"
    assert kv["name"] == "mfa_bwd_kv_fast_kernel<F16, 256, 32, 0, false>"
    assert q["workgroups"] == 32 * 8 * 32 and kv["workgroups"] == 32 * 8 * 32
    for r in (f, q, kv):
        assert r["lds_bytes"] <= 160 * 1024


def test_bf16_and_d64_instantiations():
    assert one(mfa.multihead_plan(mh(1, 4, 1024, 128, prec=P.BF16)))["name"].startswith(
        "mfa_fwd2_kernel<BF16, 128")
    assert one(mfa.multihead_plan(mh(1, 16, 4096, 64, causal=True)))["name"] == \
        "mfa_fwd2_share_kernel<F16, 64, 64, true, true, true, true>"


def test_fp32_inputs_take_generic_kernel():
    base = mfa.AttentionDescriptor.make(low_precision=False)
    d = mfa.MultiHeadDescriptor.make(base, 1, 2, 256, 64)
    assert one(mfa.multihead_plan(d))["name"].startswith("mfa_fwd_kernel<")


def test_misaligned_query_falls_back_to_generic_kernel():
    d = mh(1, 2, 256, 64)
    b = mfa.AttentionBuffers()
    b.Q, b.K, b.V, b.O = 0x100002, 0x200000, 0x300000, 0x400000  # Q off 16-byte alignment
    out = mfa.KernelPlan()
    mfa.check(mfa.lib.mfa_multihead_plan(ctypes.byref(d), 0, ctypes.byref(b), ctypes.byref(out)))
    assert out.count == 1 and out.launches[0].name.startswith(b"mfa_fwd_kernel<")
    b.Q = 0x100000
    mfa.check(mfa.lib.mfa_multihead_plan(ctypes.byref(d), 0, ctypes.byref(b), ctypes.byref(out)))
    assert out.launches[0].name.startswith(b"mfa_fwd2_")


def test_quantized_plans():
    base = mfa.AttentionDescriptor.make(8192, 8192, 128, low_precision=True, precision=P.FP16)
    qi = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16, integer_matmul=True)
    assert one(mfa.quantized_plan(qi))["name"] == "mfa_fwd_i8_kernel<F16, 128, 128, 2, 2, true>"
    # Dequant-exact forward, FP16 Q + per-tensor INT8 K/V: one kernel widening the bytes as
    # it stages them (attention_fwd_kv8.hip), no pass.
    qx = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(qx)] == ["mfa_fwd2_kv8_kernel<F16, 128, 64, 1, false>"]
    # backwardQuery: one dequantisation pass per quantised operand (kv_dequant.hip), then the
    # tuned 16-bit kernel on the dense copies (K/V tiles stream through LDS) ...
    assert [r["name"] for r in mfa.quantized_plan(qx, K.backwardQuery)] == \
        ["mfa_kv_dequant_kernel<F16, 1>"] * 2 + ["mfa_bwd_q_fast_kernel<F16, 128, 64, false, 0>"]
    # ... except with few query rows per kv head, where the pass does not pay: the same kernel
    # stages the stored bytes through an LDS byte ring and widens them there (kv_bytes.h).
    few = mfa.AttentionDescriptor.make(64, 8192, 128, low_precision=True, precision=P.FP16)
    qf = mfa.quantized_descriptor(few, P.FP16, P.INT8, P.INT8, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(qf, K.backwardQuery)] == \
        ["mfa_bwd_q_fast_kernel<F16, 128, 64, false, 1>"]
    # backwardKeyValue reads each key block's K/V once into registers and widens them there:
    # the INT8 instantiation (SRC_I8 = 1), no pass.
    assert [r["name"] for r in mfa.quantized_plan(qx, K.backwardKeyValue)] == \
        ["mfa_bwd_kv_fast_kernel<F16, 128, 64, 1, false>"]
    # INT4 K/V with an FP16 Q: the same on-load kernel (SRC_I4 = 2).
    q4h = mfa.quantized_descriptor(base, P.FP16, P.INT4, P.INT4, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(q4h)] == ["mfa_fwd2_kv8_kernel<F16, 128, 64, 2, false>"]
    # BF16 Q at the same shape, and FP16 Q at D = 256 (BASELINE configs[4]'s width): the
    # same on-load kernel, no pass.
    bb = mfa.AttentionDescriptor.make(8192, 8192, 128, low_precision=True, precision=P.BF16)
    qb = mfa.quantized_descriptor(bb, P.BF16, P.INT8, P.INT8, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(qb)] == ["mfa_fwd2_kv8_kernel<BF16, 128, 64, 1, false>"]
    b256 = mfa.AttentionDescriptor.make(4096, 4096, 256, low_precision=True, precision=P.FP16)
    q256 = mfa.quantized_descriptor(b256, P.FP16, P.INT8, P.INT8, B=2, H=32)
    assert [r["name"] for r in mfa.quantized_plan(q256)] == ["mfa_fwd2_kv8_kernel<F16, 256, 32, 1, false>"]
    # Causal INT8 at the C2 shape: the mirrored shared-tile kernel widening K/V on load.
    c2 = mfa.AttentionDescriptor.make(4096, 4096, 128, causal=True, low_precision=True,
                                      precision=P.FP16)
    qc2 = mfa.quantized_descriptor(c2, P.FP16, P.INT8, P.INT8, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(qc2)] == ["mfa_fwd2_share_kv8_kernel<F16, 128, 64, 1>"]
    # A quantised Q takes the dequantisation pass for every operand.
    q4 = mfa.quantized_descriptor(base, P.INT8, P.INT4, P.INT4, B=1, H=16)
    names = [r["name"] for r in mfa.quantized_plan(q4)]
    assert names[:3] == ["mfa_kv_dequant_kernel<F16, 2>"] * 2 + ["mfa_kv_dequant_kernel<F16, 1>"]
    assert names[3] == "mfa_fwd_pipe_kernel"
    # A non-zero zero point leaves the integer-matmul kernel (dequant-exact path instead).
    zp = mfa.QuantizedTensor(None, int(P.INT8), 0.5, 3)
    assert mfa.quantized_plan(qi, K.forward, None, zp, zp)[-1]["name"].startswith("mfa_fwd2_kv8_kernel<")
    # Decode-like shapes (few query rows per kv head) read the quantised tensors directly.
    dec = mfa.AttentionDescriptor.make(16, 8192, 128, low_precision=True, precision=P.FP16)
    qd = mfa.quantized_descriptor(dec, P.FP16, P.INT8, P.INT8, B=1, H=4)
    names = [r["name"] for r in mfa.quantized_plan(qd)]
    assert names == ["mfa_fwd_decode16_kernel<F16, 128, 1>", "mfa_decode_merge_kernel"], names


def test_blockwise_kv_on_load_plans(monkeypatch):
    # Block-wise K/V scales (round 6): the on-load forward's block-wise instantiation, no
    # dequantisation pass, at D <= 128 when the block size is a multiple of a thread's chunk
    # (16 elements; 8 at D = 64); other block sizes, D = 256 and transposed K/V keep the pass.
    # By default it runs where the pass does not (fewer than 128 query rows per kv head; the
    # pass + 16-bit kernel is faster above); MFA_KV8_BW=1 takes it at any size.
    base = mfa.AttentionDescriptor.make(8, 8192, 128, low_precision=True, precision=P.FP16)
    few = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16, Hkv=4)

    def bwt(bs):
        t = mfa.QuantizedTensor(None, int(P.INT8), 1.0, 0)
        t.block_scales, t.block_size = 0x1000, bs
        return t
    assert [r["name"] for r in mfa.quantized_plan(few, K.forward, None, bwt(64), bwt(64))] == \
        ["mfa_fwd2_kv8_kernel<F16, 128, 64, 1, true>"]
    big = mfa.quantized_descriptor(mfa.AttentionDescriptor.make(
        8192, 8192, 128, low_precision=True, precision=P.FP16), P.FP16, P.INT8, P.INT8, B=1, H=16)
    assert [r["name"] for r in mfa.quantized_plan(big, K.forward, None, bwt(64), bwt(64))][:2] == \
        ["mfa_kv_dequant_kernel<F16, 1>"] * 2
    monkeypatch.setenv("MFA_KV8_BW", "1")

    def bw(bs, prec=P.INT8):
        t = mfa.QuantizedTensor(None, int(prec), 1.0, 0)
        t.block_scales, t.block_size = 0x1000, bs
        return t

    def names(D, bs, prec=P.INT8, causal=False, qp=P.FP16):
        base = mfa.AttentionDescriptor.make(8192, 8192, D, causal=causal, low_precision=True,
                                            precision=qp)
        q = mfa.quantized_descriptor(base, qp, prec, prec, B=1, H=16)
        return [r["name"] for r in mfa.quantized_plan(q, K.forward, None, bw(bs, prec), bw(bs, prec))]

    assert names(128, 64) == ["mfa_fwd2_kv8_kernel<F16, 128, 64, 1, true>"]
    assert names(128, 16, P.INT4) == ["mfa_fwd2_kv8_kernel<F16, 128, 64, 2, true>"]
    assert names(128, 128, qp=P.BF16) == ["mfa_fwd2_kv8_kernel<BF16, 128, 64, 1, true>"]
    assert names(64, 8) == ["mfa_fwd2_kv8_kernel<F16, 64, 64, 1, true>"]
    # Causal at D = 128: the adjacent-pair on-load kernel with the mask (the mirrored on-load
    # kernel takes per-tensor scales only).
    assert names(128, 32, causal=True) == ["mfa_fwd2_kv8_kernel<F16, 128, 64, 1, true>"]
    for D, bs in ((128, 24), (128, 8), (256, 64)):
        n = names(D, bs)
        assert n[:2] == ["mfa_kv_dequant_kernel<F16, 1>"] * 2, (D, bs, n)


def test_kv8_override_takes_the_dequant_pass(monkeypatch):
    # MFA_KV8=0 (A/B): the dequantisation pass + the 16-bit shared-tile kernel instead.
    monkeypatch.setenv("MFA_KV8", "0")
    base = mfa.AttentionDescriptor.make(8192, 8192, 128, low_precision=True, precision=P.FP16)
    qx = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=16)
    names = [r["name"] for r in mfa.quantized_plan(qx)]
    assert names[:2] == ["mfa_kv_dequant_kernel<F16, 1>"] * 2
    assert names[2] == "mfa_fwd_pipe_kernel" and len(names) == 3


def test_environment_override_is_visible_in_plan(monkeypatch):
    d = mh(1, 16, 4096, 128, causal=True)
    monkeypatch.setenv("MFA_FWD_PAIR", "o")
    assert one(mfa.multihead_plan(d))["name"] == "mfa_fwd2_pair_kernel<F16, 128, 64, 4, true>"
    monkeypatch.setenv("MFA_DISABLE_FAST", "1")
    assert one(mfa.multihead_plan(d))["name"].startswith("mfa_fwd_kernel<")


def test_attention_kernel_reports_dispatched_variant():
    for causal, kind in ((True, K.forward), (False, K.backwardQuery), (False, K.backwardKeyValue)):
        d = mfa.AttentionDescriptor.make(4096, 4096, 128, low_precision=True,
                                         precision=P.FP16, causal=causal)
        kern = mfa.attention_kernel(mfa.kernel_descriptor(d, kind))
        md = mfa.MultiHeadDescriptor.make(
            mfa.AttentionDescriptor.make(low_precision=True, precision=P.FP16), 1, 1, 4096, 128)
        p = one(mfa.multihead_plan(md, kind))
        assert kern.variant.decode() == p["name"]
        assert kern.threadgroup_size == p["threads"]
        assert kern.threadgroup_memory_allocation == p["lds_bytes"]


def test_empty_shape_plans_nothing():
    assert mfa.multihead_plan(mh(1, 2, 0, 64, C=64)) == []
    assert mfa.multihead_plan(mh(1, 2, 0, 64, C=0)) == []
    for kind in (K.backwardQuery, K.backwardKeyValue):
        assert mfa.multihead_plan(mh(1, 2, 0, 64, C=64), kind) == []  # dK = dV = 0, no kernel


@pytest.mark.parametrize("kind", [K.forward, K.backwardQuery, K.backwardKeyValue])
def test_queries_over_no_keys_rejected(kind):
    """A softmax over zero keys is undefined; the reference refuses non-positive sequence
    lengths (QuantizedAttention.swift:791).  The call fails before any launch."""
    with pytest.raises(mfa.MFAError, match="softmax over no keys"):
        mfa.multihead_plan(mh(1, 2, 64, 64, C=0), kind)


def test_invalid_descriptor_fails_like_the_call():
    bad = mh(2, 8, 64, 32, Hkv=3)
    bad.broadcast_mode = int(mfa.Broadcast.groupedQuery)
    with pytest.raises(mfa.MFAError):
        mfa.multihead_plan(bad)


def test_no_launch_recorded_by_plan():
    mfa.last_launches()
    mfa.multihead_plan(mh(1, 16, 4096, 128, causal=True))
    assert mfa.last_launches() == []


@pytest.mark.parametrize("qh,kh,vh,kc,vc,ok", [
    (8, 2, 2, 64, 64, True),    # GQA-shaped custom
    (8, 3, 3, 64, 64, False),   # H % Hkv != 0
    (8, 2, 4, 64, 64, False),   # K and V head counts differ
    (8, 2, 2, 64, 32, False),   # K and V sequence lengths differ
])
def test_custom_broadcast_still_checks_addressable_shapes(qh, kh, vh, kc, vc, ok):
    base = mfa.AttentionDescriptor.make()
    d = mfa.MultiHeadDescriptor.make(base, 2, qh, 64, 32, Hkv=kh, C=kc, mode=mfa.Broadcast.custom)
    d.value_shape = mfa.MultiHeadShape(2, vh, vc, 32, 0)
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(d)) == int(ok)
    d2 = mfa.MultiHeadDescriptor.make(base, 2, qh, 64, 32, Hkv=kh, C=kc, mode=mfa.Broadcast.custom)
    d2.key_shape = mfa.MultiHeadShape(3, kh, kc, 32, 0)  # batch mismatch
    assert mfa.lib.mfa_multihead_broadcast_compatible(ctypes.byref(d2)) == 0


def test_custom_mismatch_rejected_by_the_call():
    base = mfa.AttentionDescriptor.make()
    d = mfa.MultiHeadDescriptor.make(base, 2, 8, 64, 32, Hkv=2, mode=mfa.Broadcast.custom)
    d.value_shape = mfa.MultiHeadShape(2, 2, 48, 32, 0)  # V shorter than K
    b = mfa.AttentionBuffers()
    b.Q = b.K = b.V = b.O = 0x100000  # never dereferenced: validation fails first
    assert mfa.lib.mfa_multihead_forward(ctypes.byref(d), ctypes.byref(b), None) == 1
    with pytest.raises(mfa.MFAError):
        mfa.multihead_plan(d)


# transposeState (AttentionDescriptor.swift:150-165): O -> O and dO, Q/K/V -> dQ/dK/dV.  Every
# transpose is honoured; strided operands and outputs run the generic kernels.
@pytest.mark.parametrize("tr", [(False, False, False, True), (True, True, True, False),
                                (True, True, True, True), (False, True, False, True)])
def test_transposes_accepted_on_generic_kernels(tr):
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.FP16, transpose=tr)
    d = mfa.MultiHeadDescriptor.make(base, 1, 2, 128, 64)
    assert one(mfa.multihead_plan(d))["name"].startswith("mfa_fwd_kernel<")
    assert one(mfa.multihead_plan(d, K.backwardQuery))["name"].startswith("mfa_bwd_q_kernel<")
    assert one(mfa.multihead_plan(d, K.backwardKeyValue))["name"].startswith("mfa_bwd_kv_kernel<")
    full = mfa.AttentionDescriptor.make(128, 128, 64, transpose=tr)
    for kind in (K.forward, K.backwardQuery, K.backwardKeyValue):
        kd = mfa.kernel_descriptor(full, kind)
        assert kd.transpose_state[int(mfa.Operand.O)] == tr[3]
        assert kd.transpose_state[int(mfa.Operand.dO)] == tr[3]
        assert kd.transpose_state[int(mfa.Operand.dQ)] == tr[0]
        assert kd.transpose_state[int(mfa.Operand.dK)] == tr[1]
        assert kd.transpose_state[int(mfa.Operand.dV)] == tr[2]


def test_quantized_transposes_accepted():
    base = mfa.AttentionDescriptor.make(256, 256, 128, low_precision=True, precision=P.FP16,
                                        transpose=(False, True, False, True))
    qd = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=2)
    names = [r["name"] for r in mfa.quantized_plan(qd)]
    assert names[-1].startswith("mfa_fwd_kernel<")  # transposed O: generic kernel


@pytest.mark.parametrize("D", [288, 320, 384, 512, 1024])
@pytest.mark.parametrize("prec,tag", [(P.FP32, "Arith32<64>, 64"), (P.FP16, "Arith16<F16, 128>, 128"),
                                      (P.BF16, "Arith16<BF16, 128>, 128")])
def test_large_head_dimension_plan(D, prec, tag):
    lp = prec != P.FP32
    base = mfa.AttentionDescriptor.make(low_precision=lp, precision=prec if lp else None,
                                        causal=True)
    d = mfa.MultiHeadDescriptor.make(base, 2, 3, 300, D)
    f = one(mfa.multihead_plan(d))
    assert f["name"] == f"mfa_fwd_bigd_kernel<{tag}>"
    nob = -(-D // (64 if prec == P.FP32 else 128))
    assert f["workgroups"] == 3 * 2 * 3 * nob  # 128-row blocks x B x H x output slices
    q = one(mfa.multihead_plan(d, K.backwardQuery))
    kv = one(mfa.multihead_plan(d, K.backwardKeyValue))
    assert q["name"].startswith("mfa_bwd_q_bigd_kernel<" + tag)
    assert kv["name"].startswith("mfa_bwd_kv_bigd_kernel<" + tag)


def test_large_head_dimension_quantized_plan():
    # INT8 K/V at D = 384: one dequantisation pass per operand, then the D-blocked forward,
    # whatever the number of query rows (decode shapes included).
    for R in (1, 512):
        base = mfa.AttentionDescriptor.make(R, 1024, 384, low_precision=True, precision=P.FP16)
        qd = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=1, H=2)
        names = [r["name"] for r in mfa.quantized_plan(qd)]
        assert names[:2] == ["mfa_kv_dequant_kernel<F16, 1>"] * 2, names
        assert names[2].startswith("mfa_fwd_bigd_kernel<Arith16<F16, 128>")


def test_absorbed_mla_rejects_transposes():
    d = mla_desc(1, 2, 64, 64, 64, 256)
    d.base.transpose_q = 1
    p = 0x100000
    st = mfa.lib.mfa_mla_forward_absorbed(ctypes.byref(d), p, p, p, p, None, p, None, None)
    assert st == 2


def mla_desc(B, H, Sq, Skv, D, Lat):
    d = mfa.MLADescriptor()
    d.base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.BF16)
    d.batch_size, d.num_heads = B, H
    d.sequence_length_q, d.sequence_length_kv = Sq, Skv
    d.head_dim, d.kv_latent_dim = D, Lat
    d.precision = int(P.BF16)
    return d


def test_mla_one_decompressed_buffer_is_an_error():
    d = mla_desc(1, 2, 64, 64, 64, 256)
    p = 0x100000
    st = mfa.lib.mfa_mla_forward(ctypes.byref(d), p, p, p, p, p, None, p, None, None)
    assert st == 4 and b"both" in mfa.lib.mfa_last_error()
    st = mfa.lib.mfa_mla_forward(ctypes.byref(d), p, p, p, p, None, p, p, None, None)
    assert st == 4


def test_absorbed_workspace_covers_split_partials():
    # Decode (S_q 1, B 32, H 16): 16 query rows per batch item -> 32 blocks, split keys.
    dec = mfa.lib.mfa_mla_absorbed_workspace_size(ctypes.byref(mla_desc(32, 16, 1, 4096, 128, 512)))
    qt = 32 * 16 * 512 * 2
    assert dec > 2 * qt  # Q~, O~ and the FP32 partials
    # Prefill (S_q 4096): enough blocks, no split: Q~ and O~ only.
    pre = mfa.lib.mfa_mla_absorbed_workspace_size(ctypes.byref(mla_desc(1, 16, 4096, 4096, 128, 512)))
    assert pre == 2 * 16 * 4096 * 512 * 2


def test_decode_bench_shape_is_one_launch():
    # The bench's decode rows (B32 H16 S_kv 8192, S_q 1 and 16): one split per unit.
    for R in (1, 16):
        base = mfa.AttentionDescriptor.make(R, 8192, 128, low_precision=True, precision=P.FP16)
        desc = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=32, H=16)
        assert [r["name"] for r in mfa.quantized_plan(desc)] == ["mfa_fwd_decode16_kernel<F16, 128, 1>"]


def test_decode_kernel_forms():
    # Split-KV decode routing (attention_decode.hip): at most 16 rows per kv head take the
    # 16x16x32 kernel at every width, more rows the 32-row kernel; the merge pass runs one row
    # per wave, or one row per 4-wave workgroup above 32 partials (key splits) per row.
    def names(R, C, D, B, H, Hkv, kv, causal=False, window=None):
        base = mfa.AttentionDescriptor.make(R, C, D, causal=causal, window=window,
                                            low_precision=True, precision=P.FP16)
        return [r["name"] for r in mfa.quantized_plan(
            mfa.quantized_descriptor(base, P.FP16, kv, kv, B=B, H=H, Hkv=Hkv))]
    assert names(1, 16384, 256, 8, 32, 4, P.INT8) == ["mfa_fwd_decode16_kernel<F16, 256, 1>",
                                                     "mfa_decode_merge_kernel"]
    assert names(4, 65536, 128, 1, 32, 8, P.INT8) == ["mfa_fwd_decode16_kernel<F16, 128, 1>",
                                                     "mfa_decode_merge4_kernel"]
    assert names(1, 8192, 256, 32, 16, 16, P.INT4) == ["mfa_fwd_decode16_kernel<F16, 256, 2>"]
    assert names(4, 8192, 128, 4, 32, 4, P.INT4)[0] == "mfa_fwd_decode_kernel<F16, 128, 2>"  # 32 rows
    assert names(16, 4096, 64, 2, 8, 8, P.INT8, causal=True)[0] == "mfa_fwd_decode16_kernel<F16, 64, 1>"
    assert names(8, 4096, 128, 2, 8, 8, P.INT4, window=64)[0] == "mfa_fwd_decode16_kernel<F16, 128, 2>"
