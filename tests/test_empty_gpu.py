"""GPU edge cases at the sequence boundaries: empty query sequences are no-ops (backward
writes dK = dV = 0, the sums over no queries), and queries over an empty key sequence are
refused before any launch (the reference refuses non-positive sequence lengths,
QuantizedAttention.swift:791).  Empty tensors reach the C ABI as null pointers, which the
calls accept for operands with no elements."""
import pytest
import torch

import mfa_amd as mfa

pytestmark = pytest.mark.gpu
P = mfa.Precision
DEV = "cuda:0"


def desc(B, H, R, C, D, Hkv=None, prec=P.FP16):
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec)
    return mfa.MultiHeadDescriptor.make(base, B, H, R, D, Hkv=Hkv, C=C)


def half(*shape):
    return (torch.rand(shape, device=DEV) - 0.5).half()


@pytest.mark.parametrize("C", [0, 64])
def test_forward_no_queries_is_a_noop(gpu, C):
    B, H, D = 2, 4, 64
    q, o = half(B, H, 0, D), torch.empty((B, H, 0, D), device=DEV)
    k, v = half(B, H, C, D), half(B, H, C, D)
    mfa.last_launches()
    mfa.MultiHeadAttention().forward(desc(B, H, 0, C, D), q, k, v, o)
    torch.cuda.synchronize()
    assert mfa.last_launches() == []


@pytest.mark.parametrize("prec", [P.FP16, P.FP32])
def test_forward_no_keys_refused(gpu, prec):
    B, H, R, D = 1, 2, 64, 64
    dt = torch.float16 if prec == P.FP16 else torch.float32
    q = torch.rand((B, H, R, D), device=DEV).to(dt)
    k = v = torch.empty((B, H, 0, D), dtype=dt, device=DEV)
    o = torch.full((B, H, R, D), 7.0, device=DEV)
    d = desc(B, H, R, 0, D, prec=prec)
    if prec == P.FP32:
        d.base = mfa.AttentionDescriptor.make()
    with pytest.raises(mfa.MFAError, match="softmax over no keys"):
        mfa.MultiHeadAttention().forward(d, q, k, v, o)
    torch.cuda.synchronize()
    assert (o == 7.0).all()  # untouched


@pytest.mark.parametrize("phase", ["both", "keyValue", "query"])
@pytest.mark.parametrize("H,Hkv", [(4, 4), (8, 2)])
def test_backward_no_queries_zero_kv_grads(gpu, phase, H, Hkv):
    B, C, D = 2, 96, 64
    e = lambda *s: torch.empty(s, device=DEV)
    q, do = half(B, H, 0, D), half(B, H, 0, D)
    k, v = half(B, Hkv, C, D), half(B, Hkv, C, D)
    o, dq = e(B, H, 0, D), e(B, H, 0, D)
    l = torch.empty((B, H, 0), dtype=torch.float16, device=DEV)
    dbuf = torch.empty((B, H, 0), dtype=torch.bfloat16, device=DEV)
    dk = torch.full((B, Hkv, C, D), float("nan"), device=DEV)
    dv = torch.full((B, Hkv, C, D), float("nan"), device=DEV)
    mfa.last_launches()
    mfa.MultiHeadAttention().backward(desc(B, H, 0, C, D, Hkv=Hkv), q, k, v, o, do, l, dq, dk,
                                      dv, dbuf, phase=phase)
    torch.cuda.synchronize()
    assert mfa.last_launches() == []  # memsets only
    if phase == "query":
        assert torch.isnan(dk).all() and torch.isnan(dv).all()
    else:
        assert (dk == 0).all() and (dv == 0).all()


def test_backward_no_keys_refused(gpu):
    B, H, R, D = 1, 2, 64, 64
    q, do = half(B, H, R, D), half(B, H, R, D)
    k = v = torch.empty((B, H, 0, D), dtype=torch.float16, device=DEV)
    o, dq = torch.zeros((B, H, R, D), device=DEV), torch.zeros((B, H, R, D), device=DEV)
    l = torch.zeros((B, H, R), dtype=torch.float16, device=DEV)
    dbuf = torch.zeros((B, H, R), dtype=torch.bfloat16, device=DEV)
    dk = dv = torch.empty((B, H, 0, D), device=DEV)
    with pytest.raises(mfa.MFAError, match="softmax over no keys"):
        mfa.MultiHeadAttention().backward(desc(B, H, R, 0, D), q, k, v, o, do, l, dq, dk, dv,
                                          dbuf)


def quant_setup(R, C, B=1, H=2, D=64):
    base = mfa.AttentionDescriptor.make(R, C, D, low_precision=True, precision=P.FP16)
    d = mfa.quantized_descriptor(base, P.FP16, P.INT8, P.INT8, B=B, H=H)
    tq = mfa.quantized_tensor(half(B, H, R, D), P.FP16)
    tk = mfa.quantized_tensor(torch.randint(-127, 128, (B, H, C, D), dtype=torch.int8,
                                            device=DEV), P.INT8, scale=0.01)
    tv = mfa.quantized_tensor(torch.randint(-127, 128, (B, H, C, D), dtype=torch.int8,
                                            device=DEV), P.INT8, scale=0.01)
    return d, tq, tk, tv


def test_quantized_forward_empty_sequences(gpu):
    B, H, D = 1, 2, 64
    d, tq, tk, tv = quant_setup(0, 64)
    mfa.last_launches()
    mfa.QuantizedAttention().forward(d, tq, tk, tv, torch.empty((B, H, 0, D), device=DEV))
    torch.cuda.synchronize()
    assert mfa.last_launches() == []
    d, tq, tk, tv = quant_setup(64, 0)
    o = torch.empty((B, H, 64, D), device=DEV)
    with pytest.raises(mfa.MFAError, match="softmax over no keys"):
        mfa.QuantizedAttention().forward(d, tq, tk, tv, o)


def test_quantized_backward_key_value_no_queries(gpu):
    B, H, C, D = 1, 2, 64, 64
    d, tq, tk, tv = quant_setup(0, C)
    dk = torch.full((B, H, C, D), float("nan"), device=DEV)
    dv = torch.full((B, H, C, D), float("nan"), device=DEV)
    e = torch.empty((B, H, 0), device=DEV)
    mfa.QuantizedAttention().backwardKeyValue(d, tq, tk, tv, torch.empty((B, H, 0, D), device=DEV),
                                              e, e, dk, dv)
    torch.cuda.synchronize()
    assert (dk == 0).all() and (dv == 0).all()


def test_mla_no_keys_refused(gpu):
    B, H, Sq, D, Lat = 1, 2, 16, 64, 256
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=P.FP16)
    lat = torch.empty((B, 0, Lat), dtype=torch.float16, device=DEV)
    wk, wv = half(Lat, H * D), half(Lat, H * D)
    q = half(B, H, Sq, D)
    o = torch.empty((B, H, Sq, D), device=DEV)
    kb = vb = torch.empty((B, 0, H, D), dtype=torch.float16, device=DEV)
    with pytest.raises(mfa.MFAError):
        mfa.mla_forward(base, lat, wk, wv, q, o, B, H, Sq, 0, D, Lat, P.FP16, k_buf=kb, v_buf=vb)
