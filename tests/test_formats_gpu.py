"""GPU round trip of the persisted QuantizedTensor format: K/V quantised on the GPU
(mfa_quantize), encoded to the Codable JSON, decoded back into HBM, then run through
QuantizedAttention.forward — the output must be bit-identical to the run on the original
device buffers, for tensor-wise, block-wise and row-wise modes."""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import mfa_formats as F

pytestmark = pytest.mark.gpu
P = mfa.Precision
DEV = "cuda:0"


@pytest.mark.parametrize("mode", [F.QuantizationMode.tensor_wise(), F.QuantizationMode.blockwise(32),
                                  F.QuantizationMode.row_wise()], ids=lambda m: m.case)
@pytest.mark.parametrize("prec", [P.INT8, P.INT4])
def test_quantized_tensor_json_round_trip(gpu, mode, prec):
    B, H, S, D = 1, 2, 96, 64
    g = torch.Generator(device=DEV).manual_seed(5)
    q = torch.randn((B, H, S, D), device=DEV, generator=g).half()
    k = torch.randn((B, H, S, D), device=DEV, generator=g)
    v = torch.randn((B, H, S, D), device=DEV, generator=g)
    view = lambda x: x.view(B * H * S, D)
    kr = F.QuantizedTensorRecord.quantize(view(k), prec, mode)
    vr = F.QuantizedTensorRecord.quantize(view(v), prec, mode)
    kd = F.QuantizedTensorRecord.decode(kr.encode(), DEV)
    vd = F.QuantizedTensorRecord.decode(vr.encode(), DEV)
    assert torch.equal(kd.data, kr.data) and kd.parameters == kr.parameters
    if mode.case != "tensorWise":
        assert torch.equal(kd.block_scales, kr.block_scales)
    if mode.case == "rowWise":
        with pytest.raises(mfa.MFAError):
            kd.abi()
        return

    base = mfa.AttentionDescriptor.make(S, S, D, low_precision_intermediates=False)
    desc = mfa.quantized_descriptor(base, P.FP16, prec, prec, B=B, H=H)
    tq = mfa.quantized_tensor(q, P.FP16)
    outs = []
    for kk, vv in ((kr, vr), (kd, vd)):
        o = torch.full((B, H, S, D), float("nan"), device=DEV)
        mfa.QuantizedAttention().forward(desc, tq, kk.abi(), vv.abi(), o)
        torch.cuda.synchronize()
        outs.append(o)
    assert torch.isfinite(outs[0]).all()
    assert torch.equal(outs[0], outs[1])
    # and the dequantised view agrees with the unquantised input to the format's resolution
    deq = torch.empty(B * H * S * D, device=DEV)
    mfa.check(mfa.lib.mfa_dequantize(mfa.ctypes.byref(kd.abi()), B * H * S * D, D,
                                     deq.data_ptr(), None))
    torch.cuda.synchronize()
    rel = (deq.view_as(k) - k).norm() / k.norm()
    assert rel.item() < (0.02 if prec == P.INT8 else 0.25)
