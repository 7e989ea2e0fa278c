"""Library-owned scratch is per (device, stream): two MLA calls on two streams
with library-owned K/V (mfa_mla_forward) or Q~/O~/partials (absorbed) give each the result
they give alone; a caller workspace of mfa_mla_absorbed_workspace_size() bytes holds the
split-KV partials too."""
import ctypes

import pytest
import torch

import mfa_amd as mfa

pytestmark = pytest.mark.gpu
BF16 = mfa.Precision.BF16


def mla_inputs(B, H, Sq, Skv, D, Lat, seed, dev):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    r = lambda *s: ((torch.rand(s, generator=g, device=dev) - 0.5) * 0.5).to(torch.bfloat16)
    return r(B * Skv, Lat), r(Lat, H * D), r(Lat, H * D), r(B, H, Sq, D)


@pytest.mark.parametrize("absorbed,shape", [
    (False, (1, 8, 512, 512, 128, 512)),
    (True, (1, 8, 512, 512, 128, 512)),
    (True, (32, 16, 1, 2048, 128, 512)),   # decode: split keys, partials in scratch
])
def test_two_streams_do_not_share_scratch(gpu, absorbed, shape):
    B, H, Sq, Skv, D, Lat = shape
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=BF16)
    fn = mfa.mla_forward_absorbed if absorbed else mfa.mla_forward
    ins = [mla_inputs(B, H, Sq, Skv, D, Lat, s, gpu) for s in (3, 4)]
    outs = [torch.zeros((B, H, Sq, D), dtype=torch.float32, device=gpu) for _ in range(2)]
    ref = []
    for (lat, wk, wv, q), o in zip(ins, outs):
        fn(base, lat, wk, wv, q, o, B, H, Sq, Skv, D, Lat, BF16)
        torch.cuda.synchronize()
        ref.append(o.clone())
        o.zero_()
    streams = [torch.cuda.Stream(device=gpu) for _ in range(2)]
    for _ in range(10):  # interleaved on two streams, no synchronisation between them
        for (lat, wk, wv, q), o, s in zip(ins, outs, streams):
            fn(base, lat, wk, wv, q, o, B, H, Sq, Skv, D, Lat, BF16, stream=s.cuda_stream)
    torch.cuda.synchronize()
    for o, r in zip(outs, ref):
        assert torch.equal(o, r)


def test_absorbed_caller_workspace_holds_partials(gpu):
    B, H, Sq, Skv, D, Lat = 32, 16, 1, 2048, 128, 512
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=BF16)
    lat, wk, wv, q = mla_inputs(B, H, Sq, Skv, D, Lat, 5, gpu)
    d = mfa.MLADescriptor()
    d.base = base
    d.batch_size, d.num_heads = B, H
    d.sequence_length_q, d.sequence_length_kv = Sq, Skv
    d.head_dim, d.kv_latent_dim = D, Lat
    d.precision = int(BF16)
    n = mfa.lib.mfa_mla_absorbed_workspace_size(ctypes.byref(d))
    ws = torch.full((n,), 0xFF, dtype=torch.uint8, device=gpu)
    o1 = torch.zeros((B, H, Sq, D), dtype=torch.float32, device=gpu)
    o2 = torch.zeros_like(o1)
    mfa.mla_forward_absorbed(base, lat, wk, wv, q, o1, B, H, Sq, Skv, D, Lat, BF16)
    mfa.mla_forward_absorbed(base, lat, wk, wv, q, o2, B, H, Sq, Skv, D, Lat, BF16, workspace=ws)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    assert torch.isfinite(o1).all()
