"""Runtime quantiser timing at the C3 K/V size (16.8 M fp32 elements), HIP events."""
import sys
sys.path.insert(0, "metal-flash-attention-plus_amd/python")
import torch
import mfa_amd as mfa
P = mfa.Precision
x = torch.randn((16 * 8192, 128), device="cuda:0")
for mode, name in ((mfa.QuantMode.tensorWise, "tensor"), (mfa.QuantMode.rowWise, "row"), (mfa.QuantMode.blockwise, "block64")):
    for tgt in (P.INT8, P.INT4):
        f = lambda: mfa.quantize(x, tgt, mode, x.shape[0], x.shape[1], 64)
        for _ in range(3):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            f()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name} {tgt}: {ms*1e3:.1f} us per call ({x.numel()*4/ms/1e6:.0f} GB/s of fp32 input)", flush=True)
