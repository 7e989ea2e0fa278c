import sys, time, torch
sys.path.insert(0, 'metal-flash-attention-plus_amd/python')
import mfa_amd as mfa
P = mfa.Precision
n = 4096
a = (torch.rand((n, n), device='cuda') - 0.5).half()
b = (torch.rand((n, n), device='cuda') - 0.5).half()
c = torch.empty((n, n), device='cuda', dtype=torch.float16)
import os
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
for ta, tb, nn in ((0, 0, '0'), (0, 0, '3'), (0, 1, '0'), (1, 0, '0'), (0, 0, '0'), (0, 0, '3')):
    os.environ['MFA_GEMM_NN'] = nn
    f = lambda: mfa.gemm(a, b, c, n, n, n, P.FP16, P.FP16, transpose_a=bool(ta), transpose_b=bool(tb))
    for _ in range(5): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    ref = (a.float().T if ta else a.float()) @ (b.float().T if tb else b.float())
    err = (c.float() - ref).abs().max().item()
    print(f"T{ta}{tb} nn{nn} {ms:.4f} ms {2*n**3/ms/1e9:.1f} TF maxerr {err:.3e}")
