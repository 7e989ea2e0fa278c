"""Development: interleaved A/B of MFA_GEMM_IMG on 4096^3 fp16 NN/NT/TN and the C4 decompress shape."""
import os, sys, torch
os.environ.setdefault("MFA_DEV", "1")  # the library reads A/B switches only under MFA_DEV=1
sys.path.insert(0, 'metal-flash-attention-plus_amd/python')
import mfa_amd as mfa
P = mfa.Precision


def timed(f, n=30):
    for _ in range(5): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


for (M, N, K) in ((4096, 4096, 4096), (4096, 2048, 512)):
    a = (torch.rand((M, K), device='cuda') - 0.5).half()
    b = (torch.rand((K, N), device='cuda') - 0.5).half()
    c = torch.empty((M, N), device='cuda', dtype=torch.float16)
    res = {}
    for r in range(6):
        for img in ('0', '1'):
            os.environ['MFA_GEMM_IMG'] = img
            f = lambda: mfa.gemm(a, b, c, M, N, K, P.FP16, P.FP16)
            res.setdefault(img, []).append(timed(f))
            if r == 0:
                err = (c.float() - a.float() @ b.float()).abs().max().item()
                print(f"{M}x{N}x{K} img{img} maxerr {err:.3e}")
    for img, v in res.items():
        v = sorted(v)[1:-1]
        ms = sum(v) / len(v)
        print(f"{M}x{N}x{K} img{img} {ms*1e3:.1f} us {2*M*N*K/ms/1e9:.1f} TF")
