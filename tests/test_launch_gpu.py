"""Launch plumbing on the GPU (csrc/mfa_launch.h, mfa_api.cpp scratch):
 * the dynamic-LDS attribute is set per (kernel, device), not per kernel signature: three
   forward kernels with the same FwdParams signature and different LDS sizes each get their
   own entry in a fresh process (a once-flag per signature skipped all but the
   first);
 * mfa_release_scratch frees the scratch a stream holds (L when the caller passes none);
 * the plan record reports how many launches a call issues (`total`)."""
import os
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

_REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_SCRIPT = textwrap.dedent("""
    import sys, torch
    sys.path.insert(0, %r)
    import mfa_amd as mfa
    dev = torch.device("cuda:0")
    mha = mfa.MultiHeadAttention()
    names = []
    def run(S, D, dtype, prec, causal):
        q, k, v = (torch.randn(1, 2, S, D, device=dev).to(dtype) * 0.3 for _ in range(3))
        o = torch.empty(1, 2, S, D, device=dev)
        base = mfa.AttentionDescriptor.make(low_precision=dtype != torch.float32,
                                            precision=prec, causal=causal)
        desc = mfa.MultiHeadDescriptor.make(base, 1, 2, S, D)
        mha.forward(desc, q, k, v, o)
        torch.cuda.synchronize()
        names.append(mfa.last_launches()[-1]["name"])
        return o
    assert mfa.lib.mfa_kernel_attribute_count() == 0
    run(256, 128, torch.float16, mfa.Precision.FP16, False)
    run(2048, 128, torch.float16, mfa.Precision.FP16, True)
    run(256, 64, torch.float32, mfa.Precision.FP32, False)
    n = mfa.lib.mfa_kernel_attribute_count()
    assert len(set(names)) == 3, names
    assert n == 3, (n, names)
    print("OK", n, names)
""")


def test_lds_attribute_per_kernel_fresh_process():
    code = _SCRIPT % os.path.join(_REPO, "metal-flash-attention-plus_amd", "python")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "OK 3" in r.stdout


def test_release_scratch_and_plan_total():
    import torch
    sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))
    import mfa_amd as mfa

    dev = torch.device("cuda:0")
    s = torch.cuda.Stream(dev)
    q, k, v = (torch.randn(1, 2, 256, 64, device=dev).half() for _ in range(3))
    o = torch.empty(1, 2, 256, 64, device=dev)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
    desc = mfa.MultiHeadDescriptor.make(base, 1, 2, 256, 64)
    with torch.cuda.stream(s):
        mfa.MultiHeadAttention().forward(desc, q, k, v, o, None, stream=s.cuda_stream)
    s.synchronize()
    assert mfa.lib.mfa_release_scratch(ctypes_ptr(s.cuda_stream)) >= 1
    assert mfa.lib.mfa_release_scratch(ctypes_ptr(s.cuda_stream)) == 0
    torch.cuda.synchronize()
    plan = mfa.KernelPlan()
    import ctypes
    mfa.check(mfa.lib.mfa_multihead_plan(ctypes.byref(desc), int(mfa.KernelType.forward), None,
                                         ctypes.byref(plan)))
    assert plan.total == plan.count == 1


def ctypes_ptr(x):
    import ctypes
    return ctypes.c_void_p(x)
