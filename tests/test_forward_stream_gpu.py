"""GPU parity of the stream-split causal forward (attention_fwd_stream.hip).

The kernel cuts the causal (query block, key tile) work of all heads into W equal ranges; a
block cut between ranges is merged from partial states handed between workgroups.  Small
shapes with a forced range count (MFA_FWD_STREAM_WGS) put every hand-off case on the GPU:
blocks cut into 2 and into 3+ parts, closers that merge from registers and (with
MFA_FWD_STREAM_SLOW=1) closers that publish so that whichever part counts in last merges from
the workspace, ranges that start with a published part and end with a closing one, odd block
counts, partial blocks, R != C, GQA, D below the padded width.

Checked against the CPU oracle at the reference's mixed tolerances (O 5e-3 fp16 / 1e-2 bf16
abs on unit gaussians, L 7e-3 + half an fp16 ulp; SquareAttentionTest.swift:557-571), and
bit for bit between the register merge and the workspace merge, and between two runs.
"""
import os

import numpy as np
import pytest
import torch

import mfa_amd as mfa
from harness import maxerr, run_forward
from test_forward_v2_gpu import check, gaussian

pytestmark = pytest.mark.gpu
FP16, BF16 = mfa.Precision.FP16, mfa.Precision.BF16


class env:
    def __init__(self, **kv):
        self.kv = {k: str(v) for k, v in kv.items()}

    def __enter__(self):
        self.old = {k: os.environ.get(k) for k in self.kv}
        os.environ.update(self.kv)

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def launched():
    return [r["name"] for r in mfa.last_launches()]


CASES = [
    # B, H, Hkv, R, C, D, W (ranges)
    (1, 2, 2, 1024, 1024, 128, 3),    # ranges [closer] / [publisher, ..., closer] / [publisher, ...]
    (1, 2, 2, 1024, 1024, 128, 13),   # 7-tile ranges: the heaviest block in 3 parts
    (1, 2, 2, 1024, 1024, 64, 7),
    (2, 4, 2, 768, 768, 128, 10),     # odd block count (middle block), GQA, B = 2
    (1, 3, 3, 300, 300, 128, 4),      # a partial last block
    (1, 2, 2, 600, 1000, 128, 5),     # R < C: rows see keys up to their index only
    (1, 2, 2, 1000, 600, 64, 6),      # R > C: the last blocks see every key
    (1, 2, 2, 520, 520, 72, 5),       # D < DP
    (1, 16, 16, 1024, 1024, 128, 64),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("prec", [FP16, BF16])
def test_stream_vs_oracle(gpu, case, prec):
    B, H, Hkv, R, C, D, W = case
    seed = R + 3 * C + D + W
    Q = gaussian((B, H, R, D), seed)
    K, V = gaussian((B, Hkv, C, D), seed + 1), gaussian((B, Hkv, C, D), seed + 2)
    with env(MFA_FWD_STREAM=1, MFA_FWD_STREAM_WGS=W):
        mfa.last_launches()
        o, l = check(Q, K, V, prec, causal=True)
        names = launched()
        assert names and names[-1].startswith("mfa_fwd2_stream_kernel"), names
        # The workspace merge (closers publish, the last to count in merges) gives the same bits.
        with env(MFA_FWD_STREAM_SLOW=1):
            o2, l2 = run_forward(Q, K, V, prec=prec, causal=True)
        assert torch.equal(o, o2) and torch.equal(l, l2)
        o3, l3 = run_forward(Q, K, V, prec=prec, causal=True)
        assert torch.equal(o, o3) and torch.equal(l, l3)


@pytest.mark.parametrize("prec", [FP16, BF16])
def test_stream_matches_pair_kernel(gpu, prec):
    # The default range count on a shape the default heuristic gives the stream kernel, against
    # the mirrored shared-tile kernel on the same inputs (different merge order: tolerance).
    B, H, S, D = 1, 16, 2048, 128
    Q, K, V = (gaussian((B, H, S, D), 40 + i) for i in range(3))
    with env(MFA_FWD_STREAM=1):
        o1, l1 = run_forward(Q, K, V, prec=prec, causal=True)
    with env(MFA_FWD_STREAM=0):
        o0, l0 = run_forward(Q, K, V, prec=prec, causal=True)
    assert maxerr(o1, o0) <= (2e-3 if prec == FP16 else 8e-3)
    assert maxerr(l1.float(), l0.float()) <= 1.6e-2


def test_stream_default_route(gpu):
    # A causal shape past the mirrored kernel's range takes the stream kernel by default; the
    # plan says so and the launch log agrees.
    B, H, S, D = 4, 16, 4096, 128
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    plan = [p["name"] for p in mfa.multihead_plan(desc)]
    q = torch.zeros((B, H, S, D), dtype=torch.float16, device="cuda:0")
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    l = torch.empty((B, H, S), dtype=torch.float16, device="cuda:0")
    mfa.last_launches()
    mfa.MultiHeadAttention().forward(desc, q, q, q, o, l)
    torch.cuda.synchronize()
    assert launched() == plan and plan[0].startswith("mfa_fwd2_stream_kernel"), (plan, launched())
    # All-zero inputs: every row averages V = 0 uniformly, L = log2(row + 1).
    assert torch.count_nonzero(o).item() == 0
    ref = torch.log2(torch.arange(1, S + 1, dtype=torch.float64, device="cuda:0"))
    assert (l.double() - ref).abs().max().item() <= 1.6e-2


@pytest.mark.parametrize("prec", [FP16, BF16])
def test_stream_large_causal_heads(gpu, prec):
    # B4 H16 S4096 D128 causal (default stream route) against a float64 restatement at a few
    # (batch, head) slices.
    B, H, S, D = 4, 16, 4096, 128
    g = torch.Generator(device="cuda:0").manual_seed(11)
    dt = torch.float16 if prec == FP16 else torch.bfloat16
    q, k, v = ((torch.rand((B, H, S, D), generator=g, device="cuda:0") * 2 - 1).to(dt)
               for _ in range(3))
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=prec, causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
    o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
    l = torch.empty((B, H, S), dtype=torch.float16, device="cuda:0")
    mfa.last_launches()
    mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
    torch.cuda.synchronize()
    assert launched()[-1].startswith("mfa_fwd2_stream_kernel")
    for bb, hh in ((0, 0), (1, 7), (3, 15)):
        Qd, Kd, Vd = (t[bb, hh].double() for t in (q, k, v))
        s = (Qd @ Kd.T) / np.sqrt(D)
        s = s + torch.triu(torch.full_like(s, float("-inf")), diagonal=1)
        m = s.max(dim=1, keepdim=True).values
        p = torch.exp(s - m)
        ref_o = (p @ Vd) / p.sum(dim=1, keepdim=True)
        ref_l = (m.squeeze(1) + torch.log(p.sum(dim=1))) / np.log(2)
        assert (o[bb, hh].double() - ref_o).abs().max().item() <= (5e-3 if prec == FP16 else 1e-2)
        assert (l[bb, hh].double() - ref_l).abs().max().item() <= 7e-3 + 4e-3


def _torch_ref_check(q, k, v, o, l, slices, tol_o):
    D = q.shape[-1]
    for bb, hh in slices:
        Qd, Kd, Vd = (t[bb, hh].double() for t in (q, k, v))
        s = (Qd @ Kd.T) / np.sqrt(D)
        s = s + torch.triu(torch.full_like(s, float("-inf")), diagonal=1)
        m = s.max(dim=1, keepdim=True).values
        p = torch.exp(s - m)
        ref_o = (p @ Vd) / p.sum(dim=1, keepdim=True)
        ref_l = (m.squeeze(1) + torch.log(p.sum(dim=1))) / np.log(2)
        assert (o[bb, hh].double() - ref_o).abs().max().item() <= tol_o
        assert (l[bb, hh].double() - ref_l).abs().max().item() <= 7e-3 + 4e-3


def test_stream_workspace_counter_region_grows(gpu):
    # the stream kernel's arrival counters sit at the front of the library
    # workspace and its partial states right behind them.  A second call on the same stream
    # whose counter region is longer than the first's (D128 B4 -> D64 B8 at H16 S4096) must not
    # read the first call's partial states as counters: both results against a float64
    # restatement, and the second call repeated bit for bit.
    g = torch.Generator(device="cuda:0").manual_seed(5)
    outs = []
    for B, D in ((4, 128), (8, 64)):
        H, S = 16, 4096
        q, k, v = ((torch.rand((B, H, S, D), generator=g, device="cuda:0") * 2 - 1).half()
                   for _ in range(3))
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, causal=True)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        o = torch.full((B, H, S, D), float("nan"), dtype=torch.float32, device="cuda:0")
        l = torch.full((B, H, S), float("nan"), dtype=torch.float16, device="cuda:0")
        mfa.last_launches()
        mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
        torch.cuda.synchronize()
        assert launched()[-1].startswith("mfa_fwd2_stream_kernel"), launched()
        assert not torch.isnan(o).any() and not torch.isnan(l).any()
        _torch_ref_check(q, k, v, o, l, ((0, 0), (B // 2, 7), (B - 1, 15)), 5e-3)
        outs.append((desc, q, k, v, o.clone(), l.clone()))
    desc, q, k, v, o1, l1 = outs[1]
    o = torch.empty_like(o1)
    l = torch.empty_like(l1)
    mfa.MultiHeadAttention().forward(desc, q, k, v, o, l)
    torch.cuda.synchronize()
    assert torch.equal(o, o1) and torch.equal(l, l1)


def test_stream_workspace_zeroing_under_graph_capture(gpu):
    # a call captured into a HIP graph only records its workspace memset.  An eager
    # call on the same stream between the capture and the replay must still zero the counter
    # region, which the eager call before the capture (a shorter counter prefix) filled with
    # partial states.  Order: eager long-prefix (B8 D64), eager short-prefix (B4 D128, leaves
    # partial states behind its 4 KiB of counters), capture the long-prefix call, then the
    # long-prefix call eagerly, the graph replayed, and the eager call again: every result equal
    # to the first one bit for bit.
    H, S = 16, 4096
    g = torch.Generator(device="cuda:0").manual_seed(9)
    st = torch.cuda.Stream()
    mha = mfa.MultiHeadAttention()

    def problem(B, D):
        q, k, v = ((torch.rand((B, H, S, D), generator=g, device="cuda:0") * 2 - 1).half()
                   for _ in range(3))
        base = mfa.AttentionDescriptor.make(low_precision=True, precision=FP16, causal=True)
        desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)
        o = torch.empty((B, H, S, D), dtype=torch.float32, device="cuda:0")
        l = torch.empty((B, H, S), dtype=torch.float16, device="cuda:0")
        return desc, q, k, v, o, l

    long_p, short_p = problem(8, 64), problem(4, 128)
    torch.cuda.synchronize()

    def run(pr):
        desc, q, k, v, o, l = pr
        mha.forward(desc, q, k, v, o, l, stream=st.cuda_stream)

    with torch.cuda.stream(st):
        mfa.last_launches()
        run(long_p)
        st.synchronize()
        assert launched()[-1].startswith("mfa_fwd2_stream_kernel"), launched()
        ref_o, ref_l = long_p[4].clone(), long_p[5].clone()
        _torch_ref_check(*long_p[1:4], ref_o, ref_l, ((0, 0), (7, 15)), 5e-3)
        run(short_p)
        st.synchronize()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph, stream=st):
            run(long_p)
        for phase in ("eager", "replay", "eager again"):
            long_p[4].fill_(float("nan"))
            if phase == "replay":
                graph.replay()
            else:
                run(long_p)
            st.synchronize()
            assert torch.equal(long_p[4], ref_o) and torch.equal(long_p[5], ref_l), phase
