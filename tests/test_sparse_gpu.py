"""GPU parity for sparse key ranges on the tuned 16-bit forward (attention_fwd_v2.hip).

The HAS_SPARSE_RANGES mask (AttentionKernel+Softmax.swift:278-304) gives every query row a
half-open key range [x, y), indexed (b*H_kv + kv)*R + row; SparseMQABuilder.buildBlockSparse
(SparseMQABuilder.swift:30-62) turns a block pattern into such ranges.  The tuned kernel skips
the key tiles outside the union of a query block's ranges; rows left with no unmasked key get
the reference's finite-mask result (uniform average of V, L = mask*c + log2 C), written by the
owning wave after the tile loop.  Tolerances: SquareAttentionTest.swift:557-571 (mixed O 5e-2); L here is kept in fp32
(lowPrecisionIntermediates off) so the fully masked rows' L stays finite.
"""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol
from harness import maxerr, run_forward, seen

pytestmark = pytest.mark.gpu
FP16, BF16 = mfa.Precision.FP16, mfa.Precision.BF16


def gaussian(shape, seed):
    return np.random.default_rng(seed).standard_normal(shape).astype(np.float32)


def block_ranges(pattern, block, R, C):
    """Per-row ranges from a [R/block, C/block] pattern through the library's builder."""
    nqb, nkb = pattern.shape
    rb = np.zeros((nqb, 2), dtype=np.uint32)
    mfa.lib.mfa_sparse_build_block_sparse(np.ascontiguousarray(pattern, dtype=np.uint8).ctypes.data,
                                          nqb, nkb, block, rb.ctypes.data)
    rows = np.repeat(rb, block, axis=0)[:R]
    rows[:, 1] = np.minimum(rows[:, 1], C)
    return rows


def banded_pattern(nqb, nkb, width, seed, empty_every=0):
    rng = np.random.default_rng(seed)
    pat = np.zeros((nqb, nkb), dtype=np.uint8)
    for i in range(nqb):
        c = min(nkb - 1, i * nkb // nqb + int(rng.integers(-1, 2)))
        pat[i, max(0, c - width // 2):min(nkb, c + width // 2 + 1)] = 1
        if empty_every and i % empty_every == empty_every - 1:
            pat[i] = 0
    return pat


def check(Q, K, V, prec, ranges, causal=False, window=None):
    mfa.last_launches()  # drop what earlier tests launched on this thread
    o, l = run_forward(Q, K, V, prec=prec, causal=causal, window=window, ranges=ranges,
                       low_precision_intermediates=False)
    plan = [x["name"] for x in mfa.last_launches()]
    ref = ol.attention(seen(Q, prec), seen(K, prec), seen(V, prec), causal=causal, window=window,
                       ranges=ranges)
    on, ln = o.cpu().numpy(), l.float().cpu().numpy()
    assert np.isfinite(on).all()
    assert maxerr(on, ref["O"]) <= 5e-2
    # Rows with a key keep L ~ O(10); fully masked rows carry L = fp32(mask * c) + log2 C.
    big = np.abs(ref["L"]) > 1e6
    assert maxerr(ln[~big], ref["L"][~big]) <= 1e-2
    if big.any():
        assert np.allclose(ln[big], ref["L"][big], rtol=1e-6, atol=0)
    return plan


@pytest.mark.parametrize("prec", [FP16, BF16])
@pytest.mark.parametrize("D", [64, 128])
def test_block_sparse_tuned_kernel(gpu, prec, D):
    B, H, Hkv, S, blk = 1, 4, 2, 1000, 64
    nb = (S + blk - 1) // blk
    ranges = np.stack([block_ranges(banded_pattern(nb, nb, 3, 900 + kv), blk, S, S)
                       for kv in range(Hkv)])[None]
    Q = gaussian((B, H, S, D), 901)
    K, V = gaussian((B, Hkv, S, D), 902), gaussian((B, Hkv, S, D), 903)
    plan = check(Q, K, V, prec, ranges)
    assert len(plan) == 1 and "mfa_fwd2_kernel" in plan[0], plan  # empty rows in-kernel


@pytest.mark.parametrize("causal,window", [(True, None), (False, 90), (False, 300)])
def test_block_sparse_with_empty_rows_and_masks(gpu, causal, window):
    """Empty block rows, and rows whose range the causal / window predicates empty, take the
    finite-mask uniform average; the union skip must not drop keys other rows need."""
    B, H, Hkv, R, C, D, blk = 2, 2, 1, 700, 700, 128, 64
    nb = (R + blk - 1) // blk
    ranges = np.stack([block_ranges(banded_pattern(nb, nb, 5, 910 + b, empty_every=4), blk, R, C)
                       for b in range(B)])[:, None]
    # Ragged per-row ranges inside a block: some rows empty, some narrowed.
    ranges[0, 0, 5::11, 1] = ranges[0, 0, 5::11, 0]
    ranges[1, 0, 3::13, 0] = np.minimum(ranges[1, 0, 3::13, 0] + 17, ranges[1, 0, 3::13, 1])
    Q = gaussian((B, H, R, D), 911)
    K, V = gaussian((B, Hkv, C, D), 912), gaussian((B, Hkv, C, D), 913)
    check(Q, K, V, FP16, ranges, causal=causal, window=window)


def test_ranges_beyond_sequence(gpu):
    """Ranges reaching past C (the reference clamps at the key bound) and x >= y rows."""
    B, H, R, C, D = 1, 2, 300, 257, 64
    lo = np.random.default_rng(920).integers(0, C + 40, (B, H, R))
    hi = lo + np.random.default_rng(921).integers(-5, 200, (B, H, R))
    ranges = np.stack([lo, np.maximum(hi, 0)], -1).astype(np.uint32)
    Q = gaussian((B, H, R, D), 922)
    K, V = gaussian((B, H, C, D), 923), gaussian((B, H, C, D), 924)
    check(Q, K, V, BF16, ranges)


@pytest.mark.parametrize("D", [64, 128])
def test_mostly_empty_rows(gpu, D):
    """a pattern whose rows are mostly empty (every block row but one per four has
    no keys, and single rows emptied in the live ones) over a long key range: the empty rows of
    a wave share one mean of V, summed once per wave."""
    B, H, Hkv, R, C, blk = 1, 2, 2, 512, 2048, 64
    nqb, nkb = R // blk, C // blk
    pat = np.zeros((nqb, nkb), dtype=np.uint8)
    pat[::4, : nkb // 2] = 1
    ranges = np.stack([block_ranges(pat, blk, R, C) for _ in range(Hkv)])[None]
    ranges[0, 0, 7::9, 1] = ranges[0, 0, 7::9, 0]
    assert (ranges[..., 0] >= ranges[..., 1]).mean() > 0.7
    Q = gaussian((B, H, R, D), 930)
    K, V = gaussian((B, Hkv, C, D), 931), gaussian((B, Hkv, C, D), 932)
    plan = check(Q, K, V, FP16, ranges)
    assert len(plan) == 1 and "mfa_fwd2_kernel" in plan[0], plan


# --------------------------------------------------------------- ranges on the shared tiles
# Adjacent pairs of 128-row blocks share every staged tile (attention_fwd_v2.hip, the
# shared-tile kernel): with ranges the pair stages the union of its blocks' key ranges and each
# group computes and masks only its own.  MFA_FWD_SHARE=1 takes that kernel at any size.
@pytest.mark.parametrize("prec", [FP16, BF16])
@pytest.mark.parametrize("D", [64, 128])
def test_block_sparse_shared_tiles(gpu, prec, D, monkeypatch):
    monkeypatch.setenv("MFA_FWD_SHARE", "1")
    B, H, Hkv, S, blk = 1, 4, 2, 1000, 64
    nb = (S + blk - 1) // blk
    ranges = np.stack([block_ranges(banded_pattern(nb, nb, 3, 940 + kv, empty_every=5), blk, S, S)
                       for kv in range(Hkv)])[None]
    Q = gaussian((B, H, S, D), 941)
    K, V = gaussian((B, Hkv, S, D), 942), gaussian((B, Hkv, S, D), 943)
    plan = check(Q, K, V, prec, ranges)
    assert len(plan) == 1 and plan[0].startswith("mfa_fwd2_share_kernel") and ", false" in plan[0], plan


def test_block_sparse_shared_disjoint_blocks(gpu, monkeypatch):
    """The two blocks of a pair keep disjoint key ranges (the first block the first 300 keys, the
    second the last 300), with empty and narrowed single rows and an odd block count: each group
    must compute only its own tiles of the staged union."""
    monkeypatch.setenv("MFA_FWD_SHARE", "1")
    B, H, R, C, D = 2, 2, 5 * 128 + 40, 1100, 128
    ranges = np.zeros((B, H, R, 2), dtype=np.uint32)
    blk = np.arange(R) // 128
    ranges[..., 0] = np.where(blk % 2 == 0, 0, C - 300)[None, None]
    ranges[..., 1] = np.where(blk % 2 == 0, 300, C)[None, None]
    ranges[0, 0, 7::23, 1] = ranges[0, 0, 7::23, 0]            # empty rows
    ranges[1, 1, 11::17, 0] = ranges[1, 1, 11::17, 0] + 90      # narrowed rows
    Q = gaussian((B, H, R, D), 951)
    K, V = gaussian((B, H, C, D), 952), gaussian((B, H, C, D), 953)
    plan = check(Q, K, V, FP16, ranges)
    assert plan[0].startswith("mfa_fwd2_share_kernel"), plan


def test_mostly_empty_rows_shared_tiles(gpu, monkeypatch):
    monkeypatch.setenv("MFA_FWD_SHARE", "1")
    B, H, Hkv, R, C, blk = 1, 2, 2, 512, 2048, 64
    nqb, nkb = R // blk, C // blk
    pat = np.zeros((nqb, nkb), dtype=np.uint8)
    pat[::4, : nkb // 2] = 1
    ranges = np.stack([block_ranges(pat, blk, R, C) for _ in range(Hkv)])[None]
    Q = gaussian((B, H, R, 128), 960)
    K, V = gaussian((B, Hkv, C, 128), 961), gaussian((B, Hkv, C, 128), 962)
    plan = check(Q, K, V, BF16, ranges)
    assert plan[0].startswith("mfa_fwd2_share_kernel"), plan


def test_block_sparse_bench_shape_routes_shared(gpu):
    """The bench's block-sparse row (B1 H16 S4096 D128, band of 8 of 32 key blocks) takes the
    shared-tile kernel by default; heads 0 and 15 against the oracle."""
    B, H, S, D, blk = 1, 16, 4096, 128, 128
    nb = S // blk
    pat = np.zeros((nb, nb), dtype=np.uint8)
    for i in range(nb):
        lo = min(max(0, i - 4), nb - 8)
        pat[i, lo:lo + 8] = 1
    ranges = np.stack([block_ranges(pat, blk, S, S) for _ in range(H)])[None]
    g = np.random.default_rng(970)
    Q, K, V = (g.standard_normal((B, H, S, D)).astype(np.float32) for _ in range(3))
    mfa.last_launches()
    o, l = run_forward(Q, K, V, prec=FP16, ranges=ranges, low_precision_intermediates=False)
    plan = [x["name"] for x in mfa.last_launches()]
    assert plan[0].startswith("mfa_fwd2_share_kernel") and ", false" in plan[0], plan
    for hh in (0, 15):
        sub = lambda x: np.ascontiguousarray(x[:, hh:hh + 1])
        ref = ol.attention(seen(sub(Q), FP16), seen(sub(K), FP16), seen(sub(V), FP16),
                           ranges=np.ascontiguousarray(ranges[:, hh:hh + 1]))
        assert maxerr(o[:, hh:hh + 1].cpu().numpy(), ref["O"]) <= 5e-3
