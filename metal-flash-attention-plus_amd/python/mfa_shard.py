"""Batch x head sharding of the attention hot path across GPUs (one process per GPU).

SURVEY.md §8(e): attention is independent per (batch, head) slice, so the units of work are
split into contiguous per-rank ranges and each rank runs the ordinary single-GPU kernels on its
slices — no collective on the data path (the reference has no multi-device path at all; its
batching is MultiHeadAttention.swift:33-83's 3-D grid over (row block, head, batch)).

Units:
  * forward: (b, head block) where a head block is H_kv consecutive query heads
    [j·H_kv, (j+1)·H_kv).  With the reference's GQA mapping kv = h % H_kv
    (AttentionKernel+Source.swift:96-117) every block reads all H_kv key/value heads in
    order, so a contiguous run of blocks is a dense [B', H', S, D] view of Q/O/L with the same
    K/V — one launch per batch segment.  MHA (H_kv == H) splits by single heads: a head range
    [h0, h1) reads the kv heads [h0, h1), so K/V are sliced with it (strong scaling of one
    batch element over heads, SURVEY.md §8e's C2/C3/C4 plan).
  * backward: dK/dV are sums over a kv group's query heads, which must stay on one rank:
    MHA (H_kv == H) shards by (b, h); GQA/MQA shards by whole batch elements.
"""
from __future__ import annotations

from typing import List, Tuple


def split_range(n: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced split of range(n): the first n % world ranks get one extra unit."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def forward_slices(B: int, H: int, Hkv: int, world: int, rank: int) -> List[Tuple[int, int, int]]:
    """This rank's forward work as (b, h0, h1) query-head ranges, one per batch segment."""
    if H % Hkv:
        raise ValueError("H must be a multiple of H_kv")
    unit = 1 if Hkv == H else Hkv  # heads per unit
    blocks = H // unit
    u0, u1 = split_range(B * blocks, world, rank)
    out = []
    u = u0
    while u < u1:
        b, j = divmod(u, blocks)
        j1 = min(blocks, j + (u1 - u))
        out.append((b, j * unit, j1 * unit))
        u += j1 - j
    return out


def backward_slices(B: int, H: int, Hkv: int, world: int, rank: int) -> List[Tuple[int, int, int]]:
    """This rank's backward work as (b, h0, h1) ranges; kv groups never straddle ranks."""
    if H % Hkv:
        raise ValueError("H must be a multiple of H_kv")
    if Hkv == H:
        return forward_slices(B, H, H, world, rank)
    b0, b1 = split_range(B, world, rank)
    return [(b, 0, H) for b in range(b0, b1)]


def forward_shard(mfa, base, q, k, v, o, l, world: int, rank: int, stream=None) -> int:
    """Runs this rank's forward slices through the C ABI on [B, H, S, D] device tensors (K/V
    [B, H_kv, S_kv, D]).  Returns the number of (b, h) slices processed."""
    B, H, R, D = q.shape
    Hkv, C = k.shape[1], k.shape[2]
    mha = mfa.MultiHeadAttention()
    n = 0
    for b, h0, h1 in forward_slices(B, H, Hkv, world, rank):
        hk0, hk1 = (h0, h1) if Hkv == H else (0, Hkv)
        desc = mfa.MultiHeadDescriptor.make(base, 1, h1 - h0, R, D, Hkv=hk1 - hk0, C=C)
        mha.forward(desc, q[b:b + 1, h0:h1], k[b:b + 1, hk0:hk1], v[b:b + 1, hk0:hk1],
                    o[b:b + 1, h0:h1], None if l is None else l[b:b + 1, h0:h1], stream=stream)
        n += h1 - h0
    return n


def backward_shard(mfa, base, q, k, v, o, do, l, dq, dk, dv, dbuf, world: int, rank: int,
                   stream=None) -> int:
    """Runs this rank's backward slices (backward_slices) through the C ABI: backwardQuery then
    backwardKeyValue per slice, as mfa_multihead_backward does for the whole batch.  Tensors
    are the full [B, H, S, D] / [B, H_kv, S_kv, D] device arrays (forward outputs O, L
    included); each rank writes dQ and D for its query heads and dK / dV for the kv heads it
    owns.  MHA slices are (b, head range); GQA / MQA slices are whole batch elements, so a kv
    group's dK / dV sum never crosses ranks and needs no collective.  Returns the number of
    (b, h) query-head slices processed."""
    B, H, R, D = q.shape
    Hkv, C = k.shape[1], k.shape[2]
    mha = mfa.MultiHeadAttention()
    n = 0
    for b, h0, h1 in backward_slices(B, H, Hkv, world, rank):
        hk0, hk1 = (h0, h1) if Hkv == H else (0, Hkv)
        desc = mfa.MultiHeadDescriptor.make(base, 1, h1 - h0, R, D, Hkv=hk1 - hk0, C=C)
        qs = (slice(b, b + 1), slice(h0, h1))
        ks = (slice(b, b + 1), slice(hk0, hk1))
        mha.backward(desc, q[qs], k[ks], v[ks], o[qs], do[qs], l[qs], dq[qs], dk[ks], dv[ks],
                     dbuf[qs], stream=stream)
        n += h1 - h0
    return n
