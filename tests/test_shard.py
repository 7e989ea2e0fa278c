"""Multi-GPU sharding (mfa_shard.py): plan properties and a world_size-2 gloo run on CPU.

Each rank computes its slices with the CPU oracle (standing in for the per-GPU kernels, which
the GPU test test_shard_gpu.py drives through the C ABI); rank 0 gathers the pieces and checks
them against the unsharded result.  Same barrier + max-over-ranks timing as bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import mfa_shard as sh
import oracle_lib as ol


@pytest.mark.parametrize("B,H,Hkv", [(1, 16, 16), (3, 8, 2), (2, 32, 1), (5, 4, 4), (1, 2, 2)])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_forward_slices_cover_every_head_once(B, H, Hkv, world):
    seen = np.zeros((B, H), dtype=int)
    sizes = []
    for r in range(world):
        n = 0
        for b, h0, h1 in sh.forward_slices(B, H, Hkv, world, r):
            # kv = h % Hkv preserved: MHA slices K/V with the heads, GQA keeps whole blocks
            assert Hkv == H or (h0 % Hkv == 0 and h1 % Hkv == 0)
            assert h0 < h1
            seen[b, h0:h1] += 1
            n += h1 - h0
        sizes.append(n)
    assert (seen == 1).all()
    unit = 1 if Hkv == H else Hkv
    assert max(sizes) - min(sizes) <= unit  # balanced to one unit


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8, 16])
def test_head_split_of_one_batch_element(world):
    # SURVEY §8e strong-scaling plan: C2 / C3 / C4 (B = 1, H = 16) split over N ranks by heads;
    # each rank gets ceil or floor of 16 / N heads and the union covers every head once.
    got = [sh.forward_slices(1, 16, 16, world, r) for r in range(world)]
    counts = [sum(h1 - h0 for _, h0, h1 in g) for g in got]
    assert sorted(set(counts)) in ([16 // world], [16 // world, -(-16 // world)])
    heads = sorted(h for g in got for _, h0, h1 in g for h in range(h0, h1))
    assert heads == list(range(16))


@pytest.mark.parametrize("B,H,Hkv,world", [(2, 8, 8, 3), (3, 8, 2, 2), (4, 4, 1, 4)])
def test_backward_slices_keep_kv_groups_local(B, H, Hkv, world):
    owner = -np.ones((B, H), dtype=int)
    for r in range(world):
        for b, h0, h1 in sh.backward_slices(B, H, Hkv, world, r):
            assert (owner[b, h0:h1] == -1).all()
            owner[b, h0:h1] = r
    assert (owner >= 0).all()
    for b in range(B):
        for g in range(Hkv):
            assert len(set(owner[b, g::Hkv])) == 1  # every query head of a kv group together


def test_split_range_rejects_bad_rank():
    with pytest.raises(ValueError):
        sh.split_range(4, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, B, H, Hkv, S, D, q):
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(7)
    Q = rng.standard_normal((B, H, S, D)).astype(np.float32)
    K = rng.standard_normal((B, Hkv, S, D)).astype(np.float32)
    V = rng.standard_normal((B, Hkv, S, D)).astype(np.float32)
    dist.barrier()
    pieces = []
    for b, h0, h1 in sh.forward_slices(B, H, Hkv, world, rank):
        hk0, hk1 = (h0, h1) if Hkv == H else (0, Hkv)
        r = ol.attention(Q[b:b + 1, h0:h1], K[b:b + 1, hk0:hk1], V[b:b + 1, hk0:hk1], causal=True)
        pieces.append((b, h0, h1, r["O"], r["L"]))
    dist.barrier()
    t = torch.tensor([1.0 + rank])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py's max-over-ranks timing
    gathered = [None] * world
    dist.all_gather_object(gathered, pieces)
    if rank == 0:
        O = np.full((B, H, S, D), np.nan, dtype=np.float32)
        L = np.full((B, H, S), np.nan, dtype=np.float32)
        for plist in gathered:
            for b, h0, h1, o, l in plist:
                O[b, h0:h1], L[b, h0:h1] = o[0], l[0]
        full = ol.attention(Q, K, V, causal=True)
        q.put((bool(np.array_equal(O, full["O"]) and np.array_equal(L, full["L"])),
               float(t.item())))
    dist.destroy_process_group()


@pytest.mark.parametrize("B,H,Hkv", [(2, 4, 4), (3, 4, 2), (1, 4, 4)])
def test_gloo_world2_sharded_forward_equals_unsharded(B, H, Hkv):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, B, H, Hkv, 40, 16, q))
             for r in range(2)]
    for p in procs:
        p.start()
    ok, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok and tmax == 2.0


def _bwd_worker(rank, world, port, B, H, Hkv, S, D, q):
    """Each rank runs the oracle backward on its backward_slices (standing in for the per-GPU
    kernels test_shard_gpu.py drives); rank 0 assembles dQ / dK / dV and checks them against
    the unsharded backward: kv groups never straddle ranks, so no reduction is needed."""
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank,
                            world_size=world)
    rng = np.random.default_rng(11)
    Q, dO = (rng.standard_normal((B, H, S, D)).astype(np.float32) for _ in range(2))
    K, V = (rng.standard_normal((B, Hkv, S, D)).astype(np.float32) for _ in range(2))
    pieces = []
    for b, h0, h1 in sh.backward_slices(B, H, Hkv, world, rank):
        hk0, hk1 = (h0, h1) if Hkv == H else (0, Hkv)
        r = ol.attention(Q[b:b + 1, h0:h1], K[b:b + 1, hk0:hk1], V[b:b + 1, hk0:hk1],
                         causal=True, dO=dO[b:b + 1, h0:h1])
        pieces.append((b, h0, h1, hk0, hk1, r["dQ"], r["dK"], r["dV"], r["D"]))
    gathered = [None] * world
    dist.all_gather_object(gathered, pieces)
    if rank == 0:
        dQ = np.full((B, H, S, D), np.nan, dtype=np.float32)
        dK = np.full((B, Hkv, S, D), np.nan, dtype=np.float32)
        dV = np.full_like(dK, np.nan)
        Dt = np.full((B, H, S), np.nan, dtype=np.float32)
        for plist in gathered:
            for b, h0, h1, hk0, hk1, gq, gk, gv, gd in plist:
                dQ[b, h0:h1], Dt[b, h0:h1] = gq[0], gd[0]
                dK[b, hk0:hk1], dV[b, hk0:hk1] = gk[0], gv[0]
        full = ol.attention(Q, K, V, causal=True, dO=dO)
        q.put(all(np.array_equal(x, full[n]) for x, n in
                  ((dQ, "dQ"), (dK, "dK"), (dV, "dV"), (Dt, "D"))))
    dist.destroy_process_group()


@pytest.mark.parametrize("B,H,Hkv", [(2, 4, 4), (3, 4, 2), (2, 4, 1)])
def test_gloo_world2_sharded_backward_equals_unsharded(B, H, Hkv):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bwd_worker, args=(r, 2, port, B, H, Hkv, 40, 16, q))
             for r in range(2)]
    for p in procs:
        p.start()
    ok = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok
