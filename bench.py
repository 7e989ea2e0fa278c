#!/usr/bin/env python3
"""Headline benchmark: attention TFLOPS/GPU (fwd, seq=4096, d=128), fp16 vs INT8.

Workload (BASELINE.json configs[1]): fp16 forward, B=1 per GPU, H=16, S=4096, D=128, causal,
O fp32 (the reference's output layout).  One step = one forward pass over the batch through
the C ABI (mfa_multihead_forward).  Multi-GPU: one process per GPU, batch x head sharded
with no collective on the data path; each rank runs its own batch element (weak scaling).
FLOPs are algorithmic: 4·D per unmasked (query, key) pair.

Also reported (same JSON line): the INT8-K/V path and the fp16 path at configs[2]'s shape
(H16 S8192 D128, non-causal) and their ratio; the kernel's MFMA roofline fraction measured
live with HIP events on the launch stream; the CPU oracle timed on a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

_REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(_REPO, "metal-flash-attention-plus_amd", "python"))

# gfx950 dense fp16/bf16 MFMA peak: 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz
# (MI355X_MICROARCH.md: v_mfma_f32_32x32x16_f16 = 32768 FLOP per 32 cycles per SIMD).
PEAK_FP16_TFLOPS = 256 * 4 * 1024 * 2.4e9 / 1e12  # 2516.6
PEAK_INT8_TOPS = 2 * PEAK_FP16_TFLOPS


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--heads", type=int, default=16)
    ap.add_argument("--seq", type=int, default=4096)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--no-int8", action="store_true")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-c5", action="store_true")
    ap.add_argument("--no-mla", action="store_true")
    ap.add_argument("--no-sparse", action="store_true", help="skip the block-sparse row")
    ap.add_argument("--no-next", action="store_true", help="skip the SURVEY §8(f) rows")
    ap.add_argument("--c5-batch", type=int, default=8)
    ap.add_argument("--no-strong", action="store_true",
                    help="skip the heads-split (strong-scaling) C2 row")
    ap.add_argument("--fake-device", action="store_true",
                    help="CPU dry run of the launch / rank / timing plumbing (gloo, no GPU, "
                         "no kernels); used by the CPU test of the --gpus spawn path")
    return ap.parse_args()


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` started without a launcher: run N rank processes under
    torch.distributed.run (one per GPU, 127.0.0.1 rendezvous) and return their exit code.
    The parent imports nothing that touches the GPU."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if args.fake_device:
        return fake_device_run(args, world, rank)
    import torch
    import mfa_amd as mfa

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x: float) -> float:
        if dist is None:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def warm(fn, seconds=0.2):
        """Time-based warm-up: repeat fn until `seconds` of back-to-back launches have run
        (the clock settles over ~0.1 s from a cold chip), at least twice."""
        fn()
        torch.cuda.synchronize()
        t, n = time.perf_counter(), 0
        while n < 2 or time.perf_counter() - t < seconds:
            fn()
            n += 1
            if n % 8 == 0 or n < 4:
                torch.cuda.synchronize()
        torch.cuda.synchronize()

    def ev_time(fn, steps=20):
        """HIP-event time per call on the current stream after a time-based warm-up;
        at least 20 timed calls whatever --steps says."""
        steps = max(20, steps)
        warm(fn)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    def timed_steps(fn, n):
        """n calls of fn bracketed by barrier + synchronize, timed by HIP events on the
        launch stream; seconds, max over ranks."""
        barrier()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        barrier()
        return max_over_ranks(e0.elapsed_time(e1) * 1e-3)

    import mfa_shard as shard
    H, S, D = args.heads, args.seq, args.dim
    B = 1  # per rank
    # Weak scaling: the global batch is world x B; mfa_shard gives each rank its own batch
    # element(s) (no collective on the data path).  Each rank materialises only its slices.
    my = shard.forward_slices(B * world, H, H, world, rank)
    assert sum(h1 - h0 for _, h0, h1 in my) == B * H
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)

    def uniform(shape, dtype):
        return ((torch.rand(shape, generator=g, device=dev) * 2 - 1) * 0.25).to(dtype)

    result = {}
    mha = mfa.MultiHeadAttention()
    stream = torch.cuda.current_stream(dev).cuda_stream

    # ---------------------------------------------------------------- INT8 vs fp16 at C3
    if not args.no_int8:
        S3 = 8192
        qf = uniform((B, H, S3, D), torch.float16)
        kf = uniform((B, H, S3, D), torch.float32)
        vf = uniform((B, H, S3, D), torch.float32)
        o3 = torch.empty((B, H, S3, D), dtype=torch.float32, device=dev)
        l3 = torch.empty((B, H, S3), dtype=torch.float16, device=dev)
        kq, ks, _, _ = mfa.quantize(kf, mfa.Precision.INT8, rows=B * H * S3, cols=D)
        vq, vs, _, _ = mfa.quantize(vf, mfa.Precision.INT8, rows=B * H * S3, cols=D)
        k4, ks4, _, _ = mfa.quantize(kf, mfa.Precision.INT4, rows=B * H * S3, cols=D)
        v4, vs4, _, _ = mfa.quantize(vf, mfa.Precision.INT4, rows=B * H * S3, cols=D)
        torch.cuda.synchronize()
        base3 = mfa.AttentionDescriptor.make(S3, S3, D, low_precision=True,
                                             precision=mfa.Precision.FP16)
        qdesc = mfa.quantized_descriptor(base3, mfa.Precision.FP16, mfa.Precision.INT8,
                                         mfa.Precision.INT8, B=B, H=H, integer_matmul=True)
        qdesc_exact = mfa.quantized_descriptor(base3, mfa.Precision.FP16, mfa.Precision.INT8,
                                               mfa.Precision.INT8, B=B, H=H)
        qa = mfa.QuantizedAttention()
        tq = mfa.quantized_tensor(qf, mfa.Precision.FP16)
        tk = mfa.quantized_tensor(kq, mfa.Precision.INT8, scale=float(ks.item()))
        tv = mfa.quantized_tensor(vq, mfa.Precision.INT8, scale=float(vs.item()))
        kh, vh = kf.half(), vf.half()
        desc3 = mfa.MultiHeadDescriptor.make(base3, B, H, S3, D)
        qdesc4 = mfa.quantized_descriptor(base3, mfa.Precision.FP16, mfa.Precision.INT4,
                                          mfa.Precision.INT4, B=B, H=H)
        tk4 = mfa.quantized_tensor(k4, mfa.Precision.INT4, scale=float(ks4.item()))
        tv4 = mfa.quantized_tensor(v4, mfa.Precision.INT4, scale=float(vs4.item()))

        ms_i8 = ev_time(lambda: qa.forward(qdesc, tq, tk, tv, o3, l3, stream=stream))
        ms_i8x = ev_time(lambda: qa.forward(qdesc_exact, tq, tk, tv, o3, l3, stream=stream))
        ms_i4 = ev_time(lambda: qa.forward(qdesc4, tq, tk4, tv4, o3, l3, stream=stream))
        ms_f16 = ev_time(lambda: mha.forward(desc3, qf, kh, vh, o3, l3, stream=stream))
        f3 = mfa.attention_flops(B, H, S3, S3, D, causal=False)
        result["int8"] = {
            "workload": "INT8 K/V (per-tensor, zp 0) + fp16 Q, H16 S8192 D128 non-causal "
                        "(BASELINE configs[2])",
            "int8_kernel": mfa.quantized_plan(qdesc, mfa.KernelType.forward, tq, tk, tv)[0]["name"],
            "int8_dequant_exact_kernels": [r["name"] for r in mfa.quantized_plan(
                qdesc_exact, mfa.KernelType.forward, tq, tk, tv)],
            "int8_tops": round(f3 / (ms_i8 * 1e-3) / 1e12, 2),
            "int8_roofline_frac": round(f3 / (ms_i8 * 1e-3) / 1e12 / PEAK_INT8_TOPS, 4),
            "fp16_tflops_same_shape": round(f3 / (ms_f16 * 1e-3) / 1e12, 2),
            "ratio_int8_over_fp16": round(ms_f16 / ms_i8, 3),
            "int8_dequant_exact_tflops": round(f3 / (ms_i8x * 1e-3) / 1e12, 2),
            "int4_dequant_exact_tflops": round(f3 / (ms_i4 * 1e-3) / 1e12, 2),
            "int8_ms": round(ms_i8, 4), "int8_dequant_exact_ms": round(ms_i8x, 4),
            "int4_dequant_exact_ms": round(ms_i4, 4),
            "fp16_ms": round(ms_f16, 4),
        }
        del qf, kf, vf, o3, l3, kq, vq, kh, vh, k4, v4

        # Causal INT8 K/V prefill at the C2 shape (dequant-exact, K/V widened on load in the
        # mirrored shared-tile schedule), against the same forward on fp16 K/V.
        S2 = args.seq
        q2 = uniform((B, H, S2, D), torch.float16)
        k2f = uniform((B, H, S2, D), torch.float32)
        v2f = uniform((B, H, S2, D), torch.float32)
        k2q, k2s, _, _ = mfa.quantize(k2f, mfa.Precision.INT8, rows=B * H * S2, cols=D)
        v2q, v2s, _, _ = mfa.quantize(v2f, mfa.Precision.INT8, rows=B * H * S2, cols=D)
        k2h, v2h = k2f.half(), v2f.half()
        o2c = torch.empty((B, H, S2, D), dtype=torch.float32, device=dev)
        l2c = torch.empty((B, H, S2), dtype=torch.float16, device=dev)
        base2c = mfa.AttentionDescriptor.make(S2, S2, D, causal=True, low_precision=True,
                                              precision=mfa.Precision.FP16)
        qd2c = mfa.quantized_descriptor(base2c, mfa.Precision.FP16, mfa.Precision.INT8,
                                        mfa.Precision.INT8, B=B, H=H)
        tq2 = mfa.quantized_tensor(q2, mfa.Precision.FP16)
        tk2 = mfa.quantized_tensor(k2q, mfa.Precision.INT8, scale=float(k2s.item()))
        tv2 = mfa.quantized_tensor(v2q, mfa.Precision.INT8, scale=float(v2s.item()))
        desc2c = mfa.MultiHeadDescriptor.make(base2c, B, H, S2, D)
        ms_c8 = ev_time(lambda: qa.forward(qd2c, tq2, tk2, tv2, o2c, l2c, stream=stream))
        ms_c16 = ev_time(lambda: mha.forward(desc2c, q2, k2h, v2h, o2c, l2c, stream=stream))
        f2c = mfa.attention_flops(B, H, S2, S2, D, causal=True)
        result["int8_causal"] = {
            "workload": f"QuantizedAttention forward, INT8 K/V (per-tensor) + fp16 Q, B{B} H{H} "
                        f"S{S2} D{D} causal (the C2 shape), dequant-exact",
            "kernels": [r["name"] for r in mfa.quantized_plan(qd2c, mfa.KernelType.forward,
                                                              tq2, tk2, tv2)],
            "int8_tflops": round(f2c / (ms_c8 * 1e-3) / 1e12, 2),
            "fp16_tflops_same_shape": round(f2c / (ms_c16 * 1e-3) / 1e12, 2),
            "int8_ms": round(ms_c8, 4), "fp16_ms": round(ms_c16, 4),
        }
        del q2, k2f, v2f, k2q, v2q, k2h, v2h, o2c, l2c

        # INT8 K/V decode (the KV-cache shape INT8 K/V exists for): B32 H16, 8192 cached keys,
        # 1 and 16 query rows per head; HBM-bound on the INT8 K/V read (2·D bytes per key).
        Bd, Hd, Cd, Dd = 32, 16, 8192, 128
        kd8 = torch.randint(0, 256, (Bd, Hd, Cd, Dd), dtype=torch.uint8, device=dev, generator=g)
        vd8 = torch.randint(0, 256, (Bd, Hd, Cd, Dd), dtype=torch.uint8, device=dev, generator=g)
        tkd = mfa.quantized_tensor(kd8, mfa.Precision.INT8, scale=0.25 / 127)
        tvd = mfa.quantized_tensor(vd8, mfa.Precision.INT8, scale=0.25 / 127)
        dec = {}
        for Rd in (1, 16):
            qd8 = uniform((Bd, Hd, Rd, Dd), torch.float16)
            od8 = torch.empty((Bd, Hd, Rd, Dd), dtype=torch.float32, device=dev)
            ld8 = torch.empty((Bd, Hd, Rd), dtype=torch.float16, device=dev)
            based = mfa.AttentionDescriptor.make(Rd, Cd, Dd, low_precision=True,
                                                 precision=mfa.Precision.FP16)
            qdd = mfa.quantized_descriptor(based, mfa.Precision.FP16, mfa.Precision.INT8,
                                           mfa.Precision.INT8, B=Bd, H=Hd)
            tqd = mfa.quantized_tensor(qd8, mfa.Precision.FP16)
            msd = ev_time(lambda: qa.forward(qdd, tqd, tkd, tvd, od8, ld8, stream=stream))
            kv_bytes = 2 * Bd * Hd * Cd * Dd
            io_bytes = kv_bytes + qd8.numel() * 2 + od8.numel() * 4 + ld8.numel() * 2
            dec[f"s_q{Rd}"] = {
                "ms": round(msd, 4),
                "GBps": round(io_bytes / msd / 1e6, 1),
                "hbm_frac": round(io_bytes / msd / 1e6 / 8000.0, 4),
                "kernels": [r["name"] for r in mfa.quantized_plan(qdd, mfa.KernelType.forward,
                                                                   tqd, tkd, tvd)],
            }
            if Rd == 1:
                # The same cache as INT4 (two elements per byte): half the K/V bytes.
                kd4 = kd8[..., : Dd // 2].contiguous()
                vd4 = vd8[..., : Dd // 2].contiguous()
                tk4 = mfa.quantized_tensor(kd4, mfa.Precision.INT4, scale=0.25 / 7)
                tv4 = mfa.quantized_tensor(vd4, mfa.Precision.INT4, scale=0.25 / 7)
                qd4 = mfa.quantized_descriptor(based, mfa.Precision.FP16, mfa.Precision.INT4,
                                               mfa.Precision.INT4, B=Bd, H=Hd)
                ms4 = ev_time(lambda: qa.forward(qd4, tqd, tk4, tv4, od8, ld8, stream=stream))
                io4 = kv_bytes // 2 + qd8.numel() * 2 + od8.numel() * 4 + ld8.numel() * 2
                dec["s_q1_int4"] = {
                    "ms": round(ms4, 4),
                    "GBps": round(io4 / ms4 / 1e6, 1),
                    "hbm_frac": round(io4 / ms4 / 1e6 / 8000.0, 4),
                    "kernels": [r["name"] for r in mfa.quantized_plan(qd4, mfa.KernelType.forward,
                                                                       tqd, tk4, tv4)],
                }
                del kd4, vd4
            del qd8, od8, ld8
        result["int8_decode"] = {
            "workload": f"QuantizedAttention forward, INT8 K/V (per-tensor) + fp16 Q, B{Bd} H{Hd} "
                        f"S_kv {Cd} D{Dd}, S_q 1 and 16 (decode / KV cache), non-causal; "
                        f"s_q1_int4: the same shape with INT4 K/V",
            "bytes": "INT8 (INT4) K + V once, plus Q (fp16), O (fp32) and L (fp16); roof 8 TB/s HBM",
            **dec,
        }
        del kd8, vd8

    # ---------------------------------------------------------------- C5: fwd + bwd, D=256
    if not args.no_c5:
        B5, H5, S5, D5 = args.c5_batch, 32, 4096, 256
        q5, k5, v5, do5 = (uniform((B5, H5, S5, D5), torch.float16) for _ in range(4))
        o5 = torch.empty((B5, H5, S5, D5), dtype=torch.float32, device=dev)
        l5 = torch.empty((B5, H5, S5), dtype=torch.float16, device=dev)
        dq5, dk5, dv5 = (torch.empty_like(o5) for _ in range(3))
        db5 = torch.empty((B5, H5, S5), dtype=torch.bfloat16, device=dev)
        base5 = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc5 = mfa.MultiHeadDescriptor.make(base5, B5, H5, S5, D5)

        def step5():
            mha.forward(desc5, q5, k5, v5, o5, l5, stream=stream)
            mha.backward(desc5, q5, k5, v5, o5, do5, l5, dq5, dk5, dv5, db5, stream=stream)

        n5 = 20
        warm(step5)
        el5 = timed_steps(step5, n5)
        f5 = (mfa.attention_flops(B5, H5, S5, S5, D5) +
              mfa.attention_flops(B5, H5, S5, S5, D5, kind="backward"))
        result["fwd_bwd_d256"] = {
            "workload": f"BASELINE configs[4] shard: fp16 fwd+bwd (bwdQ then bwdKV, 7 GEMMs), "
                        f"B={B5} per GPU (64 over 8 GPUs), H32 S4096 D256, non-causal",
            "tflops": round(f5 * n5 * world / el5 / 1e12, 2),
            "roofline_frac": round(f5 * n5 / el5 / 1e12 / PEAK_FP16_TFLOPS, 4),
            "flop_convention": "4*D (fwd) + 10*D (bwd) per pair; the 7-GEMM backward executes 14*D",
            "ms_per_step": round(el5 / n5 * 1e3, 3),
        }
        del q5, k5, v5, do5, o5, l5, dq5, dk5, dv5, db5

    # --------------------------------------------- quantized fwd + bwd (INT8 K/V) vs fp16
    if not args.no_c5 and not args.no_int8:
        Bq, Hq, Sq, Dq = 2, 32, 4096, 256
        q8, do8 = (uniform((Bq, Hq, Sq, Dq), torch.float16) for _ in range(2))
        kf8 = uniform((Bq, Hq, Sq, Dq), torch.float32)
        vf8 = uniform((Bq, Hq, Sq, Dq), torch.float32)
        k8, ks8, _, _ = mfa.quantize(kf8, mfa.Precision.INT8, rows=Bq * Hq * Sq, cols=Dq)
        v8, vs8, _, _ = mfa.quantize(vf8, mfa.Precision.INT8, rows=Bq * Hq * Sq, cols=Dq)
        kh8, vh8 = kf8.half(), vf8.half()
        del kf8, vf8
        o8 = torch.empty((Bq, Hq, Sq, Dq), dtype=torch.float32, device=dev)
        l8 = torch.empty((Bq, Hq, Sq), dtype=torch.float16, device=dev)
        dq8, dk8, dv8 = (torch.empty_like(o8) for _ in range(3))
        db8 = torch.empty((Bq, Hq, Sq), dtype=torch.bfloat16, device=dev)
        base8 = mfa.AttentionDescriptor.make(Sq, Sq, Dq, low_precision=True,
                                             precision=mfa.Precision.FP16)
        qd8 = mfa.quantized_descriptor(base8, mfa.Precision.FP16, mfa.Precision.INT8,
                                       mfa.Precision.INT8, B=Bq, H=Hq)
        tq8 = mfa.quantized_tensor(q8, mfa.Precision.FP16)
        tk8 = mfa.quantized_tensor(k8, mfa.Precision.INT8, scale=float(ks8.item()))
        tv8 = mfa.quantized_tensor(v8, mfa.Precision.INT8, scale=float(vs8.item()))
        qa8 = mfa.QuantizedAttention()
        desc8 = mfa.MultiHeadDescriptor.make(base8, Bq, Hq, Sq, Dq)

        def step_q8():
            qa8.forward(qd8, tq8, tk8, tv8, o8, l8, stream=stream)
            qa8.backwardQuery(qd8, tq8, tk8, tv8, o8, do8, l8, dq8, db8, stream=stream)
            qa8.backwardKeyValue(qd8, tq8, tk8, tv8, do8, l8, db8, dk8, dv8, stream=stream)

        def step_f16():
            mha.forward(desc8, q8, kh8, vh8, o8, l8, stream=stream)
            mha.backward(desc8, q8, kh8, vh8, o8, do8, l8, dq8, dk8, dv8, db8, stream=stream)

        ms_q8 = ev_time(step_q8)
        plan_q8 = [r["name"] for kind in (mfa.KernelType.forward, mfa.KernelType.backwardQuery,
                                          mfa.KernelType.backwardKeyValue)
                   for r in mfa.quantized_plan(qd8, kind, tq8, tk8, tv8)]
        ms_f8 = ev_time(step_f16)
        f8 = (mfa.attention_flops(Bq, Hq, Sq, Sq, Dq) +
              mfa.attention_flops(Bq, Hq, Sq, Sq, Dq, kind="backward"))
        result["int8_fwd_bwd_d256"] = {
            "workload": f"QuantizedAttention forward + backwardQuery + backwardKeyValue, INT8 "
                        f"K/V (per-tensor) + fp16 Q/dO, B{Bq} H{Hq} S{Sq} D{Dq} non-causal "
                        f"(C5-like), against MultiHeadAttention fp16 forward + backward",
            "int8_tflops": round(f8 / (ms_q8 * 1e-3) / 1e12, 2),
            "fp16_tflops": round(f8 / (ms_f8 * 1e-3) / 1e12, 2),
            "ratio_int8_over_fp16": round(ms_f8 / ms_q8, 3),
            "int8_ms": round(ms_q8, 3), "fp16_ms": round(ms_f8, 3),
            "int8_kernels": plan_q8,
        }
        del q8, do8, k8, v8, kh8, vh8, o8, l8, dq8, dk8, dv8, db8

    # ---------------------------------------------------------------- C4: MLA
    if not args.no_mla:
        B4, H4, S4, D4, LAT = 1, 16, 4096, 128, 512
        lat = uniform((B4 * S4, LAT), torch.bfloat16)
        wk = (uniform((LAT, H4 * D4), torch.float32) * 0.176).to(torch.bfloat16)
        wv = (uniform((LAT, H4 * D4), torch.float32) * 0.176).to(torch.bfloat16)
        q4 = uniform((B4, H4, S4, D4), torch.bfloat16)
        o4 = torch.empty((B4, H4, S4, D4), dtype=torch.float32, device=dev)
        kb4 = torch.empty((B4 * S4, H4 * D4), dtype=torch.bfloat16, device=dev)
        vb4 = torch.empty_like(kb4)
        base4 = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)

        def step4():
            mfa.mla_forward(base4, lat, wk, wv, q4, o4, B4, H4, S4, S4, D4, LAT,
                            mfa.Precision.BF16, k_buf=kb4, v_buf=vb4, stream=stream)

        warm(step4)
        n4 = 20
        el4 = timed_steps(step4, n4)
        f4 = 2 * (2 * B4 * S4 * LAT * H4 * D4) + mfa.attention_flops(B4, H4, S4, S4, D4)
        result["mla"] = {
            "workload": "BASELINE configs[3]: mlaCompressed bf16, latent 512 -> 16 heads x 128 "
                        "(K, V decompression GEMMs + attention), S4096, non-causal",
            "tflops": round(f4 * n4 * world / el4 / 1e12, 2),
            "roofline_frac": round(f4 * n4 / el4 / 1e12 / PEAK_FP16_TFLOPS, 4),
            "ms_per_step": round(el4 / n4 * 1e3, 4),
        }
        del lat, wk, wv, q4, o4, kb4, vb4

    # ------------------------------------------- sparse ranges (block-sparse) on the tuned path
    if not args.no_sparse:
        import numpy as np
        Hs, Ss, Ds, blk, band = 16, 4096, 128, 128, 8
        nb = Ss // blk
        pat = np.zeros((nb, nb), dtype=np.uint8)
        for i in range(nb):  # a band of `band` key blocks around the diagonal
            c0 = min(max(0, i - band // 2), nb - band)
            pat[i, c0:c0 + band] = 1
        rb = np.zeros((nb, 2), dtype=np.uint32)
        mfa.lib.mfa_sparse_build_block_sparse(pat.ctypes.data, nb, nb, blk, rb.ctypes.data)
        rows = np.ascontiguousarray(np.broadcast_to(np.repeat(rb, blk, axis=0), (B, Hs, Ss, 2)))
        mask_s = torch.from_numpy(rows.view(np.int32)).to(dev)
        qs, ks_, vs_ = (uniform((B, Hs, Ss, Ds), torch.float16) for _ in range(3))
        os_ = torch.empty((B, Hs, Ss, Ds), dtype=torch.float32, device=dev)
        ls = torch.empty((B, Hs, Ss), dtype=torch.float16, device=dev)
        base_s = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                              sparse_mask=mfa.MaskType.sparseRanges)
        desc_s = mfa.MultiHeadDescriptor.make(base_s, B, Hs, Ss, Ds)
        base_d = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16)
        desc_d = mfa.MultiHeadDescriptor.make(base_d, B, Hs, Ss, Ds)
        ms_sp = ev_time(lambda: mha.forward(desc_s, qs, ks_, vs_, os_, ls, mask=mask_s,
                                            stream=stream))
        mfa.last_launches()
        mha.forward(desc_s, qs, ks_, vs_, os_, ls, mask=mask_s, stream=stream)
        plan_s = [r["name"] for r in mfa.last_launches()]
        ms_dn = ev_time(lambda: mha.forward(desc_d, qs, ks_, vs_, os_, ls, stream=stream))
        pairs = int((rows[0, 0, :, 1].astype(np.int64) - rows[0, 0, :, 0]).sum()) * B * Hs
        fs = 4.0 * Ds * pairs
        # Backward on the same ranges (both phases; the tuned kernels' mask instantiation skips
        # the key tiles / steps no row of a block sees) against the dense backward.
        dos = uniform((B, Hs, Ss, Ds), torch.float16)
        dqs = torch.empty((B, Hs, Ss, Ds), dtype=torch.float32, device=dev)
        dks, dvs = torch.empty_like(dqs), torch.empty_like(dqs)
        dbs = torch.empty((B, Hs, Ss), dtype=torch.bfloat16, device=dev)
        mha.forward(desc_s, qs, ks_, vs_, os_, ls, mask=mask_s, stream=stream)
        bw_sp = ev_time(lambda: mha.backward(desc_s, qs, ks_, vs_, os_, dos, ls, dqs, dks, dvs, dbs,
                                             mask=mask_s, stream=stream))
        mfa.last_launches()
        mha.backward(desc_s, qs, ks_, vs_, os_, dos, ls, dqs, dks, dvs, dbs, mask=mask_s,
                     stream=stream)
        plan_bs = [r["name"] for r in mfa.last_launches()]
        mha.forward(desc_d, qs, ks_, vs_, os_, ls, stream=stream)
        bw_dn = ev_time(lambda: mha.backward(desc_d, qs, ks_, vs_, os_, dos, ls, dqs, dks, dvs, dbs,
                                             stream=stream))
        result["block_sparse"] = {
            "workload": f"sparse ranges from buildBlockSparse, fp16 B{B} H{Hs} S{Ss} D{Ds}, "
                        f"{blk}x{blk} blocks, band of {band} key blocks per row block "
                        f"(density {band / nb:.3f})",
            "tflops_on_kept_pairs": round(fs / (ms_sp * 1e-3) / 1e12, 2),
            "roofline_frac": round(fs / (ms_sp * 1e-3) / 1e12 / PEAK_FP16_TFLOPS, 4),
            "ms": round(ms_sp, 4), "dense_ms": round(ms_dn, 4),
            "speedup_vs_dense": round(ms_dn / ms_sp, 2),
            "kernels": plan_s,
            "bwd_tflops_on_kept_pairs": round(2.5 * fs / (bw_sp * 1e-3) / 1e12, 2),
            "bwd_flop_convention": "10*D per kept pair (the 7-GEMM backward executes 14*D)",
            "bwd_ms": round(bw_sp, 4), "bwd_dense_ms": round(bw_dn, 4),
            "bwd_speedup_vs_dense": round(bw_dn / bw_sp, 2),
            "bwd_kernels": plan_bs,
        }
        del qs, ks_, vs_, os_, ls, mask_s, dos, dqs, dks, dvs, dbs

    # ------------------------------------------------- SURVEY §8(f) rows (one GPU's view)
    if not args.no_next:
        nx = 20
        nxt = {}
        # Absorbed MLA at a decode shape: HBM-bound on the latent cache read.
        Bd, Hd, Sqd, Skd, Dd, LATd = 32, 16, 1, 4096, 128, 512
        latd = uniform((Bd * Skd, LATd), torch.bfloat16)
        wkd = (uniform((LATd, Hd * Dd), torch.float32) * 0.176).to(torch.bfloat16)
        wvd = (uniform((LATd, Hd * Dd), torch.float32) * 0.176).to(torch.bfloat16)
        qd = uniform((Bd, Hd, Sqd, Dd), torch.bfloat16)
        od = torch.empty((Bd, Hd, Sqd, Dd), dtype=torch.float32, device=dev)
        based = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.BF16)
        argsd = (based, latd, wkd, wvd, qd, od, Bd, Hd, Sqd, Skd, Dd, LATd, mfa.Precision.BF16)
        ms_abs = ev_time(lambda: mfa.mla_forward_absorbed(*argsd, stream=stream), nx)
        ms_dec = ev_time(lambda: mfa.mla_forward(*argsd, stream=stream), nx)
        nxt["mla_absorbed_decode"] = {
            "workload": "absorbed MLA, bf16, B32 H16 S_q 1 S_kv 4096, latent 512 -> D 128",
            "ms": round(ms_abs, 4), "decompress_ms": round(ms_dec, 4),
            "speedup_vs_decompress": round(ms_dec / ms_abs, 2),
            "latent_GBps": round(Bd * Skd * LATd * 2 / ms_abs / 1e6, 1),
        }
        del latd, wkd, wvd, qd, od
        # General GEMM (GEMMDescriptor surface): NN (tuned path) and NT / TN (general kernel).
        ng = 4096
        ga = uniform((ng, ng), torch.float16)
        gb = uniform((ng, ng), torch.float16)
        gc = torch.empty((ng, ng), dtype=torch.float32, device=dev)
        for ta, tb in ((False, False), (False, True), (True, False)):
            ms = ev_time(lambda: mfa.gemm(ga, gb, gc, ng, ng, ng, mfa.Precision.FP16,
                                          mfa.Precision.FP32, transpose_a=ta, transpose_b=tb,
                                          stream=stream), nx)
            key = "gemm_fp16_" + ("T" if ta else "N") + ("T" if tb else "N") + "_4096"
            nxt[key] = {"ms": round(ms, 4), "tflops": round(2 * ng ** 3 / ms / 1e9, 1),
                        "roofline_frac": round(2 * ng ** 3 / ms / 1e9 / PEAK_FP16_TFLOPS, 4)}
        del ga, gb, gc
        # Hadamard rotation: 8 bytes per element against the 8 TB/s HBM roof.
        hx = uniform((1 << 28,), torch.float32)
        ms_h = ev_time(lambda: mfa.HadamardRotation().rotate(hx, 128, (1 << 28) // 128,
                                                             stream=stream), nx)
        gbs = 8 * (1 << 28) / ms_h / 1e6
        nxt["hadamard_fp32_1GiB_block128"] = {"ms": round(ms_h, 4), "GBps": round(gbs, 1),
                                              "roofline_frac": round(gbs / 8000.0, 4)}
        del hx
        result["next_rows"] = nxt

    # ------------------------------------------------- strong scaling: C2 split by heads
    # SURVEY §8e's plan for C2 / C3 / C4 (B = 1, H = 16): the heads of ONE batch element split
    # over the N ranks (mfa_shard.forward_slices, no collective).  Reported beside the weak
    # headline: whole-job TFLOP/s of the one C2 problem, per rank, and the per-GPU occupancy
    # against this run's weak per-GPU rate (a rank with H/N heads has 1/N of the blocks).
    if not args.no_strong:
        mine = shard.forward_slices(1, H, H, world, rank)
        nh = sum(h1 - h0 for _, h0, h1 in mine)
        qs, ks, vs = (uniform((1, nh, S, D), torch.float16) for _ in range(3))
        os_ = torch.empty((1, nh, S, D), dtype=torch.float32, device=dev)
        ls = torch.empty((1, nh, S), dtype=torch.float16, device=dev)
        bs = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                          causal=True)
        ds = mfa.MultiHeadDescriptor.make(bs, 1, nh, S, D)
        fn_s = lambda: mha.forward(ds, qs, ks, vs, os_, ls, stream=stream)
        warm(fn_s)
        ns = max(20, args.steps)
        el_s = timed_steps(fn_s, ns)
        f_all = mfa.attention_flops(1, H, S, S, D, causal=True)
        result["strong_heads"] = {
            "workload": f"C2 (B1 H{H} S{S} D{D} causal fp16) split by heads over {world} rank(s)",
            "heads_per_rank": nh if world == 1 else f"{H // world}-{-(-H // world)}",
            "scaling": "strong",
            "tflops": round(f_all * ns / el_s / 1e12, 2),
            "tflops_per_rank": round(f_all * ns / el_s / 1e12 / world, 2),
            "ms_per_step": round(el_s / ns * 1e3, 4),
            "kernel": mfa.multihead_plan(ds)[0]["name"]}
        del qs, ks, vs, os_, ls

    # ---------------------------------------------------------------- headline: C2
    # Measured last: the sections above have brought the chip to its steady clock (a cold
    # start reads 10-15 % low for the first ~0.1 s of back-to-back launches).
    q, k, v = (uniform((B, H, S, D), torch.float16) for _ in range(3))
    o = torch.empty((B, H, S, D), dtype=torch.float32, device=dev)
    l = torch.empty((B, H, S), dtype=torch.float16, device=dev)
    base = mfa.AttentionDescriptor.make(low_precision=True, precision=mfa.Precision.FP16,
                                        causal=True)
    desc = mfa.MultiHeadDescriptor.make(base, B, H, S, D)

    def step():
        mha.forward(desc, q, k, v, o, l, stream=stream)

    warm(step)  # untimed, time-based (the sections above may all be switched off)
    for _ in range(args.warmup):
        step()
    barrier()
    mfa.last_launches()
    # The timed region: barrier + synchronize on both sides.  The K steps are timed by HIP
    # events on the launch stream, so `value` carries no host-side launch /
    # synchronisation latency; the wall clock of the same region is reported beside it.
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record()
    for _ in range(args.steps):
        step()
    ev1.record()
    barrier()
    wall = max_over_ranks(time.perf_counter() - t0)
    elapsed = max_over_ranks(ev0.elapsed_time(ev1) * 1e-3)
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one kernel per step on this stream
    flops_step = mfa.attention_flops(B, H, S, S, D, causal=True)
    total_flops = flops_step * args.steps * world
    value = total_flops / elapsed / 1e12
    achieved = flops_step / (kernel_ms * 1e-3) / 1e12

    # The kernel the library launched for this shape: the plan query (mfa_multihead_plan)
    # names it, and the launch log of the timed calls must agree (one launch per step).
    plan = mfa.multihead_plan(desc, mfa.KernelType.forward, Q=q, K=k, V=v, O=o, L=l)
    ran = mfa.last_launches()
    assert len(plan) == 1 and ran and all(r == plan[0] for r in ran), (plan, ran)
    kname = plan[0]["name"]
    pmc = pmc_record(kname, S, H, D)
    if "strong_heads" in result:
        # Per-GPU occupancy of the heads split: its per-rank rate over this run's weak per-GPU
        # rate (1.0 at N = 1 up to timing noise).
        result["strong_heads"]["per_rank_vs_weak"] = round(
            result["strong_heads"]["tflops_per_rank"] / (value / world), 4)
    result = {
        "metric": "attn TFLOPS/GPU (fwd seq=4096 d=128) fp16 vs INT8; % MFMA roofline",
        "value": round(value, 2),
        "unit": "TFLOPS",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "wall_ms_per_step": round(wall / args.steps * 1e3, 4),
        "wall_value": round(total_flops / wall / 1e12, 2),
        "timing": "value and ms_per_step: HIP events around the K timed steps on the launch "
                  "stream, max over ranks; wall_*: host clock of the same barrier-bracketed "
                  "region (includes launch and synchronisation latency)",
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "fp16",
        "data": "synthetic (uniform [-0.25, 0.25), device RNG)",
        "config": {"workload": "fp16 fwd causal, O fp32, L fp16 (BASELINE configs[1])",
                   "batch_per_gpu": B, "heads": H, "seq_len": S, "head_dim": D,
                   "parallelism": f"batch-sharded x{world}, no collective",
                   "flop_convention": "4*D per unmasked pair (causal S(S+1)/2)",
                   "gflop_per_step_per_gpu": round(flops_step / 1e9, 3)},
        "roofline": {"bound": "mfma", "achieved": round(achieved, 2),
                     "peak": round(PEAK_FP16_TFLOPS, 1), "unit": "TFLOP/s",
                     "frac": round(achieved / PEAK_FP16_TFLOPS, 4),
                     "traffic": pmc.get("hbm_bytes"),
                     # north_star's two utilisation figures for the dominant kernel: MFMA busy
                     # (PMC: SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)) and
                     # achieved HBM GB/s (PMC bytes per launch / this run's kernel time) against
                     # the ~8 TB/s HBM3E peak.
                     "mfma_busy": pmc.get("mfma_busy"),
                     "hbm_GBps": (round(pmc["hbm_bytes"] / (kernel_ms * 1e-3) / 1e9, 1)
                                  if pmc.get("hbm_bytes") else None),
                     "hbm_peak_GBps": 8000.0,
                     "pmc_source": pmc.get("source"),
                     "kernel": kname, "kernel_ms": round(kernel_ms, 4)},
        **result,
    }
    del q, k, v, o, l

    # ---------------------------------------------------------------- CPU baseline
    if rank == 0 and world == 1 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(S, D, H)
        if "next_rows" in result:
            cpu_next_rows(result["next_rows"])

    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def fake_device_run(args, world: int, rank: int):
    """--fake-device: the rank / barrier / max-over-ranks / JSON plumbing of a real run on
    the CPU (gloo), with no GPU and no kernels; a step is a no-op.  Lets a CPU test check
    that `bench.py --gpus N` starts N ranks and reports n_gpus = N."""
    import torch
    import torch.distributed as dist_
    if world > 1:
        dist_.init_process_group("gloo")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pass
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist_.all_reduce(t, op=dist_.ReduceOp.MAX)
        el = float(t.item())
        ranks = [None] * world
        dist_.all_gather_object(ranks, rank)
    else:
        ranks = [0]
    if rank == 0:
        print(json.dumps({"metric": "fake-device dry run", "value": 0.0, "unit": "none",
                          "n_gpus": world, "ranks": ranks, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": el / max(args.steps, 1) * 1e3,
                          "data": "none (--fake-device)"}), flush=True)
    if world > 1:
        dist_.destroy_process_group()


def pmc_record(kernel: str, S: int, H: int, D: int) -> dict:
    """PMC figures of `kernel` per launch from the newest committed rocprofv3 summary
    (profiles/r*_pmc_traffic.json, tools/pmc_traffic.py): HBM bytes (2 x FETCH_SIZE +
    WRITE_SIZE, the gfx950 correction of MI355X_MICROARCH.md) and the MFMA busy fraction;
    collected at the default bench shape only; {} otherwise."""
    if (S, H, D) != (4096, 16, 128):
        return {}
    import glob
    files = sorted(glob.glob(os.path.join(_REPO, "profiles", "r*_pmc_traffic.json")))
    for fn in reversed(files):
        with open(fn) as f:
            rec = json.load(f).get(kernel)
        if rec is not None:
            out = {"hbm_bytes": round(rec["hbm_bytes"]), "source": os.path.basename(fn)}
            if "mfma_busy" in rec:
                out["mfma_busy"] = round(rec["mfma_busy"], 4)
            return out
    return {}


def cpu_baseline(S: int, D: int, H: int):
    """The CPU oracle (C restatement of Network.swift's naive reference) on the whole
    headline workload (all H heads, causal), on the host's threads (OpenMP over query rows;
    at most 16, the box's CPU share)."""
    sys.path.insert(0, os.path.join(_REPO, "tests"))
    import numpy as np
    import oracle_lib as ol
    threads = min(16, os.cpu_count() or 1)
    threads = ol.set_threads(threads)
    rng = np.random.default_rng(0)
    q, k, v = ((rng.random((1, H, S, D), dtype=np.float32) * 2 - 1) * 0.25 for _ in range(3))
    t0 = time.perf_counter()
    ol.attention(q, k, v, causal=True)
    dt = time.perf_counter() - t0
    flops = 4.0 * D * (S * (S + 1) // 2) * H
    return {"value": round(flops / dt / 1e12, 5), "unit": "TFLOPS", "cores": threads,
            "kind": "port",
            "sample": f"the full headline workload (B=1, H={H}, S={S}, D={D}, causal, fp32 "
                      f"inputs), oracle/mfa_oracle.c forward, {dt:.2f} s wall on {threads} "
                      "threads; naive restatement of Network.swift (double accumulation) with "
                      "the reference CPU oracle's causal column limit colLimit = row + 1 "
                      "(KernelRegressionTests.swift:92), so it computes exactly the "
                      "S(S+1)/2 unmasked pairs it is credited with"}


def cpu_next_rows(nxt: dict):
    """The oracle's CPU rate beside each §8(f) row, on bounded samples (same threads as
    cpu_baseline): GEMM 1024^3, Hadamard 64 MiB, absorbed-MLA decode on 4 of the 32 batch
    items (oracle attention on the decompressed K/V: the reference's CPU path)."""
    sys.path.insert(0, os.path.join(_REPO, "tests"))
    import numpy as np
    import oracle_lib as ol
    threads = ol.set_threads(min(16, os.cpu_count() or 1))
    rng = np.random.default_rng(1)
    n = 1024
    a, b = rng.random((n, n), dtype=np.float32), rng.random((n, n), dtype=np.float32)
    t0 = time.perf_counter()
    ol.gemm(a, b)
    dt = time.perf_counter() - t0
    cpu_gemm = {"tflops": round(2 * n ** 3 / dt / 1e12, 5), "cores": threads,
                "sample": "oracle GEMM 1024^3 fp32 (double accumulation)"}
    for k in nxt:
        if k.startswith("gemm_"):
            nxt[k]["cpu"] = cpu_gemm
    x = rng.standard_normal(1 << 24).astype(np.float32)
    t0 = time.perf_counter()
    ol.hadamard(x, 128, float(np.float32(1 / np.sqrt(128.0))))
    dt = time.perf_counter() - t0
    if "hadamard_fp32_1GiB_block128" in nxt:
        nxt["hadamard_fp32_1GiB_block128"]["cpu"] = {
            "GBps": round(8 * x.size / dt / 1e9, 3), "cores": 1,
            "sample": "oracle FWHT (the reference kernel's loops, one block after another), 64 MiB"}
    if "mla_absorbed_decode" in nxt:
        Bs, H, Skv, D, LAT = 4, 16, 4096, 128, 512
        lat = rng.standard_normal((Bs * Skv, LAT)).astype(np.float32)
        wk = (rng.standard_normal((LAT, H * D)) * LAT ** -0.5).astype(np.float32)
        wv = (rng.standard_normal((LAT, H * D)) * LAT ** -0.5).astype(np.float32)
        q = rng.standard_normal((Bs, H, 1, D)).astype(np.float32)
        t0 = time.perf_counter()
        K = ol.gemm(lat, wk).reshape(Bs, Skv, H, D).transpose(0, 2, 1, 3)
        V = ol.gemm(lat, wv).reshape(Bs, Skv, H, D).transpose(0, 2, 1, 3)
        ol.attention(np.ascontiguousarray(q), np.ascontiguousarray(K), np.ascontiguousarray(V))
        dt = time.perf_counter() - t0
        nxt["mla_absorbed_decode"]["cpu"] = {
            "ms_full_workload": round(dt * 1e3 * 32 / Bs, 1), "cores": threads,
            "sample": f"oracle decompress GEMMs + attention on {Bs} of the 32 batch items, "
                      f"{dt:.2f} s, scaled x{32 // Bs}"}


if __name__ == "__main__":
    main()
