#!/usr/bin/env python3
"""Generates the committed golden fixtures under tests/golden/ (TEST INFRASTRUCTURE).

The reference (Swift + Metal) cannot be built or run in this image, and its test suite holds no
committed output vectors: every fixture here is produced by the CPU oracle
(oracle/mfa_oracle.c, a restatement of the reference's naive CPU attention,
Tests/FlashAttentionTests/.../Network.swift and QuantizedAttentionTest.swift:822-936), on the
reference's own deterministic input generators:
  * KernelRegressionTests.swift:41-50 LCG, scale 0.25, seeds Q=11 K=22 V=33 dO=44;
  * QuantizedAttentionTest.swift:446-450 nextRandom stream seeded 0x5EED5EED.
The oracle itself is pinned by tests/test_oracle.py (known answers taken from the reference's
tests, an independent numpy restatement, finite differences).  These files freeze its outputs
so that the GPU parity tests and later rounds compare against fixed vectors.

Run:  python tests/golden/make_golden.py   (writes *.npz next to this file)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_lib as ol  # noqa: E402


def lcg4(shape, seeds):
    n = int(np.prod(shape))
    return [ol.lcg(s, n).reshape(shape) for s in seeds]


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **{k: np.ascontiguousarray(v) for k, v in arrays.items()})
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


def main():
    # C1 (BASELINE configs[0]): 1 head, fp32, S=128, D=64, forward + backward, non-causal.
    Q, K, V, dO = lcg4((1, 1, 128, 64), (11, 22, 33, 44))
    r = ol.attention(Q, K, V, dO=dO)
    save("c1_fp32_s128_d64.npz", Q=Q, K=K, V=V, dO=dO, O=r["O"], L=r["L"], D=r["D"],
         dQ=r["dQ"], dK=r["dK"], dV=r["dV"])

    # Causal batched case (KernelRegressionTests.swift:72-147 shape family): B2 H2 S96 D32.
    Q, K, V, dO = lcg4((2, 2, 96, 32), (111, 122, 133, 144))
    r = ol.attention(Q, K, V, causal=True, dO=dO)
    save("causal_fp32_b2h2_s96_d32.npz", Q=Q, K=K, V=V, dO=dO, O=r["O"], L=r["L"], D=r["D"],
         dQ=r["dQ"], dK=r["dK"], dV=r["dV"])

    # Sliding window (row > col + W masked) with cross-attention R != C: B1 H2 R80 C112 D32 W24.
    Q = ol.lcg(211, 1 * 2 * 80 * 32).reshape(1, 2, 80, 32)
    K = ol.lcg(222, 1 * 2 * 112 * 32).reshape(1, 2, 112, 32)
    V = ol.lcg(233, 1 * 2 * 112 * 32).reshape(1, 2, 112, 32)
    r = ol.attention(Q, K, V, window=24)
    save("window_fp32_r80_c112_d32_w24.npz", Q=Q, K=K, V=V, O=r["O"], L=r["L"])

    # QuantizedAttentionTest.testQuantizedForwardCorrectness stream (S32 D16): INT8 bytes and
    # scales of Q, K, V (tensor-wise, GEMMQuantization.swift:305-350, :487-521) and the
    # forward on the dequantised values.
    S, D = 32, 16
    g = ol.LCGStream(0x5EED5EED)
    Qs, Ks, Vs = (g.draw(S * D).reshape(1, 1, S, D) for _ in range(3))
    out = {"Q": Qs, "K": Ks, "V": Vs}
    deq = {}
    for name, x in (("Q", Qs), ("K", Ks), ("V", Vs)):
        for prec, tag in ((ol.INT8, "i8"), (ol.INT4, "i4")):
            s = ol.quant_scale_tensor(x, prec)
            q = ol.quantize(x, prec, s)
            out[f"{name}_{tag}"] = q
            out[f"{name}_{tag}_scale"] = np.array([s], dtype=np.float32)
            if prec == ol.INT8:
                deq[name] = ol.dequantize(q, x.size, prec, s).reshape(x.shape)
    out["O_fp32"] = ol.attention(Qs, Ks, Vs)["O"]
    out["O_deq_i8"] = ol.attention(deq["Q"], deq["K"], deq["V"])["O"]
    save("quant_stream_s32_d16.npz", **out)

    # Blockwise INT8 (QuantizedAttentionTest.testBlockwiseAttentionForward data, bs 8).
    rows, cols, bs = 32, 32, 8
    i = np.arange(rows * cols)
    br, bc = (i // cols) // bs, (i % cols) // bs
    Kb = (((i % 7).astype(np.float32) - 3) * ((br + 1) * (bc + 1)).astype(np.float32)
          * np.float32(0.1)).astype(np.float32)
    sc = ol.quant_scales_block(Kb, rows, cols, bs, ol.INT8)
    qb = ol.quantize_block(Kb, cols, bs, ol.INT8, sc)
    save("blockwise_i8_32x32_bs8.npz", x=Kb, scales=sc, q=qb)


if __name__ == "__main__":
    main()
