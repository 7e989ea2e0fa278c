"""CPU tests: pin the oracle against the reference's own known-answer tests and against an
independent float64 restatement (no GPU needed).

Reference known answers used (paths relative to the reference repo):
  - QuantizedAttentionTest.testQuantizationParameters            (:30-59)
  - QuantizedAttentionTest.testQuantizeAndDequantize             (:61-161)
  - QuantizedAttentionTest.testQuantizedTensorCreation           (:163-191)
  - QuantizedAttentionTest.testBlockwiseQuantizationRoundTrip    (:657-701)
  - BlockwiseCompensationTest compensation identity              (:10-11, :58-112)
  - KernelRegressionTests.deterministicData / bf16Bytes          (:41-59)
  - Network.swift:14-60 finite-difference validation of the analytic gradients
"""
import math

import numpy as np
import pytest

import oracle_lib as ol

INT8, INT4 = ol.INT8, ol.INT4


# --------------------------------------------------------------------------- quantisation
def test_quantization_parameters_known_answer():
    x = np.array([-10.0, -5.0, 0.0, 5.0, 10.0], dtype=np.float32)
    assert abs(ol.quant_scale_tensor(x, INT8) - 10.0 / 127.0) <= 1e-6
    assert abs(ol.quant_scale_tensor(x, INT4) - 10.0 / 7.0) <= 1e-6
    # Exact float32 arithmetic: absmax / 127 in float.
    assert ol.quant_scale_tensor(x, INT8) == np.float32(10.0) / np.float32(127.0)


@pytest.mark.parametrize("prec", [INT8, INT4])
def test_quantize_dequantize_round_trip(prec):
    x = np.arange(-10.0, 10.0 + 1e-9, 0.5, dtype=np.float32)
    s = ol.quant_scale_tensor(x, prec)
    q = ol.quantize(x, prec, s)
    y = ol.dequantize(q, x.size, prec, s)
    assert np.all(np.abs(y - x) < 2 * s)


def test_quantized_tensor_creation_round_trip():
    x = (np.arange(100, dtype=np.float32) * np.float32(0.1) - np.float32(5.0)).astype(np.float32)
    s = ol.quant_scale_tensor(x, INT8)
    y = ol.dequantize(ol.quantize(x, INT8, s), 100, INT8, s)
    assert np.all(np.abs(y - x) < 2 * s)


def test_blockwise_round_trip_known_answer():
    rows, cols, bs = 16, 32, 8
    i = np.arange(rows * cols)
    br, bc = (i // cols) // bs, (i % cols) // bs
    data = ((i % 7).astype(np.float32) - 3) * ((br + 1) * (bc + 1)).astype(np.float32)
    scales = ol.quant_scales_block(data, rows, cols, bs, INT8)
    assert scales.size == ((rows + bs - 1) // bs) * ((cols + bs - 1) // bs)
    q = ol.quantize_block(data, cols, bs, INT8, scales)
    y = ol.dequantize_block(q, data.size, cols, bs, INT8, scales)
    nbc = (cols + bs - 1) // bs
    blk = scales[(i // cols // bs) * nbc + (i % cols) // bs]
    assert np.all(np.abs(y - data) <= blk * 2.01)


def test_int8_rounding_and_clamping():
    # round half away from zero (Swift round), Int8(clamping:)
    x = np.array([2.5, -2.5, 0.5, -0.5, 1.49, 300.0, -300.0], dtype=np.float32)
    q = ol.quantize(x, INT8, 1.0).view(np.int8)
    assert q.tolist() == [3, -3, 1, -1, 1, 127, -128]


def test_int4_packing_known_answer():
    # element 2i -> low nibble, (q + 8) clamped to [0, 15] (GEMMQuantization.swift:500-516)
    x = np.array([1.0, -1.0, 7.0, -8.0, 20.0], dtype=np.float32)
    q = ol.quantize(x, INT4, 1.0)
    assert q.tolist() == [0x79, 0x0F, 0x8F]  # odd tail padded with nibble 8 (value 0)
    qb = ol.quantize_block(x, 5, 8, INT4, np.array([1.0], dtype=np.float32))
    assert qb.tolist() == [0x79, 0x0F, 0x0F]  # block-wise leaves the tail nibble 0
    y = ol.dequantize(q, 5, INT4, 1.0)
    assert y.tolist() == [1.0, -1.0, 7.0, -8.0, 7.0]


def test_row_wise_scales():
    x = np.array([[1, -4, 2], [0.5, 0.25, -0.125]], dtype=np.float32)
    s = ol.quant_scales_row(x, 2, 3, INT8)
    assert s.tolist() == [np.float32(4) / np.float32(127), np.float32(0.5) / np.float32(127)]


def test_blockwise_compensation_identity():
    # acc = Σ_b s_a s_b (Sqq - z_b SqA - z_a SqB + cnt z_a z_b) equals Σ (qa-za)(qb-zb) s_a s_b,
    # the dequantize-on-load product the kernels compute.
    rng = np.random.default_rng(0)
    M, N, K, bs = 3, 4, 24, 8
    qa = rng.integers(-128, 128, (M, K))
    qb = rng.integers(-128, 128, (K, N))
    nb = K // bs
    sa, sb = rng.random(nb) + 0.1, rng.random(nb) + 0.1
    za, zb = rng.integers(-3, 4, nb), rng.integers(-3, 4, nb)
    comp = np.zeros((M, N))
    direct = np.zeros((M, N))
    for b in range(nb):
        sl = slice(b * bs, (b + 1) * bs)
        A, Bm = qa[:, sl].astype(np.float64), qb[sl, :].astype(np.float64)
        sqq, sqa, sqb = A @ Bm, A.sum(1, keepdims=True), Bm.sum(0, keepdims=True)
        comp += sa[b] * sb[b] * (sqq - zb[b] * sqa - za[b] * sqb + bs * za[b] * zb[b])
        direct += sa[b] * sb[b] * ((A - za[b]) @ (Bm - zb[b]))
    assert np.allclose(comp, direct, rtol=1e-12, atol=1e-9)


# --------------------------------------------------------------------------- generators
def _lcg_python(seed, count, scale):
    M = (1 << 64) - 1
    st = (seed * 6364136223846793005 + 1442695040888963407) & M
    out = []
    for _ in range(count):
        st = (st * 6364136223846793005 + 1442695040888963407) & M
        unit = np.float32(st >> 40) / np.float32(1 << 24)
        out.append((unit * np.float32(2) - np.float32(1)) * np.float32(scale))
    return np.array(out, dtype=np.float32)


def test_lcg_matches_independent_restatement():
    for seed in (11, 22, 33, 707):
        assert np.array_equal(ol.lcg(seed, 64, 0.25), _lcg_python(seed, 64, 0.25))
    x = ol.lcg(11, 100000)
    assert x.min() >= -0.25 and x.max() < 0.25


def test_quantized_test_stream_generator():
    # nextRandom: Float(Int32(truncatingIfNeeded: seed)) / Float(Int32.max)
    M = (1 << 64) - 1
    st = 0x5EED5EED
    ref = []
    for _ in range(16):
        st = (st * 6364136223846793005 + 1442695040888963407) & M
        i32 = np.uint32(st & 0xFFFFFFFF).view(np.int32)
        ref.append(np.float32(i32) / np.float32(2147483647) * np.float32(2) - np.float32(1))
    g = ol.LCGStream(0x5EED5EED)
    assert np.array_equal(g.draw(16), np.array(ref, dtype=np.float32))


def test_16bit_conversions_match_numpy_and_reference_formula():
    rng = np.random.default_rng(1)
    x = np.concatenate([rng.standard_normal(20000).astype(np.float32) * s
                        for s in (1e-7, 1e-5, 1e-3, 1.0, 1e2, 6e4)])
    assert np.array_equal(ol.round16(x, "fp16"), x.astype(np.float16).astype(np.float32))
    # bf16 RNE exactly as KernelRegressionTests.bf16Bytes: (bits + 0x7FFF + lsb) >> 16
    bits = x.view(np.uint32).astype(np.uint64)
    rne = (((bits + 0x7FFF + ((bits >> 16) & 1)) >> 16) << 16).astype(np.uint32).view(np.float32)
    assert np.array_equal(ol.round16(x, "bf16"), rne)
    trunc = ((bits >> 16) << 16).astype(np.uint32).view(np.float32)
    assert np.array_equal(ol.round16(x, "bf16_trunc"), trunc)


# --------------------------------------------------------------------------- attention
def numpy_attention(Q, K, V, scale=None, causal=False, window=None, amask=None, ranges=None,
                    dO=None):
    """Independent float64 restatement (matrix form, base-e softmax)."""
    B, H, R, D = Q.shape
    Hkv, C = K.shape[1], K.shape[2]
    scale = 1 / math.sqrt(D) if scale is None else scale
    mask_value = -(np.float32(0.875) / np.float32(1.442695041)) * np.float32(3.402823466e38)
    O = np.zeros((B, H, R, D)); L = np.zeros((B, H, R))
    grads = dO is not None
    if grads:
        dQ = np.zeros((B, H, R, D)); dK = np.zeros((B, Hkv, C, D)); dV = np.zeros((B, Hkv, C, D))
        Dt = np.zeros((B, H, R))
    r_idx = np.arange(R)[:, None]
    c_idx = np.arange(C)[None, :]
    for b in range(B):
        for h in range(H):
            kv = h % Hkv
            q, k, v = (x.astype(np.float64) for x in (Q[b, h], K[b, kv], V[b, kv]))
            S = q @ k.T
            if amask is not None:
                S = S + amask[b, h]
            m = np.zeros((R, C), bool)
            if causal:
                m |= c_idx > r_idx
            if window is not None:
                m |= r_idx > c_idx + window
            if ranges is not None:
                rg = ranges[b, kv]
                m |= (c_idx < rg[:, 0:1]) | (c_idx >= rg[:, 1:2])
            S = np.where(m, float(mask_value), S)
            z = S * scale
            mx = z.max(1, keepdims=True)
            P = np.exp(z - mx)
            ssum = P.sum(1, keepdims=True)
            P /= ssum
            O[b, h] = P @ v
            L[b, h] = (mx[:, 0] + np.log(ssum[:, 0])) * np.log2(np.e)
            if grads:
                do = dO[b, h].astype(np.float64)
                Dn = (do * O[b, h]).sum(1)
                dP = do @ v.T
                dS = P * (dP - Dn[:, None]) * scale
                dQ[b, h] = dS @ k
                dK[b, kv] += dS.T @ q
                dV[b, kv] += P.T @ do
                Dt[b, h] = scale * Dn
    out = {"O": O, "L": L}
    if grads:
        out.update(dQ=dQ, dK=dK, dV=dV, D=Dt)
    return out


CASES = [
    dict(shape=(1, 1, 17, 9, 9), kw={}),
    dict(shape=(2, 4, 33, 40, 16), kw=dict(causal=True)),
    dict(shape=(1, 4, 30, 30, 8), kw=dict(window=5), hkv=2),
    dict(shape=(1, 2, 25, 31, 12), kw=dict(scale=0.3, amask=True)),
    dict(shape=(2, 2, 20, 20, 8), kw=dict(ranges=True), hkv=1),
]


@pytest.mark.parametrize("case", CASES)
def test_oracle_matches_independent_numpy(case):
    B, H, R, C, D = case["shape"]
    Hkv = case.get("hkv", H)
    rng = np.random.default_rng(R * 7 + C)
    Q = rng.standard_normal((B, H, R, D)).astype(np.float32)
    K = rng.standard_normal((B, Hkv, C, D)).astype(np.float32)
    V = rng.standard_normal((B, Hkv, C, D)).astype(np.float32)
    dO = rng.standard_normal((B, H, R, D)).astype(np.float32)
    kw = dict(case["kw"])
    if kw.pop("amask", False):
        kw["amask"] = rng.standard_normal((B, H, R, C)).astype(np.float32)
    if kw.pop("ranges", False):
        lo = rng.integers(0, C // 2, (B, Hkv, R))
        kw["ranges"] = np.stack([lo, lo + rng.integers(1, C // 2, (B, Hkv, R))], -1).astype(np.uint32)
    got = ol.attention(Q, K, V, dO=dO, **kw)
    ref = numpy_attention(Q, K, V, dO=dO, **kw)
    for name in ("O", "L", "D", "dQ", "dK", "dV"):
        assert np.allclose(got[name], ref[name], rtol=1e-5, atol=1e-5), name


def test_fully_masked_row_is_uniform_average():
    # The reference's finite mask value (AttentionKernel+Softmax.swift:257) makes a row that is
    # masked everywhere an average of V over the keys.
    rng = np.random.default_rng(3)
    Q, K, V = (rng.standard_normal((1, 1, 6, 4)).astype(np.float32) for _ in range(3))
    ranges = np.zeros((1, 1, 6, 2), dtype=np.uint32)
    ranges[..., 1] = 6
    ranges[0, 0, 2] = (3, 3)  # empty
    out = ol.attention(Q, K, V, ranges=ranges)
    assert np.allclose(out["O"][0, 0, 2], V[0, 0].mean(0), atol=1e-6)


def test_finite_difference_gradients():
    # Network.swift:14-60: Φ = Σ dO∘O, compare analytic dQ/dK/dV with central differences.
    rng = np.random.default_rng(5)
    B, H, R, C, D = 1, 1, 5, 6, 3
    Q = rng.standard_normal((B, H, R, D)).astype(np.float32)
    K = rng.standard_normal((B, H, C, D)).astype(np.float32)
    V = rng.standard_normal((B, H, C, D)).astype(np.float32)
    dO = rng.standard_normal((B, H, R, D)).astype(np.float32)
    ana = ol.attention(Q, K, V, dO=dO, causal=True)

    def phi(q, k, v):
        return float((ol.attention(q, k, v, causal=True)["O"].astype(np.float64) * dO).sum())

    eps = 1e-2
    for name, X in (("dQ", Q), ("dK", K), ("dV", V)):
        num = np.zeros_like(X, dtype=np.float64)
        for idx in np.ndindex(X.shape):
            Xp, Xm = X.copy(), X.copy()
            Xp[idx] += eps
            Xm[idx] -= eps
            args_p = [Q, K, V]
            args_m = [Q, K, V]
            pos = {"dQ": 0, "dK": 1, "dV": 2}[name]
            args_p[pos], args_m[pos] = Xp, Xm
            num[idx] = (phi(*args_p) - phi(*args_m)) / (2 * eps)
        assert np.allclose(ana[name], num, rtol=2e-2, atol=2e-3), name


def test_gemm_oracle():
    rng = np.random.default_rng(9)
    A = rng.standard_normal((17, 33)).astype(np.float32)
    Bm = rng.standard_normal((33, 9)).astype(np.float32)
    assert np.allclose(ol.gemm(A, Bm), A.astype(np.float64) @ Bm, rtol=1e-5, atol=1e-5)
