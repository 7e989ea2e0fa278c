"""Hadamard rotation (HadamardRotation.swift) — oracle known answers and ABI preconditions
(CPU only; the GPU kernel's parity is tests/test_hadamard_gpu.py).

The reference ships no Hadamard test; the known answers here are the transform's own
identities: FWHT(e_0) = (1, …, 1)·scale, FWHT(FWHT(x)) = N·x exactly for small integers, and
the Sylvester matrix H_N (H_{2N} = [[H, H], [H, −H]]) applied as a dense product."""
import numpy as np
import pytest

import mfa_amd as mfa
import oracle_lib as ol


def sylvester(n: int) -> np.ndarray:
    h = np.ones((1, 1))
    while h.shape[0] < n:
        h = np.block([[h, h], [h, -h]])
    return h


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024])
def test_oracle_matches_sylvester(n):
    rng = np.random.default_rng(n)
    x = rng.integers(-8, 8, size=(3, n)).astype(np.float32)
    y = ol.hadamard(x, n, 1.0)
    assert np.array_equal(y, (x.astype(np.float64) @ sylvester(n).T).astype(np.float32))
    e0 = np.zeros((1, n), np.float32)
    e0[0, 0] = 1
    s = mfa.HadamardRotation.scale(n)
    assert np.array_equal(ol.hadamard(e0, n, s), np.full((1, n), s, np.float32))
    assert np.array_equal(ol.hadamard(ol.hadamard(x, n, 1.0), n, 1.0), x * n)


def test_scale_values():
    for k in range(11):
        n = 1 << k
        s = mfa.HadamardRotation.scale(n)
        assert s == np.float32(1 / np.sqrt(np.float64(n)))
        if k % 2 == 0:
            assert s == 2.0 ** (-k // 2)


@pytest.mark.parametrize("bs,nb", [(3, 1), (0, 1), (2048, 1), (6, 4), (16, 0)])
def test_preconditions(bs, nb):
    import ctypes
    buf = (ctypes.c_float * 64)()
    st = mfa.lib.mfa_hadamard_rotate(ctypes.addressof(buf), bs, nb, None)
    assert st == 4  # MFA_ERR_INVALID_ARGUMENT: the reference's precondition failures
    assert b"blockSize" in mfa.lib.mfa_last_error() or b"numBlocks" in mfa.lib.mfa_last_error()
