"""GPU parity for the Hadamard rotation kernel (HadamardRotation.rotate / rotateBatch):
bit-exact against the oracle's restatement of the reference's MSL kernel
(HadamardRotation.swift:111-136) — the butterflies keep the reference's stage order and
operand order, so every element is the same sequence of FP32 additions."""
import numpy as np
import pytest
import torch

import mfa_amd as mfa
import oracle_lib as ol

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.mark.parametrize("n", [1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024])
@pytest.mark.parametrize("nb", [1, 3, 257, 1000])
def test_rotate_bit_exact(gpu, n, nb):
    rng = np.random.default_rng(n * 1000 + nb)
    x = rng.standard_normal((nb, n)).astype(np.float32)
    x[0, :] *= 1e4  # outlier rows: the use case (ConvRot outlier smoothing)
    t = torch.from_numpy(x).to(DEV)
    hr = mfa.HadamardRotation()
    hr.rotate(t, n, nb)
    torch.cuda.synchronize()
    ref = ol.hadamard(x, n, hr.scale(n))
    assert np.array_equal(t.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_rotate_leaves_tail_untouched(gpu):
    # Only num_blocks * block_size elements change; the rest of the allocation is left alone.
    x = torch.arange(1000, dtype=torch.float32, device=DEV)
    mfa.HadamardRotation().rotate(x, 64, 10)
    torch.cuda.synchronize()
    assert torch.equal(x[640:].cpu(), torch.arange(640, 1000, dtype=torch.float32))


def test_rotate_batch_and_involution(gpu):
    rng = np.random.default_rng(3)
    a = rng.integers(-50, 50, size=(64, 256)).astype(np.float32)
    b = rng.integers(-50, 50, size=(9, 1024)).astype(np.float32)
    ta, tb = torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)
    hr = mfa.HadamardRotation()
    hr.rotate_batch([(ta, 256, 64), (tb, 1024, 9)])
    torch.cuda.synchronize()
    assert np.array_equal(ta.cpu().numpy(), ol.hadamard(a, 256, hr.scale(256)))
    assert np.array_equal(tb.cpu().numpy(), ol.hadamard(b, 1024, hr.scale(1024)))
    # H/√N is orthogonal and symmetric: rotating twice restores integer data exactly at N = 4^k.
    hr.rotate_batch([(ta, 256, 64), (tb, 1024, 9)])
    torch.cuda.synchronize()
    assert np.array_equal(ta.cpu().numpy(), a)
    assert np.array_equal(tb.cpu().numpy(), b)


def test_rotate_large(gpu):
    # Size-independent property at a large size (1 GiB buffer): orthogonality keeps the
    # squared norm of each block (to FP32 rounding) and the second rotation restores x.
    nb, n = 1 << 18, 1024
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn((nb, n), device=DEV, generator=g)
    y = x.clone()
    hr = mfa.HadamardRotation()
    hr.rotate(y, n, nb)
    torch.cuda.synchronize()
    nx, ny = x.double().pow(2).sum(1), y.double().pow(2).sum(1)
    assert torch.max(torch.abs(nx - ny) / nx).item() < 1e-5
    hr.rotate(y, n, nb)
    torch.cuda.synchronize()
    assert torch.max(torch.abs(y - x)).item() < 1e-4
