"""Seeded random shapes across every launch path: the small-M path (M <= 4),
the gather with and without split-K, the MFMA path (density >= 0.055 with
M >= 5, where the per-launch cost model picks it; K split over small
grids), column blocks with a row
pitch, all five variants.  Float inputs within the fp32 bound of the exact
sums, integer inputs bit-exact with the reference's own order (the oracle
restates tcsc.c).  $TCSC_FUZZ_CASES widens the sweep (default 60)."""
import os

import numpy as np
import pytest

import pyoracle
import tcsc_amd

pytestmark = pytest.mark.gpu

CASES = int(os.environ.get("TCSC_FUZZ_CASES", "60"))


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


def _case(i):
    rng = np.random.default_rng(1000 + i)
    M = int(rng.choice([1, 2, 3, 5, 8, 13, 16, 17, 40, 64, 100, 257, 300]))
    K = int(rng.integers(1, 2500))
    N = int(rng.integers(1, 700))
    density = float(rng.choice([0.005, 0.02, 0.1, 0.25, 0.5, 0.9]))
    c0 = int(rng.integers(0, N))
    c1 = int(rng.integers(c0 + 1, N + 1))
    pad = int(rng.integers(0, 9))
    return M, K, N, density, c0, c1, pad


@pytest.mark.parametrize("i", range(CASES))
def test_random_shape(gpu, oracle, i):
    import torch

    M, K, N, density, c0, c1, pad = _case(i)
    dev = torch.device("cuda:0")
    Wd = oracle.ternary((K, N), density, 2000 + i)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    nc = c1 - c0
    ldy = nc + pad
    plan = tcsc_amd.Plan(W, c0, c1)
    X, B = oracle.uniform((M, K), 3000 + i), oracle.uniform((N,), 4000 + i)
    Xi, Bi = oracle.integers((M, K), 5000 + i), oracle.integers((N,), 6000 + i)
    Y64, S64 = oracle.f64_rows(X, Wref, B)
    Wsl = Wref.column_slice(c0, c1)
    for variant in pyoracle.VARIANTS:
        for x, b, exact in ((X, B, False), (Xi, Bi, True)):
            dY = torch.full((M, ldy), 7.0, device=dev)
            plan.sgemm(torch.from_numpy(x).to(dev), torch.from_numpy(b[c0:c1].copy()).to(dev), dY, M, ldy,
                       variant, 0.2)
            torch.cuda.synchronize()
            Y = dY.cpu().numpy()
            assert np.all(Y[:, nc:] == 7.0), "wrote past the block"
            Y = Y[:, :nc]
            what = f"case {i} M={M} K={K} N={N} d={density} [{c0},{c1}) {variant}"
            if exact:
                np.testing.assert_array_equal(Y, oracle.sgemm(variant, x, Wsl, b[c0:c1].copy(), 0.2), err_msg=what)
            else:
                ok, ratio = pyoracle.check_close(Y, Y64[:, c0:c1], S64[:, c0:c1],
                                                 0.2 if variant in pyoracle.PRELU_VARIANTS else None)
                assert ok, f"{what}: worst err/bound {ratio:.3g}"
    plan.destroy()
    W.free()
