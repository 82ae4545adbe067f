"""The fast order against the reference's own dense oracles, bit for bit on
float inputs.

The fast order adds each column's nonzeros in ascending k and the bias after
the sum, for every variant.  A ternary W makes every product exact, so that
is exactly the arithmetic of the reference's dense oracles:
  * dense.c:64-77 gemm_basic   y = 0; y += X*W over k; Y = y + B
    (what main.cpp:307-331 validates tcsc_sgemm_basic / _optimized against,
    with an absolute 1e-4);
  * SparseGEMM.h:136-149 GEMM_PReLU   the same, then (y < 0) ? a*y : y.
Whenever K is not split over workgroups (TCSC_SLICES=1, or the small-M path)
the GPU output must therefore equal those oracles bit for bit -- the
reference's code compiled in place (oracle/_ref, IEEE flags) where it is
present, else the oracle's restatement of gemm_basic.  Shapes: the gather
path (one and several row tiles, ragged N), the small-M path (M = 1, 3, 16),
and the reference harness's M = 1, K = 2048, N = 8192, 50 % case at full
size (the one whose 1e-4 check a butterfly-summed small-M path missed)."""
import numpy as np
import pytest

import pyoracle
import tcsc_amd

pytestmark = [pytest.mark.gpu, pytest.mark.config_parity]


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


@pytest.fixture(scope="module")
def dense_ref(oracle):
    ref = pyoracle.load_reference()
    if ref is not None:
        return ref.gemm_basic, (lambda X, Wd, B, a: ref.gemm_prelu(X, Wd, B, a)), "reference dense.c / SparseGEMM.h"
    return oracle.gemm_basic, (lambda X, Wd, B, a: pyoracle.prelu(oracle.gemm_basic(X, Wd, B), a)), "oracle restatement"


def run(W, X, B, variant, a=0.2):
    import torch

    dev = torch.device("cuda:0")
    plan = tcsc_amd.Plan(W, 0, W.cols)
    M, N = X.shape[0], W.cols
    dX = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
    dB = torch.from_numpy(np.ascontiguousarray(B)).to(dev)
    dY = torch.full((M, N), float("nan"), device=dev)
    path, slices = plan.launch_info(M)
    plan.sgemm(dX, dB, dY, M, N, variant, a)
    torch.cuda.synchronize()
    plan.destroy()
    return dY.cpu().numpy(), path, slices


SHAPES = [  # M, K, N, density
    (1, 2048, 8192, 0.5),    # main.cpp:261's case 3 (small-M path)
    (1, 3000, 700, 0.1),     # small-M path
    (3, 1000, 300, 0.2),
    (16, 4096, 512, 0.05),
    (200, 3000, 700, 0.05),  # gather path, one row tile, ragged column block
    (700, 2000, 300, 0.1),   # gather path, three row tiles
]


@pytest.mark.parametrize("M,K,N,density", SHAPES)
def test_fast_order_equals_dense_oracle(gpu, oracle, dense_ref, monkeypatch, M, K, N, density):
    monkeypatch.setenv("TCSC_SLICES", "1")
    monkeypatch.setenv("TCSC_PATH", "gather")  # the MFMA path sums in its own order
    gemm_basic, gemm_prelu, src = dense_ref
    Wd = oracle.ternary((K, N), density, 500 + M + K)
    X, B = oracle.uniform((M, K), 600 + M), oracle.uniform((N,), 700 + N)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Yb = gemm_basic(X, Wd, B)
    Yp = gemm_prelu(X, Wd, B, 0.2)
    for variant in pyoracle.VARIANTS:
        Y, path, slices = run(W, X, B, variant)
        assert slices == 1 and path in ("gather", "small"), (path, slices)
        want = Yp if variant in pyoracle.PRELU_VARIANTS else Yb
        bad = np.flatnonzero(Y.view(np.uint32) != want.view(np.uint32))
        assert bad.size == 0, (f"{variant} ({path}) vs {src}: {bad.size} of {Y.size} differ, first at "
                               f"{np.unravel_index(bad[0], Y.shape)}: {Y.flat[bad[0]]!r} vs {want.flat[bad[0]]!r}")
    W.free()


def test_reference_harness_tolerance_holds(gpu, oracle, dense_ref, monkeypatch):
    """main.cpp's own check (dense.c compare: |res - tar| <= 1e-4) on its
    five shapes with fresh random data, tcsc_sgemm_basic through the default
    paths (small-M for M = 1, the MFMA path for M = 256 at 50 %): the M = 1
    cases are exact, the MFMA ones within 1e-4."""
    gemm_basic, _, _ = dense_ref
    for i, (M, K, N) in enumerate([(1, 512, 2048), (1, 1024, 4096), (1, 2048, 8192), (256, 512, 2048),
                                   (256, 1024, 4096)]):
        Wd = oracle.ternary((K, N), 0.5, 900 + i)
        X, B = oracle.uniform((M, K), 910 + i), oracle.uniform((N,), 920 + i)
        W = tcsc_amd.TcscMatrix.from_dense(Wd)
        Y, path, _ = run(W, X, B, "basic")
        ref = gemm_basic(X, Wd, B)
        err = float(np.abs(Y.astype(np.float64) - ref).max())
        assert err <= 1e-4, f"{M}x{K}x{N} ({path}): max |y - gemm_basic| = {err:.3g}"
        if M == 1:
            assert err == 0.0, f"{M}x{K}x{N} ({path}): the small-M path is not in the fast order"
        W.free()
