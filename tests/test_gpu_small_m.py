"""The small-M path (csrc/tcsc_small.hip): M <= 4 rows whose
X fits the LDS run one lane per output column over the plan's merged CSC
copy instead of the 256-row gather (M = 7 and 16 below check the hand-over
to the gather).  Same bars as the gather: float outputs
within 2^-20 * (|b| + sum|x|) of the exact sums, integer inputs bit-exact
with the reference's outputs for all five variants, NaN/inf classified as
the reference does; the prepared (prepare_x + sgemm_prepared) form and
column blocks with a row pitch agree."""
import numpy as np
import pytest

import pyoracle
import tcsc_amd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


def run(W, X, B, variant, a=0.2, c0=0, c1=None, ldy=None, prepared=False):
    import torch

    dev = torch.device("cuda:0")
    c1 = W.cols if c1 is None else c1
    plan = tcsc_amd.Plan(W, c0, c1)
    M, nc = X.shape[0], c1 - c0
    ldy = ldy or nc
    dX = torch.from_numpy(np.ascontiguousarray(X)).to(dev)
    dB = torch.from_numpy(np.ascontiguousarray(B[c0:c1])).to(dev)
    dY = torch.full((M, ldy), 7.0, device=dev)
    if prepared:
        plan.prepare_x(dX, M)
        plan.sgemm_prepared(dB, dY, M, ldy, variant, a)
    else:
        plan.sgemm(dX, dB, dY, M, ldy, variant, a)
    torch.cuda.synchronize()
    plan.destroy()
    Y = dY.cpu().numpy()
    assert np.all(Y[:, nc:] == 7.0)
    return Y[:, :nc]


@pytest.mark.parametrize("M", [1, 2, 3, 4, 7, 16])
def test_float_within_bound(gpu, oracle, M):
    K, N = 3000, 700
    Wd = oracle.ternary((K, N), 0.1, 200 + M)
    X, B = oracle.uniform((M, K), 300 + M), oracle.uniform((N,), 400 + M)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, Wref, B)
    for variant in pyoracle.VARIANTS:
        Y = run(W, X, B, variant)
        ok, ratio = pyoracle.check_close(Y, Y64, S64, 0.2 if variant in pyoracle.PRELU_VARIANTS else None)
        assert ok, f"M={M} {variant}: worst err/bound {ratio:.3g}"
    W.free()


@pytest.mark.parametrize("M", [1, 4, 16])
def test_integer_bit_exact_and_host_api(gpu, oracle, M):
    K, N = 1024, 300
    Wd = oracle.ternary((K, N), 0.2, 500 + M)
    X, B = oracle.integers((M, K), 600 + M), oracle.integers((N,), 700 + M)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for variant in pyoracle.VARIANTS:
        ref = oracle.sgemm(variant, X, Wref, B, 0.2)
        np.testing.assert_array_equal(run(W, X, B, variant), ref, err_msg=variant)
        np.testing.assert_array_equal(tcsc_amd.sgemm(variant, X, W, B, 0.2), ref, err_msg=variant)
    W.free()


def test_prepared_blocks_and_pitch(gpu, oracle):
    M, K, N = 3, 2000, 500
    Wd = oracle.ternary((K, N), 0.05, 801)
    X, B = oracle.uniform((M, K), 802), oracle.uniform((N,), 803)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, oracle.tcsc_from_dense(Wd), B)
    for c0, c1, ldy in ((0, 500, 500), (37, 400, 371), (480, 500, 33)):
        Ya = run(W, X, B, "prelu_onthego", c0=c0, c1=c1, ldy=ldy)
        Yb = run(W, X, B, "prelu_onthego", c0=c0, c1=c1, ldy=ldy, prepared=True)
        np.testing.assert_array_equal(Ya.view(np.uint32), Yb.view(np.uint32))
        assert pyoracle.check_close(Ya, Y64[:, c0:c1], S64[:, c0:c1], 0.2)[0]
    W.free()


def test_specials_and_off_switch(gpu, oracle, monkeypatch):
    """inf / NaN / -0.0 rows classified as the reference does; with
    TCSC_SMALL_M=0 the gather serves the same call within the bound."""
    M, K, N = 4, 256, 96
    Wd = oracle.ternary((K, N), 0.3, 901)
    X, B = oracle.uniform((M, K), 902), oracle.uniform((N,), 903)
    X[0, 5] = np.inf
    X[1, 9] = np.nan
    X[2, :] = -0.0
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for variant in pyoracle.VARIANTS:
        ref = oracle.sgemm(variant, X, Wref, B, 0.2)
        Y = run(W, X, B, variant)
        assert np.array_equal(np.isnan(Y), np.isnan(ref)), variant
        assert np.array_equal(np.isinf(Y), np.isinf(ref)), variant
        fin = np.isfinite(ref)
        np.testing.assert_allclose(Y[fin], ref[fin], rtol=0, atol=1e-5)
    monkeypatch.setenv("TCSC_SMALL_M", "0")
    Xf = oracle.uniform((M, K), 904)
    Y64, S64 = oracle.f64_rows(Xf, Wref, B)
    assert pyoracle.check_close(run(W, Xf, B, "basic"), Y64, S64)[0]
    W.free()


@pytest.mark.parametrize("K", [1, 5, 4093, 4096])
def test_ragged_k_and_unaligned_x_equal_gather(gpu, oracle, monkeypatch, K):
    """The staging's two forms -- 16-B loads where K % 4 == 0 and X is 16-B
    aligned, 4-B loads otherwise (K = 1, 5, 4093, or X one float off a 16-B
    boundary) -- and the row pair's padding (Kp = K + 1 rounded up to 4): bit
    for bit the gather's fast order with K unsplit."""
    import torch

    dev = torch.device("cuda:0")
    M, N = 2, 200
    Wd = oracle.ternary((K, N), 0.3, 1000 + K)
    X, B = oracle.uniform((M, K), 1100 + K), oracle.uniform((N,), 1200 + K)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    plan = tcsc_amd.Plan(W, 0, N)
    assert plan.launch_info(M)[0] == "small"
    dB = torch.from_numpy(B).to(dev)
    backing = torch.zeros(M * K + 1, device=dev)
    for shift in (0, 1):  # shift 1: X starts 4 B past a 16-B boundary
        dX = backing[shift:shift + M * K].view(M, K)
        dX.copy_(torch.from_numpy(X).to(dev))
        ys = {}
        for small in ("4", "0"):
            monkeypatch.setenv("TCSC_SMALL_M", small)
            monkeypatch.setenv("TCSC_SLICES", "1")
            monkeypatch.setenv("TCSC_PATH", "gather")
            dY = torch.full((M, N), float("nan"), device=dev)
            plan.sgemm(dX, dB, dY, M, N, "prelu_basic", 0.2)
            torch.cuda.synchronize()
            ys[small] = dY.cpu().numpy()
        np.testing.assert_array_equal(ys["4"].view(np.uint32), ys["0"].view(np.uint32),
                                      err_msg=f"K={K} shift={shift}")
    plan.destroy()
    W.free()
