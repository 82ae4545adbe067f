"""The MFMA path for near-dense W (csrc/tcsc_mfma.hip).

Plans of W with density >= 0.055 also hold W as bf16, and launches with
M >= 5 where the per-launch cost model picks it run Y = [h|m|l] . [W;W;W]
on the matrix cores (x = h + m + l split exactly into bf16 parts).  At the
small shapes most tests use the cost model prefers the gather, so they force
the path (TCSC_PATH=mfma) and check the launch took it; grids of few
128 x 128 tiles split K (whole 64-k blocks per slice, slabs added in slice
order).  Same bars as the gather:
float outputs within 2^-20 * (|b| + sum|x|) of the exact fp64 sums, integer
inputs bit-exact with the reference's outputs for all five variants, and
the rows the split cannot carry (inf / NaN / tiny x) recomputed in the
gather's own order: bit-identical to the gather path.
"""
import os

import numpy as np
import pytest

import pyoracle
import tcsc_amd
from conftest import GOLDEN_NAMES, load_golden, tcsc_of

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


@pytest.fixture
def path(monkeypatch):
    """path(mode): TCSC_PATH for plans created from now on (host-API cache
    dropped).  The host API runs in its fast mode here (TCSC_HOST_FAST=1), so
    its calls take the MFMA path as the device API's do; its default exact
    mode never does (tests/test_host_exact.py)."""
    monkeypatch.setenv("TCSC_HOST_FAST", "1")

    def set_mode(mode):
        if mode is None:
            monkeypatch.delenv("TCSC_PATH", raising=False)
        else:
            monkeypatch.setenv("TCSC_PATH", mode)
        tcsc_amd.cache_clear()

    yield set_mode
    monkeypatch.delenv("TCSC_PATH", raising=False)
    monkeypatch.delenv("TCSC_HOST_FAST", raising=False)
    tcsc_amd.cache_clear()


def device_run(W, X, B, variant, a=0.2, ldy=None, c0=0, c1=None, prepared=False):
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
    info = plan.info()
    info["launch"] = plan.launch_info(M)
    plan.destroy()
    Y = dY.cpu().numpy()
    assert np.all(Y[:, nc:] == 7.0), "columns beyond the plan's were written"
    return Y[:, :nc], info


def float_case(o, M, K, N, density, seed):
    Wd = o.ternary((K, N), density, seed)
    return Wd, o.uniform((M, K), seed + 1), o.uniform((N,), seed + 2)


@pytest.mark.parametrize("K", [700, 701])
def test_float_within_bound_all_variants(gpu, oracle, path, K):
    path("mfma")
    Wd, X, B = float_case(oracle, 200, K, 300, 0.5, 31)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, Wref, B)
    for variant in pyoracle.VARIANTS:
        Y, info = device_run(W, X, B, variant)
        assert info["launch"] == ("mfma", 1)
        ok, ratio = pyoracle.check_close(Y, Y64, S64, 0.2 if variant in pyoracle.PRELU_VARIANTS else None)
        assert ok, f"{variant}: worst err/bound {ratio:.3g}"
    W.free()


def test_integer_inputs_bit_exact(gpu, oracle, path):
    path("mfma")
    M, K, N = 130, 512, 257
    Wd = oracle.ternary((K, N), 0.5, 41)
    X, B = oracle.integers((M, K), 42), oracle.integers((N,), 43)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for variant in pyoracle.VARIANTS:
        Y, info = device_run(W, X, B, variant)
        assert info["launch"][0] == "mfma"
        ref = oracle.sgemm(variant, X, Wref, B, 0.2)
        np.testing.assert_array_equal(Y, ref, err_msg=variant)
        Yh = tcsc_amd.sgemm(variant, X, W, B, 0.2)  # host API: the cached plan takes the same path
        np.testing.assert_array_equal(Yh, ref, err_msg=variant)
    W.free()


@pytest.mark.parametrize("K", [40, 130, 333])
def test_big_tiles_ragged_shapes_integer_exact(gpu, oracle, path, K):
    """The large tiles (128 x 512, for grids of >= 128 256 x 256 tiles): M = 2050
    leaves a short last band of row tiles in the XCD tile order and a ragged
    last tile, N = 4000 a ragged last column tile; K = 40 is one 64-k block
    (the DMA tail clamps from the first sub-step), 130 an odd block count, 333
    a ragged last block.  The path is forced: an automatic plan skips the
    image below 64 rows of W."""
    path("mfma")
    M, N = 2050, 4000
    Wd = oracle.ternary((K, N), 0.5, 91 + K)
    X, B = oracle.integers((M, K), 92 + K), oracle.integers((N,), 93 + K)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for variant in ("basic", "prelu_basic"):
        Y, info = device_run(W, X, B, variant)
        assert info["mfma_min_M"] == 1
        np.testing.assert_array_equal(Y, oracle.sgemm(variant, X, Wref, B, 0.2), err_msg=variant)
    W.free()


def test_special_rows_match_the_gather_bit_for_bit(gpu, oracle, path, monkeypatch):
    monkeypatch.setenv("TCSC_SLICES", "1")  # the gather without split-K: one accumulator per output
    M, K, N = 96, 256, 200
    Wd, X, B = float_case(oracle, M, K, N, 0.4, 51)
    X[3, 17] = np.inf
    X[10, 0] = -np.inf
    X[20, 100] = np.nan
    X[30, 5] = np.float32(1e-40)   # fp32 denormal
    X[31, 6] = np.float32(3e-35)   # normal, below 2^-100
    X[40, :] = np.float32(1e-38)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    for variant in pyoracle.VARIANTS:
        path("mfma")
        Ym, info = device_run(W, X, B, variant)
        assert info["launch"][0] == "mfma"
        path("gather")
        Yg, info = device_run(W, X, B, variant)
        assert info["mfma_min_M"] == 0
        flagged = [3, 10, 20, 30, 31, 40]
        a_, b_ = Ym[flagged], Yg[flagged]
        nan = np.isnan(b_)
        assert nan.any() and np.array_equal(np.isnan(a_), nan), variant
        np.testing.assert_array_equal(a_[~nan].view(np.uint32), b_[~nan].view(np.uint32), err_msg=variant)
        rest = np.setdiff1d(np.arange(M), flagged)
        assert np.isfinite(Ym[rest]).all()
        Y64, S64 = oracle.f64_rows(X[rest], oracle.tcsc_from_dense(Wd), B)
        ok, ratio = pyoracle.check_close(Ym[rest], Y64, S64, 0.2 if variant in pyoracle.PRELU_VARIANTS else None)
        assert ok, f"{variant}: worst err/bound {ratio:.3g}"
    W.free()


def test_path_modes_and_small_M(gpu, oracle, path):
    Wd, X, B = float_case(oracle, 100, 300, 128, 0.05, 61)  # sparse: auto builds no MFMA image
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    path(None)
    assert device_run(W, X, B, "basic")[1]["mfma_min_M"] == 0
    path("mfma")  # forced: any density, any M
    for M in (1, 5, 100):
        Y, info = device_run(W, X[:M], B, "prelu_onthego")
        assert info["mfma_min_M"] == 1
        Y64, S64 = oracle.f64_rows(X[:M], Wref, B)
        assert pyoracle.check_close(Y, Y64, S64, 0.2)[0]
    W.free()
    # dense W, M below the threshold (M <= 4): the small-M path serves it
    path(None)
    Wd2, X2, B2 = float_case(oracle, 4, 300, 128, 0.6, 62)
    W2 = tcsc_amd.TcscMatrix.from_dense(Wd2)
    Y, info = device_run(W2, X2, B2, "basic")
    assert info["mfma_min_M"] == 5 and info["launch"][0] == "small"
    Y64, S64 = oracle.f64_rows(X2, oracle.tcsc_from_dense(Wd2), B2)
    assert pyoracle.check_close(Y, Y64, S64)[0]
    W2.free()


def test_column_block_pitch_and_prepared(gpu, oracle, path):
    path("mfma")
    Wd, X, B = float_case(oracle, 256, 512, 400, 0.5, 71)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, Wref, B)
    for c0, c1, ldy in ((0, 400, 403), (96, 333, 240), (250, 400, 150)):
        for prepared in (False, True):
            Y, info = device_run(W, X, B, "prelu_separate", c0=c0, c1=c1, ldy=ldy, prepared=prepared)
            assert info["launch"][0] == "mfma"
            ok, ratio = pyoracle.check_close(Y, Y64[:, c0:c1], S64[:, c0:c1], 0.2)
            assert ok, f"[{c0},{c1}) ldy={ldy} prepared={prepared}: {ratio:.3g}"
    W.free()


def test_repeated_rows_in_a_column(gpu, oracle, path):
    """A hand-built TCSC whose columns repeat rows (within a sign and across
    signs): every entry counts, as in the reference's loops (tcsc.c:86-93)."""
    path("mfma")
    K, N, M = 80, 70, 100
    rng = np.random.default_rng(5)
    cols_p, cols_n = [], []
    for j in range(N):
        p = np.sort(rng.integers(0, K, 40))  # repeats likely
        n = np.sort(rng.integers(0, K, 30))
        cols_p.append(p)
        cols_n.append(n)
    csp = np.concatenate([[0], np.cumsum([len(c) for c in cols_p])]).astype(np.int32)
    csn = np.concatenate([[0], np.cumsum([len(c) for c in cols_n])]).astype(np.int32)
    rip = np.concatenate(cols_p).astype(np.int32)
    rin = np.concatenate(cols_n).astype(np.int32)
    W = tcsc_amd.TcscMatrix.from_arrays(K, N, csp, csn, rip, rin)
    Wref = pyoracle.TCSC(K, N, csp, csn, rip, rin)
    X, B = oracle.integers((M, K), 81), oracle.integers((N,), 82)
    Y, info = device_run(W, X, B, "basic")
    assert info["launch"][0] == "mfma"
    np.testing.assert_array_equal(Y, oracle.sgemm("basic", X, Wref, B))
    W.free()


@pytest.mark.config_parity
def test_baseline_cfg5_sampled_rows(gpu, oracle, path):
    """BASELINE cfg 5 (M=2048, K=N=8192, 50 %) through the device API takes
    the MFMA path; sampled rows against the exact fp64 sums."""
    import torch

    from tcsc_amd import workloads

    path(None)
    cfg = workloads.CONFIGS[5]
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    K, N = cfg.K, cfg.N
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
    del inp["Wd"]
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    assert plan.info()["mfma_min_M"] == 5
    Y = torch.empty((cfg.M, N), device=dev)
    plan.sgemm(inp["X"], inp["B"], Y, cfg.M, N, "basic", 0.2)
    torch.cuda.synchronize()
    rows = np.unique(np.concatenate([[0, cfg.M - 1], np.random.default_rng(5).integers(0, cfg.M, 6)]))
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(), rin[:nneg].cpu().numpy())
    Y64, S64 = oracle.f64_rows(inp["X"][torch.from_numpy(rows).to(dev)].cpu().numpy(), W, inp["B"].cpu().numpy())
    ok, ratio = pyoracle.check_close(Y[torch.from_numpy(rows).to(dev)].cpu().numpy(), Y64, S64)
    assert ok, f"worst err/bound {ratio:.3g}"
    plan.destroy()


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_golden_fixtures_forced_mfma(gpu, oracle, path, name):
    """Every golden fixture (made by the reference's own tcsc.c) through the
    MFMA path (TCSC_PATH=mfma: any density, any M): integer fixtures bit for
    bit, float fixtures within the bound, the specials fixture with the same
    NaN / inf classification (its rows go through the fixup)."""
    path("mfma")
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    kind, a = g["meta"]["kind"], float(g["a"])
    for variant in pyoracle.VARIANTS:
        Y = tcsc_amd.sgemm(variant, g["X"], W, g["B"], a)
        ref = g["Y_" + variant]
        if kind == "int":
            np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32), err_msg=variant)
        elif kind == "special":
            assert np.array_equal(np.isnan(Y), np.isnan(ref)), variant
            assert np.array_equal(np.isinf(Y), np.isinf(ref)), variant
            fin = np.isfinite(ref)
            np.testing.assert_allclose(Y[fin], ref[fin], rtol=0, atol=1e-5)
        else:
            Y64, S64 = oracle.f64_rows(g["X"], tcsc_of(g), g["B"])
            ok, ratio = pyoracle.check_close(Y, Y64, S64, a if variant in pyoracle.PRELU_VARIANTS else None)
            assert ok, f"{variant}: worst err/bound {ratio:.3g}"
    W.free()


SPLIT_CASES = [  # (M, K, N): grids of few tiles, so K is split
    (64, 4096, 300),    # 64 x 256 tiles (M <= 64), 2 of them: 8 slices of 8 blocks
    (256, 4096, 300),   # 128 x 128 tiles, 6: 8 slices
    (100, 2050, 1000),  # 8 tiles: 4 slices of 9, 9, 9, 6 blocks (a ragged last block)
    (130, 1024, 257),   # 9 tiles, ragged row and column tiles: 2 slices
    (33, 2050, 700),    # 64 x 256 tiles, 3, a ragged row tile: 4 slices
]


@pytest.mark.parametrize("case", range(len(SPLIT_CASES)))
def test_split_k_integer_exact_all_variants(gpu, oracle, path, case):
    """Split K (k_gemm3 PARTIAL + k_reduce4): integer inputs stay exact, so
    every variant equals the reference's outputs bit for bit, and the host
    API's cached plan (fast mode) takes the same split."""
    path("mfma")
    M, K, N = SPLIT_CASES[case]
    Wd = oracle.ternary((K, N), 0.5, 700 + case)
    X, B = oracle.integers((M, K), 710 + case), oracle.integers((N,), 720 + case)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for variant in pyoracle.VARIANTS:
        Y, info = device_run(W, X, B, variant)
        assert info["launch"][0] == "mfma" and info["launch"][1] > 1, info["launch"]
        ref = oracle.sgemm(variant, X, Wref, B, 0.2)
        np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32), err_msg=variant)
    Yh = tcsc_amd.sgemm("prelu_onthego", X, W, B, 0.2)
    np.testing.assert_array_equal(Yh, oracle.sgemm("prelu_onthego", X, Wref, B, 0.2))
    W.free()


@pytest.mark.parametrize("M", [5, 17, 64])
def test_narrow_tiles_unsplit_and_split_integer_exact(gpu, oracle, path, monkeypatch, M):
    """M <= 64 runs 64 x 256 tiles; unsplit ($TCSC_MFMA_WGS=0) and split,
    integer inputs bit for bit against the reference's outputs (ragged N)."""
    path("mfma")
    K, N = 1500, 520
    Wd = oracle.ternary((K, N), 0.4, 780 + M)
    X, B = oracle.integers((M, K), 781 + M), oracle.integers((N,), 782 + M)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    for wgs, split in (("0", False), (None, True)):
        if wgs is None:
            monkeypatch.delenv("TCSC_MFMA_WGS", raising=False)
        else:
            monkeypatch.setenv("TCSC_MFMA_WGS", wgs)
        for variant in ("basic", "prelu_separate"):
            Y, info = device_run(W, X, B, variant)
            assert info["launch"][0] == "mfma" and (info["launch"][1] > 1) == split, info["launch"]
            ref = oracle.sgemm(variant, X, Wref, B, 0.2)
            np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32), err_msg=f"{variant} wgs={wgs}")
    W.free()


def test_split_k_big_tiles_sampled_rows_integer_exact(gpu, oracle, path):
    """The large tiles (128 x 512) on a grid of 128 of them (M = 1024,
    N = 8192: half the CUs) split K in 2 (9 + 9 blocks); integer inputs,
    sampled rows bit for bit against the reference's outputs."""
    path("mfma")
    M, K, N = 1024, 1100, 8192
    Wd = oracle.ternary((K, N), 0.5, 761)
    X, B = oracle.integers((M, K), 762), oracle.integers((N,), 763)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    rows = np.unique(np.concatenate([[0, 127, 128, M - 1], np.random.default_rng(7).integers(0, M, 12)]))
    for variant in ("basic", "prelu_onthego"):
        Y, info = device_run(W, X, B, variant)
        assert info["launch"] == ("mfma", 2), info["launch"]
        ref = oracle.sgemm(variant, X[rows], Wref, B, 0.2)
        np.testing.assert_array_equal(Y[rows].view(np.uint32), ref.view(np.uint32), err_msg=variant)
    W.free()


@pytest.mark.parametrize("M", [96, 40])
def test_split_k_float_blocks_pitch_prepared(gpu, oracle, path, monkeypatch, M):
    """Float inputs through the split GEMM (128 x 128 tiles at M = 96, 64 x 256
    at M = 40): column blocks (N % 4 != 0 takes k_reduce's scalar form), a row
    pitch past N, prepare_x + sgemm_prepared; within the fp32 bound, and the
    unsplit GEMM ($TCSC_MFMA_WGS=0) too."""
    path("mfma")
    K, N = 3000, 600
    Wd, X, B = float_case(oracle, M, K, N, 0.4, 731)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, oracle.tcsc_from_dense(Wd), B)
    for wgs in (None, "0"):
        if wgs is None:
            monkeypatch.delenv("TCSC_MFMA_WGS", raising=False)
        else:
            monkeypatch.setenv("TCSC_MFMA_WGS", wgs)
        for c0, c1, ldy in ((0, 600, 600), (3, 570, 571), (100, 229, 140)):
            for prepared in (False, True):
                Y, info = device_run(W, X, B, "prelu_basic", c0=c0, c1=c1, ldy=ldy, prepared=prepared)
                assert info["launch"][0] == "mfma"
                assert (info["launch"][1] > 1) == (wgs is None), info["launch"]
                ok, ratio = pyoracle.check_close(Y, Y64[:, c0:c1], S64[:, c0:c1], 0.2)
                assert ok, f"[{c0},{c1}) ldy={ldy} prepared={prepared} wgs={wgs}: {ratio:.3g}"
    W.free()


@pytest.mark.parametrize("N", [200, 203])
def test_split_k_special_rows_match_the_gather(gpu, oracle, path, monkeypatch, N):
    """Rows the bf16 split cannot carry are written exactly by the split's
    reduce (k_reduce_fix, the fixup folded in; 4 columns per thread at
    N = 200, one at 203): bit-identical to the unsplit gather."""
    monkeypatch.setenv("TCSC_SLICES", "1")
    M, K = 70, 2048
    Wd, X, B = float_case(oracle, M, K, N, 0.3, 741)
    X[5, 1000] = np.inf
    X[6, 7] = np.nan
    X[60, 2047] = np.float32(1e-39)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    path("mfma")
    Ym, info = device_run(W, X, B, "prelu_onthego")
    assert info["launch"][0] == "mfma" and info["launch"][1] > 1
    path("gather")
    Yg, _ = device_run(W, X, B, "prelu_onthego")
    flagged = [5, 6, 60]
    nan = np.isnan(Yg[flagged])
    assert np.array_equal(np.isnan(Ym[flagged]), nan)
    np.testing.assert_array_equal(Ym[flagged][~nan].view(np.uint32), Yg[flagged][~nan].view(np.uint32))
    rest = np.setdiff1d(np.arange(M), flagged)
    Y64, S64 = oracle.f64_rows(X[rest], oracle.tcsc_from_dense(Wd), B)
    assert pyoracle.check_close(Ym[rest], Y64, S64, 0.2)[0]
    W.free()


@pytest.mark.parametrize("axis", ["cols", "rows"])
def test_host_fast_mode_small_m_shards(gpu, oracle, path, monkeypatch, axis):
    """The host API in fast mode ($TCSC_HOST_FAST=1) at M = 40 over 3 blocks
    of either axis (the cost model sends each block to the GEMM's 64 x 256
    tiles with K split); within the fp32 bound.  The default exact mode gives gemm_basic's
    bits on the same call."""
    path(None)
    monkeypatch.setenv("TCSC_SHARD_AXIS", axis)
    M, K, N = 40, 2048, 900
    Wd, X, B = float_case(oracle, M, K, N, 0.3, 771)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Y64, S64 = oracle.f64_rows(X, oracle.tcsc_from_dense(Wd), B)
    tcsc_amd.set_num_shards(3)
    try:
        Y = tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2)
        ok, ratio = pyoracle.check_close(Y, Y64, S64, 0.2)
        assert ok, ratio
        monkeypatch.delenv("TCSC_HOST_FAST")
        Ye = tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2)
        want = pyoracle.prelu(oracle.gemm_basic(X, Wd, B), 0.2)
        np.testing.assert_array_equal(Ye.view(np.uint32), want.view(np.uint32))
    finally:
        tcsc_amd.set_num_shards(0)
    W.free()


def test_cost_model_takes_the_split_gemm(gpu, oracle, path):
    """Default plan, M = 256, K = N = 2048 at 50 %: the cost model prefers the
    split GEMM (4 slices) to the gather; within the bound."""
    path(None)
    M, K, N = 256, 2048, 2048
    Wd, X, B = float_case(oracle, M, K, N, 0.5, 751)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Y, info = device_run(W, X, B, "basic")
    assert info["mfma_min_M"] == 5 and info["launch"] == ("mfma", 4), info["launch"]
    rows = np.arange(0, M, 17)
    Y64, S64 = oracle.f64_rows(X[rows], oracle.tcsc_from_dense(Wd), B)
    ok, ratio = pyoracle.check_close(Y[rows], Y64, S64)
    assert ok, ratio
    W.free()


def test_reference_order_never_takes_the_mfma_path(gpu, oracle, path):
    """TCSC_ORDER_REFERENCE plans keep the gather (the reference's order is a
    sequence of fp32 adds a GEMM cannot reproduce): a near-dense W with
    M >= 5 stays bit-identical to the oracle's restatement of tcsc.c."""
    path(None)
    Wd, X, B = float_case(oracle, 128, 300, 96, 0.5, 101)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    tcsc_amd.set_order("reference")
    tcsc_amd.cache_clear()
    try:
        for variant in pyoracle.VARIANTS:
            Y, info = device_run(W, X, B, variant)
            assert info["mfma_min_M"] == 0 and info["order"] == 1
            ref = oracle.sgemm(variant, X, Wref, B, 0.2)
            np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32), err_msg=variant)
    finally:
        tcsc_amd.set_order("fast")
        tcsc_amd.cache_clear()
    W.free()
