"""Parity of the gfx950 HIP path with the oracle / the reference's own
outputs, called through the C ABI (libtcsc_amd.so).

Bars:
  * TCSC index arrays: bit-exact with tcsc_from_dense (tcsc.c:6-66).
  * Integer-valued X: every fp32 partial sum is exact, so the outputs must
    equal the reference's Y bit for bit, for all 5 variants.
  * Float X: |y - y64| <= 2^-20 * (|b| + sum |x|) per element (pyoracle.TOL_REL),
    PReLU outputs with the bound scaled by max(1, a).
  * NaN / inf / signed-zero fixture: same classification as the reference.
Full BASELINE sizes are checked on sampled rows against the exact fp64
oracle, plus size-independent properties (linearity, shard concatenation).
"""
import os

import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_NAMES, load_golden, tcsc_of

import tcsc_amd
from tcsc_amd import workloads
from tcsc_amd.shard import all_ranges

pytestmark = pytest.mark.gpu

EXACT_KINDS = ("int",)


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available()
    return torch


def check_variant(g, variant, Y, oracle):
    """Assert parity of a GPU output with the golden reference output."""
    ref = g["Y_" + variant]
    kind = g["meta"]["kind"]
    a = float(g["a"])
    if kind in EXACT_KINDS:
        np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32), err_msg=variant)
        return
    if kind == "special":
        assert np.array_equal(np.isnan(Y), np.isnan(ref)), variant
        assert np.array_equal(np.isinf(Y), np.isinf(ref)), variant
        fin = np.isfinite(ref)
        np.testing.assert_allclose(Y[fin], ref[fin], rtol=0, atol=1e-5)
        return
    Y64, S64 = oracle.f64_rows(g["X"], tcsc_of(g), g["B"])
    ok, ratio = pyoracle.check_close(Y, Y64, S64, a if variant in pyoracle.PRELU_VARIANTS else None)
    assert ok, f"{variant}: worst err/bound = {ratio:.3g}"


@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_host_api_all_variants(gpu, oracle, name):
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    for variant in pyoracle.VARIANTS:
        Y = tcsc_amd.sgemm(variant, g["X"], W, g["B"], float(g["a"]))
        check_variant(g, variant, Y, oracle)
    W.free()


@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_gpu_tcsc_from_dense_bitexact(gpu, name, monkeypatch):
    monkeypatch.setenv("TCSC_BUILDER", "gpu")
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    for a, b in zip(W.arrays(), tcsc_of(g).arrays()):
        np.testing.assert_array_equal(a, b)
    W.free()


def test_device_api_matches_host_api(gpu, torch_cuda, oracle, monkeypatch):
    """The device API's gather with K unsplit equals the host API's exact mode
    (at cfg 1's shape and 10 % density the cost model would otherwise take
    the MFMA path, which sums in its own order)."""
    monkeypatch.setenv("TCSC_SLICES", "1")
    monkeypatch.setenv("TCSC_PATH", "gather")
    torch = torch_cuda
    g = load_golden("cfg1")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    dev = torch.device("cuda:0")
    X = torch.from_numpy(g["X"]).to(dev)
    B = torch.from_numpy(g["B"]).to(dev)
    M, N = g["X"].shape[0], W.cols
    stream = torch.cuda.current_stream().cuda_stream
    plan = tcsc_amd.Plan(W, 0, N, 0, stream)
    plan.reserve(M)  # same split-K choice as the host API
    for variant in pyoracle.VARIANTS:
        Yd = torch.full((M, N + 7), 123.0, device=dev)  # ldy > N: padding untouched
        plan.sgemm(X, B, Yd, M, N + 7, variant, float(g["a"]), stream)
        torch.cuda.synchronize()
        Yh = tcsc_amd.sgemm(variant, g["X"], W, g["B"], float(g["a"]))
        out = Yd.cpu().numpy()
        np.testing.assert_array_equal(out[:, :N], Yh)
        assert np.all(out[:, N:] == 123.0)
    plan.destroy()


@pytest.mark.config_parity
@pytest.mark.parametrize("name", ["cfg1", "cfg1_int", "edge_k_not_mult4", "edge_ragged_n65", "edge_m1"])
def test_dense_baseline_matches_reference(gpu, torch_cuda, oracle, name):
    """the dense GPU baseline (rocBLAS fp32 + bias/PReLU
    epilogue) against the reference outputs: bit-exact on integer inputs,
    the fp32 bound on float inputs; ldy > N padding untouched."""
    torch = torch_cuda
    g = load_golden(name)
    dev = torch.device("cuda:0")
    M, K = g["X"].shape
    N = g["Wd"].shape[1]
    X = torch.from_numpy(np.ascontiguousarray(g["X"])).to(dev)
    Wd = torch.from_numpy(np.ascontiguousarray(g["Wd"].astype(np.float32))).to(dev)
    B = torch.from_numpy(g["B"]).to(dev)
    for variant in ("basic", "prelu_basic"):
        Y = torch.full((M, N + 3), 7.0, device=dev)
        tcsc_amd.dense_sgemm(X, Wd, B, Y, M, N, K, N + 3, variant, float(g["a"]),
                             torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        out = Y.cpu().numpy()
        assert np.all(out[:, N:] == 7.0)
        check_variant(g, variant, np.ascontiguousarray(out[:, :N]), oracle)


@pytest.mark.parametrize("path", ["gather", "mfma"])
@pytest.mark.parametrize("name", ["cfg1", "edge_k_not_mult4", "edge_long_k"])
def test_prepare_then_gather_equals_sgemm(gpu, torch_cuda, monkeypatch, name, path):
    """tcsc_gpu_prepare_x + tcsc_gpu_sgemm_prepared == tcsc_gpu_sgemm, bit for
    bit, and one staged X^T (or X3, on the MFMA path) serves several launches."""
    monkeypatch.setenv("TCSC_PATH", path)
    torch = torch_cuda
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    dev = torch.device("cuda:0")
    X = torch.from_numpy(np.ascontiguousarray(g["X"])).to(dev)
    B = torch.from_numpy(g["B"]).to(dev)
    M, N = g["X"].shape[0], W.cols
    stream = torch.cuda.current_stream().cuda_stream
    plan = tcsc_amd.Plan(W, 0, N, 0, stream)
    plan.reserve(M)
    assert plan.launch_info(M)[0] == (path if path == "mfma" or M > 4 else "small")
    Y1 = torch.empty((M, N), device=dev)
    plan.sgemm(X, B, Y1, M, N, "prelu_basic", 0.2, stream)
    plan.prepare_x(X, M, stream)
    variants = ("prelu_basic", "basic")
    Y2 = {v: torch.empty((M, N), device=dev) for v in variants}
    for v in variants:  # one staging, several gathers
        plan.sgemm_prepared(B, Y2[v], M, N, v, 0.2, stream)
    for v in variants:
        Y3 = torch.empty((M, N), device=dev)
        plan.sgemm(X, B, Y3, M, N, v, 0.2, stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(Y2[v].cpu().numpy(), Y3.cpu().numpy())
    torch.cuda.synchronize()
    plan.destroy()


@pytest.mark.parametrize("axis", ["rows", "cols"])
@pytest.mark.parametrize("shards", [2, 3, 5])
def test_multi_shard_host_path_equals_single(gpu, oracle, shards, axis, monkeypatch):
    """The host API's blocks (one per GPU on a node; several per device here)
    concatenate to the single-block result bit for bit: column blocks
    (TCSC_SHARD_AXIS=cols, the default) and row blocks, with the default
    environment.  Row blocks of a few rows take the small-M path and the
    single block the gather; the host API's exact mode keeps K
    unsplit on both, so both sum in gemm_basic's order and the bits cannot
    depend on the shard count or axis.  Both equal the dense
    oracle's gemm_basic + PReLU bit for bit."""
    for k in ("TCSC_PATH", "TCSC_SLICES", "TCSC_HOST_FAST"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("TCSC_SHARD_AXIS", axis)
    g = load_golden("grid_m16_k512_n1024_nz8")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    tcsc_amd.set_num_shards(1)
    Y1 = tcsc_amd.sgemm("prelu_onthego", g["X"], W, g["B"], 0.2)
    tcsc_amd.set_num_shards(shards)
    try:
        Ys = tcsc_amd.sgemm("prelu_onthego", g["X"], W, g["B"], 0.2)
    finally:
        tcsc_amd.set_num_shards(0)
    np.testing.assert_array_equal(Ys.view(np.uint32), Y1.view(np.uint32))
    want = pyoracle.prelu(oracle.gemm_basic(g["X"], g["Wd"].astype(np.float32), g["B"]), 0.2)
    np.testing.assert_array_equal(Y1.view(np.uint32), want.view(np.uint32))
    W.free()


@pytest.mark.parametrize("axis", ["rows", "cols"])
def test_multi_shard_host_path_large(gpu, oracle, axis, monkeypatch):
    """Row blocks of a launch-sized problem (each block its own launch on the
    same plan) against the exact sums, and against one block on integers."""
    monkeypatch.setenv("TCSC_SHARD_AXIS", axis)
    M, K, N = 1000, 1500, 700
    Wd = oracle.ternary((K, N), 0.05, 91)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    Wref = oracle.tcsc_from_dense(Wd)
    X, B = oracle.uniform((M, K), 92), oracle.uniform((N,), 93)
    Xi, Bi = oracle.integers((M, K), 94), oracle.integers((N,), 95)
    tcsc_amd.set_num_shards(3)
    try:
        Y = tcsc_amd.sgemm("basic", X, W, B)
        Yi = tcsc_amd.sgemm("prelu_basic", Xi, W, Bi, 0.2)
    finally:
        tcsc_amd.set_num_shards(0)
    Y64, S64 = oracle.f64_rows(X, Wref, B)
    ok, ratio = pyoracle.check_close(Y, Y64, S64)
    assert ok, f"worst err/bound {ratio:.3g}"
    np.testing.assert_array_equal(Yi, oracle.sgemm("prelu_basic", Xi, Wref, Bi, 0.2))
    W.free()


@pytest.mark.parametrize("host_fast", ["0", "1"])
@pytest.mark.parametrize("M,K,N,bands", [(1024, 1500, 700, 4), (1100, 700, 300, 3), (2000, 2600, 96, 8)])
def test_host_bands_bit_identical(gpu, torch_cuda, oracle, M, K, N, bands, host_fast, monkeypatch):
    """The host API's copy/compute pipeline (row bands over three streams,
    TCSC_HOST_BANDS) gives the bits of one device launch, ragged last band
    included: in the host API's exact mode (host_fast 0) the device launch
    with K unsplit, in its fast mode the device launch with the cost model's
    split-K (N=96: few column blocks, so K is split)."""
    monkeypatch.setenv("TCSC_HOST_FAST", host_fast)
    if host_fast == "0":
        monkeypatch.setenv("TCSC_SLICES", "1")
    tcsc_amd.cache_clear()
    torch = torch_cuda
    Wd = oracle.ternary((K, N), 0.05, 700 + M)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    X, B = oracle.uniform((M, K), 701 + M), oracle.uniform((N,), 702 + M)
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream().cuda_stream
    plan = tcsc_amd.Plan(W, 0, N, 0, stream)
    plan.reserve(M)
    dX, dB = torch.from_numpy(X).to(dev), torch.from_numpy(B).to(dev)
    monkeypatch.setenv("TCSC_HOST_BANDS", str(bands))
    for variant in pyoracle.VARIANTS:
        Yd = torch.empty((M, N), device=dev)
        plan.sgemm(dX, dB, Yd, M, N, variant, 0.2, stream)
        torch.cuda.synchronize()
        Yh = tcsc_amd.sgemm(variant, X, W, B, 0.2)
        np.testing.assert_array_equal(Yh.view(np.uint32), Yd.cpu().numpy().view(np.uint32), err_msg=variant)
        monkeypatch.setenv("TCSC_HOST_BANDS", "1")  # the unbanded host path, same bits
        np.testing.assert_array_equal(tcsc_amd.sgemm(variant, X, W, B, 0.2).view(np.uint32), Yh.view(np.uint32))
        monkeypatch.setenv("TCSC_HOST_BANDS", str(bands))
    plan.destroy()
    W.free()


def test_device_plan_from_device_arrays_and_gpu_builder(gpu, torch_cuda, oracle):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    X = oracle.uniform((300, 777), 5)
    Wd = oracle.ternary((777, 333), 0.05, 6)
    B = oracle.uniform((333,), 7)
    ref = oracle.tcsc_from_dense(Wd)
    dWd = torch.from_numpy(Wd).to(dev)
    csp = torch.empty(334, dtype=torch.int32, device=dev)
    csn = torch.empty(334, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(dWd, 777, 333, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(dWd, 777, 333, csp, csn, rip, rin)
    assert np.array_equal(csp.cpu().numpy(), ref.col_start_pos)
    assert np.array_equal(rin[:nneg].cpu().numpy(), ref.row_index_neg)
    assert np.array_equal(rip[:npos].cpu().numpy(), ref.row_index_pos)
    # plans over sub-ranges, straight from device arrays
    dX = torch.from_numpy(X).to(dev)
    Y64, S64 = oracle.f64_rows(X, ref, B)
    for c0, c1 in all_ranges(333, 4) + [(10, 11), (0, 333)]:
        plan = tcsc_amd.Plan.from_device(777, 333, csp, csn, rip, rin, c0, c1)
        assert plan.info()["nnz"] == int(ref.col_start_pos[c1] - ref.col_start_pos[c0]
                                         + ref.col_start_neg[c1] - ref.col_start_neg[c0])
        dB = torch.from_numpy(B[c0:c1].copy()).to(dev)
        dY = torch.empty((300, c1 - c0), device=dev)
        plan.sgemm(dX, dB, dY, 300, c1 - c0, "basic", 0.0)
        torch.cuda.synchronize()
        ok, ratio = pyoracle.check_close(dY.cpu().numpy(), Y64[:, c0:c1], S64[:, c0:c1])
        assert ok, (c0, c1, ratio)
        plan.destroy()


def test_shape_mismatch_reports_without_writing(gpu, monkeypatch):
    monkeypatch.setenv("TCSC_ON_ERROR", "continue")
    g = load_golden("cfg1")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    X = np.ones((4, 100), np.float32)  # K != W.rows
    Y = np.full((4, W.cols), 7.0, np.float32)
    with pytest.raises(tcsc_amd.TcscError, match="K=100"):  # the Python mirror checks first
        tcsc_amd.sgemm("basic", X, W, g["B"], 0.2, Y=Y)
    # the C entry point itself (as the reference's harness calls it)
    gpu.tcsc_sgemm_basic(X.reshape(-1), W.ptr, np.ascontiguousarray(g["B"]), Y.reshape(-1), 4, W.cols, 100)
    assert np.all(Y == 7.0)
    assert "shape mismatch" in tcsc_amd.last_error()


def test_zero_sized_calls(gpu, torch_cuda):
    torch = torch_cuda
    W = tcsc_amd.TcscMatrix.from_dense(np.eye(8, dtype=np.float32))
    Y = tcsc_amd.sgemm("basic", np.zeros((0, 8), np.float32), W, np.zeros(8, np.float32))
    assert Y.shape == (0, 8)
    plan = tcsc_amd.Plan(W, 3, 3)
    plan.sgemm(torch.zeros(1, device="cuda"), torch.zeros(1, device="cuda"), torch.zeros(1, device="cuda"),
               5, 0, "basic")
    torch.cuda.synchronize()


# ---------------------------------------------------------------------------
# Full BASELINE sizes (device API, sampled-row exact checks + properties)
# ---------------------------------------------------------------------------
def run_device_cfg(torch, cfg, variant, oracle, x=None):
    """BASELINE config cfg on the device API with W built on the GPU; the
    built arrays are pinned to the oracle's tcsc_from_dense of the same dense
    W first (all four arrays, bit for bit), so a builder error cannot hide
    behind a parity check that feeds the builder's own arrays to the oracle."""
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    if x is not None:
        inp["X"] = x
    K, N = cfg.K, cfg.N
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
    torch.cuda.synchronize()
    pyoracle.assert_builder_matches(oracle, inp.pop("Wd").cpu().numpy(), csp.cpu().numpy(), csn.cpu().numpy(),
                                    rip[:npos].cpu().numpy(), rin[:nneg].cpu().numpy())
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(cfg.M)
    Y = torch.empty((cfg.M, N), device=dev)
    plan.sgemm(inp["X"], inp["B"], Y, cfg.M, N, variant, 0.2)
    torch.cuda.synchronize()
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    return inp, W, Y, plan


@pytest.mark.config_parity
@pytest.mark.parametrize("cfg_idx", [2, 3, 4, 5])
def test_baseline_config_sampled_rows(gpu, torch_cuda, oracle, cfg_idx):
    torch = torch_cuda
    cfg = workloads.CONFIGS[cfg_idx]
    inp, W, Y, plan = run_device_cfg(torch, cfg, cfg.variant, oracle)
    rows = np.unique(np.concatenate([[0, 1, cfg.M - 1], np.random.default_rng(cfg_idx).integers(0, cfg.M, 29)]))
    Xs = inp["X"][torch.from_numpy(rows).to(inp["X"].device)].cpu().numpy()
    B = inp["B"].cpu().numpy()
    Y64, S64 = oracle.f64_rows(Xs, W, B)
    a = 0.2 if cfg.variant in pyoracle.PRELU_VARIANTS else None
    ok, ratio = pyoracle.check_close(Y[torch.from_numpy(rows).to(Y.device)].cpu().numpy(), Y64, S64, a)
    assert ok, f"cfg{cfg_idx}: worst err/bound {ratio:.3g}"
    # integer-valued X at full size: exact, so bit-identical to the oracle
    Xi = torch.randint(-512, 513, (cfg.M, cfg.K), device=inp["X"].device, dtype=torch.int32).float()
    Yi = torch.empty_like(Y)
    plan.sgemm(Xi, inp["B"].round(), Yi, cfg.M, cfg.N, "basic", 0.0)
    torch.cuda.synchronize()
    Xis = Xi[torch.from_numpy(rows).to(Xi.device)].cpu().numpy()
    ref = oracle.sgemm("basic", Xis, W, inp["B"].round().cpu().numpy())
    np.testing.assert_array_equal(Yi[torch.from_numpy(rows).to(Yi.device)].cpu().numpy(), ref)
    # linearity (size-independent): Y(X1 + X2) - b == (Y(X1) - b) + (Y(X2) - b) exactly for integer X
    Yj = torch.empty_like(Y)
    plan.sgemm(Xi * 2, inp["B"].round(), Yj, cfg.M, cfg.N, "basic", 0.0)
    torch.cuda.synchronize()
    b = inp["B"].round()
    assert torch.equal(Yj - b, 2 * (Yi - b))
    plan.destroy()


@pytest.mark.parametrize("slices", [2, 3, 7])
def test_split_k_paths(gpu, torch_cuda, oracle, monkeypatch, slices):
    """k-sliced launches (partial slabs + ordered reduce) against the oracle:
    integer inputs must be bit-identical, float within tolerance."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    M, K, N = 300, 1500, 200
    Wd = oracle.ternary((K, N), 0.05, 21)
    W = oracle.tcsc_from_dense(Wd)
    Wm = tcsc_amd.TcscMatrix.from_dense(Wd)
    plan = tcsc_amd.Plan(Wm)
    monkeypatch.setenv("TCSC_SLICES", str(slices))
    plan.reserve(M)
    Xi = oracle.integers((M, K), 22)
    Bi = oracle.integers((N,), 23)
    for variant in ("basic", "prelu_basic"):
        dY = torch.empty((M, N), device=dev)
        plan.sgemm(torch.from_numpy(Xi).to(dev), torch.from_numpy(Bi).to(dev), dY, M, N, variant, 0.25)
        torch.cuda.synchronize()
        ref = oracle.sgemm(variant, Xi, W, Bi, 0.25)
        np.testing.assert_array_equal(dY.cpu().numpy(), ref)
    X = oracle.uniform((M, K), 24)
    B = oracle.uniform((N,), 25)
    dY = torch.empty((M, N), device=dev)
    plan.sgemm(torch.from_numpy(X).to(dev), torch.from_numpy(B).to(dev), dY, M, N, "prelu_onthego", 0.2)
    torch.cuda.synchronize()
    Y64, S64 = oracle.f64_rows(X, W, B)
    ok, ratio = pyoracle.check_close(dY.cpu().numpy(), Y64, S64, 0.2)
    assert ok, ratio
    # host API with the same forced split
    Yh = tcsc_amd.sgemm("basic", Xi, Wm, Bi)
    np.testing.assert_array_equal(Yh, oracle.sgemm("basic", Xi, W, Bi))
    plan.destroy()


@pytest.mark.parametrize("dist,lines", [("0", "1"), ("1664", "1"), ("768", "8"), ("4000", "8")])
def test_stream_prefetch_settings_do_not_change_bits(gpu, torch_cuda, oracle, monkeypatch, dist, lines):
    """The entry-stream L2 prefetch (TCSC_PF_DIST / TCSC_PF_LINES, clamped to
    the plan's guard window) only touches lines: every setting gives the
    default's bits.  N = 200 leaves idle waves on the empty chain, whose
    prefetch window ends in the guard entries; split-K too."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    M, K, N = 300, 1500, 200
    Wd = oracle.ternary((K, N), 0.05, 31)
    Wm = tcsc_amd.TcscMatrix.from_dense(Wd)
    X = torch.from_numpy(oracle.uniform((M, K), 32)).to(dev)
    B = torch.from_numpy(oracle.uniform((N,), 33)).to(dev)
    for slices in ("1", "3"):
        monkeypatch.setenv("TCSC_SLICES", slices)
        plan = tcsc_amd.Plan(Wm)
        plan.reserve(M)
        monkeypatch.delenv("TCSC_PF_DIST", raising=False)
        monkeypatch.delenv("TCSC_PF_LINES", raising=False)
        Y0 = torch.empty((M, N), device=dev)
        plan.sgemm(X, B, Y0, M, N, "prelu_basic", 0.2)
        monkeypatch.setenv("TCSC_PF_DIST", dist)
        monkeypatch.setenv("TCSC_PF_LINES", lines)
        Y1 = torch.full((M, N), float("nan"), device=dev)
        plan.sgemm(X, B, Y1, M, N, "prelu_basic", 0.2)
        torch.cuda.synchronize()
        assert torch.equal(Y0.view(torch.int32), Y1.view(torch.int32)), (dist, lines, slices)
        plan.destroy()


@pytest.mark.parametrize("axis,shards,bands", [("cols", 2, 3), ("cols", 3, 4), ("rows", 2, 2)])
def test_host_bands_with_blocks_bit_identical(gpu, oracle, axis, shards, bands, monkeypatch):
    """The pinned-staging band pipeline under the host API's blocks: column
    blocks copy each band's Y out with Y's row pitch (the first block stages X
    in bands, the next ones reuse it), row blocks band each block's rows.
    Bits equal the same blocks without the pipeline (TCSC_HOST_BANDS=1: one
    pageable copy each way); within the bound of the exact sums."""
    M, K, N = 1300, 900, 520
    Wd = oracle.ternary((K, N), 0.05, 801)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    X, B = oracle.uniform((M, K), 802), oracle.uniform((N,), 803)
    monkeypatch.setenv("TCSC_SHARD_AXIS", axis)
    tcsc_amd.set_num_shards(shards)
    try:
        monkeypatch.setenv("TCSC_HOST_BANDS", "1")
        Y1 = tcsc_amd.sgemm("prelu_separate", X, W, B, 0.2)
        monkeypatch.setenv("TCSC_HOST_BANDS", str(bands))
        for _ in range(2):  # a second call reuses the pinned slots and the cached plans
            Yh = tcsc_amd.sgemm("prelu_separate", X, W, B, 0.2)
            np.testing.assert_array_equal(Yh.view(np.uint32), Y1.view(np.uint32))
    finally:
        tcsc_amd.set_num_shards(0)
    Y64, S64 = oracle.f64_rows(X, oracle.tcsc_from_dense(Wd), B)
    assert pyoracle.check_close(Yh, Y64, S64, 0.2)[0]
    W.free()


@pytest.mark.config_parity
@pytest.mark.parametrize("rows,cols", [(1, 1), (7, 300), (257, 513), (1000, 64), (17_000_000, 3)])
def test_gpu_from_dense_tiles_bitexact(gpu, torch_cuda, oracle, rows, cols):
    """The tiled device builder (row tiles of 256, taller past 65535 tiles)
    against the reference restatement: ragged tiles, one row, very tall
    matrices, non-ternary values (they count as 0, tcsc.c:14-17)."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(rows * 7 + cols)
    u = torch.rand((rows, cols), generator=g, device=dev)
    d = torch.zeros((rows, cols), device=dev)
    d[u < 0.03] = 1.0
    d[(u >= 0.03) & (u < 0.06)] = -1.0
    d[(u >= 0.06) & (u < 0.07)] = 0.5
    d[(u >= 0.07) & (u < 0.08)] = -1.0000001
    csp = torch.empty(cols + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(cols + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(d, rows, cols, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(d, rows, cols, csp, csn, rip, rin)
    torch.cuda.synchronize()
    dn = d.cpu().numpy()
    if rows * cols <= 1 << 22:
        ref = oracle.tcsc_from_dense(dn)
        ref_arrays = ref.arrays()
    else:  # too tall for the C restatement's int offsets in reasonable time: numpy, column by column
        ref_arrays = []
        for val in (1.0, -1.0):
            starts, idx = [0], []
            for c in range(cols):
                r = np.nonzero(dn[:, c] == val)[0].astype(np.int32)
                idx.append(r)
                starts.append(starts[-1] + r.size)
            ref_arrays.append((np.array(starts, np.int32), np.concatenate(idx)))
        ref_arrays = (ref_arrays[0][0], ref_arrays[1][0], ref_arrays[0][1], ref_arrays[1][1])
    got = (csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(), rin[:nneg].cpu().numpy())
    for a, b in zip(got, ref_arrays):
        np.testing.assert_array_equal(a, b)


def test_gpu_from_dense_fill_never_overruns(gpu, torch_cuda):
    """A matrix changed between the two calls: the fill writes at most the
    entries the first call counted (the caller's arrays are sized from it)."""
    torch = torch_cuda
    dev = torch.device("cuda:0")
    rows, cols = 600, 40
    d = torch.zeros((rows, cols), device=dev)
    d[::7, :] = 1.0
    csp = torch.empty(cols + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(cols + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(d, rows, cols, csp, csn)
    d[:, :] = 1.0  # many more +1 now
    guard = torch.full((npos + 4096,), -7, dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(d, rows, cols, csp, csn, guard[:max(npos, 1)], rin)
    torch.cuda.synchronize()
    assert torch.all(guard[npos:] == -7)


@pytest.mark.config_parity
@pytest.mark.parametrize("axis", ["cols", "rows"])
def test_cfg4_eight_way_shards_full_size(gpu, torch_cuda, oracle, axis):
    """BASELINE cfg 4 split 8 ways on one GPU, each block launched exactly as
    a rank of `bench.py --gpus 8` launches it: a column block
    is its own plan of 2,048 columns over all of X (the per-rank path with the
    cost model's split-K and the ordered reduce), a row block is the full plan
    on 512 rows of X.  Columns are independent (tcsc.c:113) and so are rows,
    so the eight blocks written into one Y must (1) match the fp64 oracle on
    sampled rows of every block, (2) equal the oracle bit for bit on integer X,
    (3) agree with the single launch over the whole matrix within the bound
    (bit for bit where the split is the same)."""
    torch = torch_cuda
    cfg = workloads.CONFIGS[4]
    M, K, N, G = cfg.M, cfg.K, cfg.N, 8
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, N, dev)
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
    torch.cuda.synchronize()
    pyoracle.assert_builder_matches(oracle, inp["Wd"].cpu().numpy(), csp.cpu().numpy(), csn.cpu().numpy(),
                                    rip[:npos].cpu().numpy(), rin[:nneg].cpu().numpy())
    X, B = inp["X"], inp["B"]
    # |b| + sum_{P u Q} |x| per element (the bound's scale): the dense product on magnitudes
    S = torch.empty((M, N), device=dev)
    Xa, Wa, Ba = X.abs(), inp.pop("Wd").abs_(), B.abs()
    tcsc_amd.dense_sgemm(Xa, Wa, Ba, S, M, N, K, N, "basic", 0.0)
    torch.cuda.synchronize()
    del Xa, Wa, Ba
    Xi = torch.randint(-512, 513, (M, K), device=dev, dtype=torch.int32).float()
    Bi = B.round()
    full = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    full.reserve(M)
    Y1, Y1i = torch.empty((M, N), device=dev), torch.empty((M, N), device=dev)
    full.sgemm(X, B, Y1, M, N, cfg.variant, 0.2)
    full.sgemm(Xi, Bi, Y1i, M, N, "basic", 0.0)
    Yg, Ygi = torch.empty((M, N), device=dev), torch.empty((M, N), device=dev)
    for c0, c1 in all_ranges(N if axis == "cols" else M, G):
        if axis == "cols":
            p = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin, c0, c1)
            p.reserve(M)
            p.sgemm(X, B[c0:c1], Yg[:, c0:c1], M, N, cfg.variant, 0.2)
            p.sgemm(Xi, Bi[c0:c1], Ygi[:, c0:c1], M, N, "basic", 0.0)
            p.destroy()
        else:
            full.sgemm(X[c0:c1].contiguous(), B, Yg[c0:c1], c1 - c0, N, cfg.variant, 0.2)
            full.sgemm(Xi[c0:c1].contiguous(), Bi, Ygi[c0:c1], c1 - c0, N, "basic", 0.0)
    torch.cuda.synchronize()
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    # sampled rows: 4 per row block (every column block is in every row)
    rng = np.random.default_rng(48)
    rows = np.unique(np.concatenate([[0, M - 1]] + [r0 + rng.integers(0, r1 - r0, 4)
                                                     for r0, r1 in all_ranges(M, G)]))
    sel = torch.from_numpy(rows).to(dev)
    Y64, S64 = oracle.f64_rows(X[sel].cpu().numpy(), W, B.cpu().numpy())
    ok, ratio = pyoracle.check_close(Yg[sel].cpu().numpy(), Y64, S64, 0.2)
    assert ok, f"cfg4 {axis} x{G}: worst err/bound {ratio:.3g}"
    ref = oracle.sgemm("basic", Xi[sel].cpu().numpy(), W, Bi.cpu().numpy())
    np.testing.assert_array_equal(Ygi[sel].cpu().numpy(), ref)
    # every element: integer X exact (so equal to the single launch), float X
    # within twice the per-element bound of the single launch (PReLU scales by max(1, a) = 1)
    assert torch.equal(Ygi, Y1i)
    bound = S.mul_(2.0 ** -19)
    assert bool(((Yg - Y1).abs() <= bound).all()), f"cfg4 {axis} x{G}: blocks vs single launch out of bound"
    full.destroy()
