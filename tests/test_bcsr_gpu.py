"""Parity of the gfx950 BCSR path (k_bcsr) with the reference's own outputs,
through the C ABI (libtcsc_amd.so).

Bar: BIT-EXACT for every fixture and variant -- the plan replays the
reference's per-element update sequence (include/sparse/bcsr.h), so even
float inputs match bit for bit.  Exception: NaN payloads (x86 produces the
negative default NaN for inf*0, gfx950 the positive one): where the
reference has a NaN the GPU must have a NaN, every other element is
bit-exact.  Full BASELINE size (cfg4 shape, 1x8 blocks): bit-exact against
the TCSC kernel (same ascending-k order for ternary W) over the whole
matrix, and against the oracle on sampled rows.
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
from conftest import BCSR_GOLDEN_NAMES, ROOT, bcsr_of, load_bcsr_golden

import tcsc_amd
from tcsc_amd import bcsr, workloads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    return tcsc_amd.lib()


@pytest.fixture(scope="module")
def torch_cuda():
    import torch

    assert torch.cuda.is_available()
    return torch


def assert_parity(Y, ref, what):
    Y = np.ascontiguousarray(Y, np.float32)
    ref = np.ascontiguousarray(ref, np.float32)
    assert Y.shape == ref.shape, what
    nan_ref = np.isnan(ref)
    assert np.array_equal(np.isnan(Y), nan_ref), what
    np.testing.assert_array_equal(Y[~nan_ref].view(np.uint32), ref[~nan_ref].view(np.uint32), err_msg=what)


def variants_of(g):
    return [v for v in pyoracle.BCSR_VARIANTS if "Y_" + v in g]


@pytest.mark.config_parity
@pytest.mark.parametrize("name", BCSR_GOLDEN_NAMES)
def test_host_api_all_variants(gpu, name):
    g = load_bcsr_golden(name)
    W = bcsr.BcsrMatrix.from_dense(g["Wd"].astype(np.float32), int(g["r"]), int(g["c"]))
    for v in variants_of(g):
        Y = bcsr.sgemm(v, g["X"], W, g["B"], float(g["a"]))
        assert_parity(Y, g["Y_" + v], f"{name}/{v}")
    W.free()


@pytest.mark.config_parity
@pytest.mark.parametrize("name", ["empty_block_rows_4x8", "m9_k40_n42_2x3", "nonternary_2x8"])
def test_host_api_on_reference_arrays(gpu, name):
    """The reference's own bcsr_from_dense arrays (not ours) through the
    by-value bcsr_t of the drop-in API."""
    g = load_bcsr_golden(name)
    W = bcsr_of(g)
    st = bcsr.struct_from_arrays(W.r, W.c, W.br, W.bc, W.b_row_start, W.b_col_idx, W.b_values)
    for v in variants_of(g):
        assert_parity(bcsr.sgemm(v, g["X"], st, g["B"], float(g["a"])), g["Y_" + v], f"{name}/{v}")


@pytest.mark.parametrize("name", ["m300_k300_n160_1x8", "ragged_m5_k67_n70_3x8", "m20_k64_n64_16x16"])
def test_device_api_matches_host_api(gpu, torch_cuda, name):
    torch = torch_cuda
    g = load_bcsr_golden(name)
    dev = torch.device("cuda:0")
    W = bcsr.BcsrMatrix.from_dense(g["Wd"].astype(np.float32), int(g["r"]), int(g["c"]))
    M, K = g["X"].shape
    N = g["B"].size
    st = torch.cuda.current_stream().cuda_stream
    plan = bcsr.BcsrPlan(W, 0, st)
    plan.reserve(M, K)
    X = torch.from_numpy(np.ascontiguousarray(g["X"])).to(dev)
    B = torch.from_numpy(g["B"]).to(dev)
    for v in variants_of(g):
        Yd = torch.full((M, N + 5), 321.0, device=dev)  # ldy > N: padding untouched
        plan.sgemm(X, B, Yd, M, N, K, N + 5, v, float(g["a"]), st)
        Yp = torch.full((M, N), 7.0, device=dev)
        plan.prepare_x(X, M, K, st)
        plan.sgemm_prepared(B, Yp, M, N, K, N, v, float(g["a"]), st)
        torch.cuda.synchronize()
        out = Yd.cpu().numpy()
        assert np.all(out[:, N:] == 321.0)
        assert_parity(out[:, :N], g["Y_" + v], f"{name}/{v} device")
        np.testing.assert_array_equal(Yp.cpu().numpy(), out[:, :N])
    assert plan.stats()["block_visits"] == W.k
    plan.destroy()
    W.free()


def test_shape_rules_fail_loudly(gpu, monkeypatch):
    """avx variants need c == 8, avx2 r == c == 8 (bcsr.c:250-256, 347-377);
    K and N must cover the blocks; errors report without writing Y."""
    monkeypatch.setenv("TCSC_ON_ERROR", "continue")
    g = load_bcsr_golden("m16_k512_n1024_4x4")
    W = bcsr.BcsrMatrix.from_dense(g["Wd"].astype(np.float32), 4, 4)
    Y = np.full((16, 1024), 5.0, np.float32)
    bcsr.sgemm("avx", g["X"], W, g["B"], Y=Y)
    assert np.all(Y == 5.0) and "8-column blocks" in tcsc_amd.last_error()
    W8 = bcsr.BcsrMatrix.from_dense(g["Wd"].astype(np.float32), 1, 8)
    bcsr.sgemm("avx2", g["X"], W8, g["B"], Y=Y)
    assert np.all(Y == 5.0) and "8x8 blocks" in tcsc_amd.last_error()
    bcsr.sgemm("basic", g["X"][:, :100], W8, g["B"], Y=Y)  # K < br*r
    assert np.all(Y == 5.0) and "shape mismatch" in tcsc_amd.last_error()
    with pytest.raises(tcsc_amd.TcscError):
        plan = bcsr.BcsrPlan(W)
        plan.sgemm(0, 0, 0, 16, 1024, 512, 1024, "avx")
    W.free()
    W8.free()


def test_bcsr_1x8_equals_tcsc_basic(gpu, torch_cuda, oracle, monkeypatch):
    """Ternary W with 1x8 blocks: bcsr_sgemm_basic adds bias first, then
    X[m,k]*w for every k of a stored block in ascending k -- zeros add +-0,
    an exact no-op here -- which is the TCSC kernel's fast order (+1/-1
    merged in ascending k) when K is not split over workgroups
    (TCSC_SLICES=1; this grid is small enough for the cost model to split
    it), except where the bias goes: the TCSC fast order adds it after the
    sum (dense.c's gemm_basic order).  With a zero bias the
    two orders are the same arithmetic: bit-identical outputs.  The bias
    path is cross-checked too: a nonzero integer bias on integer
    X makes every order exact, so bias-first BCSR and bias-last TCSC must
    agree bit for bit (basic); a nonzero float bias on
    float X keeps both within the fp32 bound of the exact sums."""
    monkeypatch.setenv("TCSC_SLICES", "1")
    torch = torch_cuda
    dev = torch.device("cuda:0")
    M, K, N = 700, 2048, 1032
    X = oracle.uniform((M, K), 81)
    Wd = oracle.ternary((K, N), 0.02, 82)
    B = np.zeros((N,), np.float32)
    Wb = bcsr.BcsrMatrix.from_dense(Wd, 1, 8)
    Wt = tcsc_amd.TcscMatrix.from_dense(Wd)
    st = torch.cuda.current_stream().cuda_stream
    pb = bcsr.BcsrPlan(Wb, 0, st)
    pt = tcsc_amd.Plan(Wt, 0, N, 0, st)
    dX, dB = torch.from_numpy(X).to(dev), torch.from_numpy(B).to(dev)
    Yb = torch.empty((M, N), device=dev)
    Yt = torch.empty((M, N), device=dev)
    pb.sgemm(dX, dB, Yb, M, N, K, N, "basic", 0.0, st)
    pt.sgemm(dX, dB, Yt, M, N, "basic", 0.0, st)
    torch.cuda.synchronize()
    assert torch.equal(Yb, Yt)
    Xi, Bi = oracle.integers((M, K), 83), oracle.integers((N,), 84, 64)
    assert np.any(Bi != 0)
    dXi, dBi = torch.from_numpy(Xi).to(dev), torch.from_numpy(Bi).to(dev)
    # basic only: bcsr_sgemm_prelu_basic applies its PReLU to the running
    # value after every block update (bcsr.c:191-215), not once to the sum
    pb.sgemm(dXi, dBi, Yb, M, N, K, N, "basic", 0.0, st)
    pt.sgemm(dXi, dBi, Yt, M, N, "basic", 0.0, st)
    torch.cuda.synchronize()
    assert torch.equal(Yb, Yt)
    Bf = oracle.uniform((N,), 85)
    dBf = torch.from_numpy(Bf).to(dev)
    pb.sgemm(dX, dBf, Yb, M, N, K, N, "basic", 0.0, st)
    pt.sgemm(dX, dBf, Yt, M, N, "basic", 0.0, st)
    torch.cuda.synchronize()
    Y64, S64 = oracle.f64_rows(X, oracle.tcsc_from_dense(Wd), Bf)
    for Y in (Yb, Yt):
        ok, ratio = pyoracle.check_close(Y.cpu().numpy(), Y64, S64)
        assert ok, ratio
    pb.destroy()
    pt.destroy()


def test_baseline_cfg4_shape_1x8(gpu, torch_cuda, oracle, monkeypatch):
    """BASELINE cfg4 (M=4096, K=N=16384, 98 % ternary) as 1x8 BCSR: whole
    output bit-identical to the TCSC kernel's basic result on a zero bias
    (where bias-first BCSR and the bias-last TCSC fast order agree), sampled
    rows bit-identical to the oracle (bcsr_sgemm_basic and prelu_basic order)."""
    monkeypatch.setenv("TCSC_SLICES", "1")
    torch = torch_cuda
    cfg = workloads.CONFIGS[4]
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    Wd = inp.pop("Wd").cpu().numpy()
    Wb = bcsr.BcsrMatrix.from_dense(Wd, 1, 8)
    st = torch.cuda.current_stream().cuda_stream
    pb = bcsr.BcsrPlan(Wb, 0, st)
    X, B = inp["X"], inp["B"]
    M, K, N = cfg.M, cfg.K, cfg.N
    Yb = torch.empty((M, N), device=dev)
    pb.sgemm(X, B, Yb, M, N, K, N, "basic", 0.0, st)
    Wt = tcsc_amd.TcscMatrix.from_dense(Wd)
    del Wd
    pt = tcsc_amd.Plan(Wt, 0, N, 0, st)
    Yt = torch.empty((M, N), device=dev)
    Z = torch.zeros_like(B)  # bias first (BCSR) and last (TCSC fast order) agree on a zero bias
    pt.sgemm(X, Z, Yt, M, N, "basic", 0.0, st)
    Yz = torch.empty_like(Yb)
    pb.sgemm(X, Z, Yz, M, N, K, N, "basic", 0.0, st)
    torch.cuda.synchronize()
    assert torch.equal(Yz, Yt)
    del Yt, Yz
    pt.destroy()
    Wt.free()
    rows = np.array([0, 1, 1234, M - 1])
    rs, ci, vals = Wb.arrays()
    Wo = pyoracle.BCSR(1, 8, K, N // 8, rs, ci, vals)
    Xs = X[torch.from_numpy(rows).to(dev)].cpu().numpy()
    Bh = B.cpu().numpy()
    np.testing.assert_array_equal(Yb[torch.from_numpy(rows).to(dev)].cpu().numpy(),
                                  oracle.bcsr_sgemm("basic", Xs, Wo, Bh))
    pb.sgemm(X, B, Yb, M, N, K, N, "prelu_basic", 0.2, st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(Yb[torch.from_numpy(rows).to(dev)].cpu().numpy(),
                                  oracle.bcsr_sgemm("prelu_basic", Xs, Wo, Bh, 0.2))
    pb.destroy()
    Wb.free()


def test_reference_test_bcsr_links_and_passes(gpu):
    """The reference's own test/test_bcsr.cpp, unmodified, linked against
    libtcsc_amd.so (oracle/Makefile `harness`): its bcsr_sgemm_basic now runs
    on the GPU and must match its gemm_basic (compare(), 1e-4)."""
    exe = os.path.join(ROOT, "oracle", "_ref", "test_bcsr_amd")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/test_bcsr_amd not built (needs /root/reference at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "Test passed!" in r.stdout, r.stdout + r.stderr
