"""Inputs the reference's loops accept that tcsc_from_dense never produces,
and state the drop-in keeps that the reference does not:

  * hand-built tcsc_t with columns out of order, a row in both the +1 and the
    -1 list, duplicate rows: the reference sums whatever the arrays say
    (tcsc.c:86-93), so the GPU must too (sorted in the plan build; integer
    inputs keep the comparison bit-exact);
  * rows outside [0, K): the reference would read outside X, the library
    reports TCSC_E_ARG instead;
  * the host API's plan cache must notice arrays rebuilt in place;
  * tcsc_gpu_sgemm_prepared / bcsr_gpu_sgemm_prepared must refuse an M that
    was not staged.
"""
import numpy as np
import pytest

import pyoracle
import tcsc_amd
from tcsc_amd import bcsr as tbcsr

pytestmark = pytest.mark.gpu


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


def shuffled_columns(W: pyoracle.TCSC, seed: int) -> pyoracle.TCSC:
    """Same matrix, every column's row list in a random order."""
    rng = np.random.default_rng(seed)
    rip, rin = W.row_index_pos.copy(), W.row_index_neg.copy()
    for cs, ri in ((W.col_start_pos, rip), (W.col_start_neg, rin)):
        for j in range(W.cols):
            seg = ri[cs[j]:cs[j + 1]]
            rng.shuffle(seg)
    return pyoracle.TCSC(W.rows, W.cols, W.col_start_pos.copy(), W.col_start_neg.copy(), rip, rin)


def messy_tcsc(K: int, N: int, seed: int) -> pyoracle.TCSC:
    """Random hand-built TCSC: per column a few +1 and -1 rows drawn with
    replacement (duplicates), some rows in both lists, any order."""
    rng = np.random.default_rng(seed)
    csp, csn, rip, rin = [0], [0], [], []
    for j in range(N):
        p = rng.integers(0, K, rng.integers(0, 9))
        q = rng.integers(0, K, rng.integers(0, 9))
        if p.size and j % 3 == 0:
            q = np.concatenate([q, p[:2]])  # rows in both lists
        rip += list(p)
        rin += list(q)
        csp.append(len(rip))
        csn.append(len(rin))
    i32 = lambda a: np.asarray(a, np.int32)  # noqa: E731
    return pyoracle.TCSC(K, N, i32(csp), i32(csn), i32(rip), i32(rin))


def to_lib(W: pyoracle.TCSC) -> tcsc_amd.TcscMatrix:
    return tcsc_amd.TcscMatrix.from_arrays(W.rows, W.cols, *W.arrays())


@pytest.mark.parametrize("maker", ["shuffled", "messy"])
def test_host_api_hand_built_tcsc(gpu, oracle, maker):
    M, K, N = 77, 300, 90
    if maker == "shuffled":
        W = shuffled_columns(oracle.tcsc_from_dense(oracle.ternary((K, N), 0.1, 31)), 32)
    else:
        W = messy_tcsc(K, N, 33)
    Wl = to_lib(W)
    Xi = oracle.integers((M, K), 34)
    Bi = oracle.integers((N,), 35)
    for variant in pyoracle.VARIANTS:
        Y = tcsc_amd.sgemm(variant, Xi, Wl, Bi, 0.25)
        np.testing.assert_array_equal(Y, oracle.sgemm(variant, Xi, W, Bi, 0.25), err_msg=variant)
    X = oracle.uniform((M, K), 36)
    B = oracle.uniform((N,), 37)
    Y64, S64 = oracle.f64_rows(X, W, B)
    ok, ratio = pyoracle.check_close(tcsc_amd.sgemm("prelu_basic", X, Wl, B, 0.2), Y64, S64, 0.2)
    assert ok, ratio
    Wl.free()


def test_device_plan_hand_built_tcsc(gpu, torch_cuda, oracle):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    M, K, N = 64, 200, 70
    W = messy_tcsc(K, N, 41)
    Xi = oracle.integers((M, K), 42)
    Bi = oracle.integers((N,), 43)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d = [t(a) if a.size else torch.zeros(1, dtype=torch.int32, device=dev) for a in W.arrays()]
    for c0, c1 in ((0, N), (5, 41)):
        plan = tcsc_amd.Plan.from_device(K, N, *d, col_begin=c0, col_end=c1)
        Y = torch.empty((M, c1 - c0), device=dev)
        plan.sgemm(t(Xi), t(Bi[c0:c1]), Y, M, c1 - c0, "optimized", 0.0)
        torch.cuda.synchronize()
        ref = oracle.sgemm("optimized", Xi, W.column_slice(c0, c1), np.ascontiguousarray(Bi[c0:c1]))
        np.testing.assert_array_equal(Y.cpu().numpy(), ref)
        plan.destroy()


def test_out_of_range_rows_rejected(gpu, torch_cuda, oracle, monkeypatch):
    torch = torch_cuda
    K, N = 50, 8
    W = oracle.tcsc_from_dense(oracle.ternary((K, N), 0.2, 51))
    bad = pyoracle.TCSC(K, N, W.col_start_pos, W.col_start_neg, W.row_index_pos.copy(), W.row_index_neg)
    bad.row_index_pos[-1] = K  # one past the last row of X
    Wl = to_lib(bad)
    with pytest.raises(tcsc_amd.TcscError, match="outside"):
        tcsc_amd.Plan(Wl)
    monkeypatch.setenv("TCSC_ON_ERROR", "continue")
    Y = np.full((3, N), 5.0, np.float32)
    tcsc_amd.sgemm("basic", np.ones((3, K), np.float32), Wl, np.zeros(N, np.float32), Y=Y)
    assert np.all(Y == 5.0)
    assert "outside" in tcsc_amd.last_error()
    Wl.free()
    dev = torch.device("cuda:0")
    d = [torch.from_numpy(a).to(dev) for a in bad.arrays()]
    with pytest.raises(tcsc_amd.TcscError, match="outside"):
        tcsc_amd.Plan.from_device(K, N, *d)


def test_cache_sees_arrays_rebuilt_in_place(gpu, oracle):
    """Same tcsc_t, same pointers and counts, new row indices: the host API
    must not run the stale plan (the reference reads the arrays every call)."""
    M, K, N = 40, 120, 30
    W = oracle.tcsc_from_dense(oracle.ternary((K, N), 0.1, 61))
    Wl = to_lib(W)
    Xi = oracle.integers((M, K), 62)
    Bi = oracle.integers((N,), 63)
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W, Bi))
    rip = Wl.row_index("pos")
    rip[:] = (rip + 7) % K  # in place: still in range, counts unchanged
    W2 = pyoracle.TCSC(K, N, W.col_start_pos, W.col_start_neg, rip.copy(), W.row_index_neg)
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W2, Bi))
    Wl.free()


@pytest.mark.parametrize("where", ["first", "last"])
def test_cache_sees_one_changed_index_in_a_large_matrix(gpu, oracle, where):
    """Past 2^20 nonzeros the fingerprint is summed on the copy workers in
    slices: a single row index changed in place, in the first or the last
    slice, must still give a fresh plan."""
    M, K, N = 8, 8192, 8192
    W = oracle.tcsc_from_dense(oracle.ternary((K, N), 0.02, 71))
    assert W.row_index_pos.size + W.row_index_neg.size > 2 ** 20
    Wl = to_lib(W)
    Xi = oracle.integers((M, K), 72)
    Bi = oracle.integers((N,), 73)
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W, Bi))
    rin = Wl.row_index("neg")
    cs = W.col_start_neg
    col = 0 if where == "first" else N - 1
    while cs[col + 1] == cs[col]:
        col += 1 if where == "first" else -1
    j = cs[col] if where == "first" else cs[col + 1] - 1
    lo = rin[j - 1] + 1 if j > cs[col] else 0  # keep the column ascending
    hi = rin[j + 1] - 1 if j + 1 < cs[col + 1] else K - 1
    new = lo if rin[j] != lo else hi
    assert new != rin[j]
    rin[j] = new
    W2 = pyoracle.TCSC(K, N, W.col_start_pos, cs, W.row_index_pos, rin.copy())
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W2, Bi))
    Wl.free()


def test_prepared_needs_a_staged_x_of_that_m(gpu, torch_cuda, oracle):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    K, N = 100, 40
    W = tcsc_amd.TcscMatrix.from_dense(oracle.ternary((K, N), 0.1, 71))
    plan = tcsc_amd.Plan(W)
    B = torch.zeros(N, device=dev)
    Y = torch.empty((64, N), device=dev)
    with pytest.raises(tcsc_amd.TcscError, match="no X is staged"):
        plan.sgemm_prepared(B, Y, 64, N, "basic")
    X = torch.ones((64, K), device=dev)
    plan.prepare_x(X, 32)
    with pytest.raises(tcsc_amd.TcscError, match="another M"):
        plan.sgemm_prepared(B, Y, 64, N, "basic")
    plan.sgemm_prepared(B, Y, 32, N, "basic")
    plan.sgemm(X, B, Y, 64, N, "basic")  # a whole call overwrites the staged X^T
    with pytest.raises(tcsc_amd.TcscError, match="no X is staged"):
        plan.sgemm_prepared(B, Y, 32, N, "basic")
    torch.cuda.synchronize()
    plan.destroy()
    W.free()


def test_bcsr_prepared_needs_a_staged_x_of_that_shape(gpu, torch_cuda, oracle):
    torch = torch_cuda
    dev = torch.device("cuda:0")
    K, N = 64, 32
    Wd = oracle.ternary((K, N), 0.1, 81)
    Wb = tbcsr.BcsrMatrix.from_dense(Wd, 1, 8)
    plan = tbcsr.BcsrPlan(Wb)
    B = torch.zeros(N, device=dev)
    Y = torch.empty((16, N), device=dev)
    with pytest.raises(tcsc_amd.TcscError, match="staged"):
        plan.sgemm_prepared(B, Y, 16, N, K, N, "basic")
    plan.prepare_x(torch.ones((16, K), device=dev), 16, K)
    plan.sgemm_prepared(B, Y, 16, N, K, N, "basic")
    with pytest.raises(tcsc_amd.TcscError, match="staged"):
        plan.sgemm_prepared(B, Y, 8, N, K, N, "basic")
    torch.cuda.synchronize()
    plan.destroy()
    Wb.free()


@pytest.mark.parametrize("variant", ["basic", "prelu_onthego"])
def test_x_beyond_2_31_elements(gpu, torch_cuda, oracle, variant):
    """Maximum sizes: X with M*K > 2^31 elements (8.6 GB), so every row-major
    offset m*K + k past row 130,944 and every X^T offset past 2^31 needs 64-bit
    arithmetic.  Sampled rows on both sides of the crossing against the fp64
    oracle (the reference's int offsets, tcsc.c:87, would overflow here)."""
    torch = torch_cuda
    M, K, N = 131072, 16400, 300
    assert M * K > 2 ** 31
    rng = np.random.default_rng(31)
    dense = rng.random((K, N))
    dense = np.where(dense < 0.01, 1.0, np.where(dense < 0.02, -1.0, 0.0)).astype(np.float32)
    W = oracle.tcsc_from_dense(dense)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev).manual_seed(5)
    X = torch.rand((M, K), device=dev, generator=g) * 2 - 1
    B = torch.from_numpy(rng.uniform(-1, 1, N).astype(np.float32)).to(dev)
    Y = torch.empty((M, N), device=dev)
    lib_w = to_lib(W)
    plan = tcsc_amd.Plan(lib_w)
    plan.reserve(M)
    plan.sgemm(X, B, Y, M, N, variant, 0.2)
    torch.cuda.synchronize()
    rows = np.array([0, 1, 65535, 65536, 130943, 130944, 130945, M - 1])
    idx = torch.from_numpy(rows).to(dev)
    Xs = X[idx].cpu().numpy()
    Ys = Y[idx].cpu().numpy()
    del X
    plan.destroy()
    lib_w.free()
    Y64, S64 = oracle.f64_rows(Xs, W, B.cpu().numpy())
    ok, worst = pyoracle.check_close(Ys, Y64, S64, 0.2 if variant.startswith("prelu") else None)
    assert ok, worst


def test_failed_rebuild_after_in_place_edit_poisons_y(gpu, oracle, monkeypatch):
    """the host API runs a cached plan speculatively while the
    fingerprint is summed.  If the arrays changed in place AND the rebuild
    fails (here a row index moved outside [0, K)), the call must not return
    the stale plan's product under TCSC_ON_ERROR=continue: Y is all NaN and
    the error is reported."""
    monkeypatch.setenv("TCSC_ON_ERROR", "continue")
    M, K, N = 40, 120, 30
    W = oracle.tcsc_from_dense(oracle.ternary((K, N), 0.1, 81))
    Wl = to_lib(W)
    Xi = oracle.integers((M, K), 82)
    Bi = oracle.integers((N,), 83)
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W, Bi))
    rip = Wl.row_index("pos")
    rip[0] = K + 5  # in place, out of range: the plan rebuild refuses it
    Y = np.zeros((M, N), np.float32)
    tcsc_amd.sgemm("basic", Xi, Wl, Bi, Y=Y)
    assert np.all(np.isnan(Y))
    assert "row" in tcsc_amd.last_error().lower() or "index" in tcsc_amd.last_error().lower()
    rip[0] = W.row_index_pos[0]  # repaired in place: a fresh plan, the right product again
    np.testing.assert_array_equal(tcsc_amd.sgemm("basic", Xi, Wl, Bi), oracle.sgemm("basic", Xi, W, Bi))
    Wl.free()


def test_more_than_2pow22_rows_in_one_host_call(gpu, oracle, monkeypatch):
    """the gather launches at most 2^22 rows; a host call with more
    (unbanded, TCSC_HOST_BANDS=1) runs as several launches.  Integer inputs:
    every sampled row bit-identical to the oracle, ragged last launch too."""
    monkeypatch.setenv("TCSC_HOST_BANDS", "1")
    M, K, N = (1 << 22) + 300, 16, 24
    Wd = oracle.ternary((K, N), 0.15, 91)  # K < 64: no MFMA image (and the host's exact mode is the gather)
    W = oracle.tcsc_from_dense(Wd)
    Wl = tcsc_amd.TcscMatrix.from_dense(Wd)
    rng = np.random.default_rng(92)
    Xi = rng.integers(-512, 513, (M, K)).astype(np.float32)
    Bi = rng.integers(-512, 513, N).astype(np.float32)
    Y = tcsc_amd.sgemm("prelu_basic", Xi, Wl, Bi, 0.25)
    rows = np.unique(np.concatenate([[0, (1 << 22) - 1, 1 << 22, M - 1], rng.integers(0, M, 60)]))
    ref = oracle.sgemm("prelu_basic", Xi[rows], W, Bi, 0.25)
    np.testing.assert_array_equal(Y[rows], ref)
    Wl.free()


def test_more_than_2pow22_rows_float_tail_same_order(gpu, oracle, monkeypatch):
    """a device call of more than 2^22 rows runs as launches of
    2^22 rows; the ragged last launch (300 rows, K = 104 > 2 chunks, so the
    cost model alone would split K for it) must sum its rows in the same
    order as the full launches: float inputs, the tail and head rows bit for
    bit equal to single 1-slice launches over the same rows."""
    import torch

    dev = torch.device("cuda:0")
    monkeypatch.setenv("TCSC_PATH", "gather")  # the gather's launches (the cost model would take the MFMA path)
    M, K, N, tail = (1 << 22) + 300, 104, 24, 300
    Wd = oracle.ternary((K, N), 0.15, 93)
    Wl = tcsc_amd.TcscMatrix.from_dense(Wd)
    plan = tcsc_amd.Plan(Wl)
    plan.reserve(M)
    assert plan.launch_info(M)[0] == "gather"
    g = torch.Generator(device=dev)
    g.manual_seed(94)
    X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    Y = torch.empty((M, N), device=dev)
    plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2)
    monkeypatch.setenv("TCSC_SLICES", "1")
    Yt = torch.empty((tail, N), device=dev)
    plan.sgemm(X[M - tail:].contiguous(), B, Yt, tail, N, "prelu_basic", 0.2)
    Yh = torch.empty((tail, N), device=dev)
    plan.sgemm(X[:tail].contiguous(), B, Yh, tail, N, "prelu_basic", 0.2)
    torch.cuda.synchronize()
    assert torch.equal(Y[M - tail:].view(torch.int32), Yt.view(torch.int32))
    assert torch.equal(Y[:tail].view(torch.int32), Yh.view(torch.int32))
    plan.destroy()
    Wl.free()
