"""The oracle is pinned before it is trusted: every restated function must
reproduce the reference's own outputs (tests/golden/*.npz, produced by the
reference's compiled sources via oracle/_ref) BIT FOR BIT."""
import numpy as np
import pytest

import pyoracle
from conftest import GOLDEN_NAMES, load_golden, tcsc_of


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_tcsc_from_dense_bitexact(oracle, name):
    g = load_golden(name)
    W = oracle.tcsc_from_dense(g["Wd"].astype(np.float32))
    assert W.equal(tcsc_of(g)), name


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_rowmajor_builder_matches(oracle, name):
    g = load_golden(name)
    W = oracle.tcsc_from_dense(g["Wd"].astype(np.float32), rowmajor=True)
    assert W.equal(tcsc_of(g)), name


@pytest.mark.parametrize("name", GOLDEN_NAMES)
@pytest.mark.parametrize("variant", pyoracle.VARIANTS)
def test_kernels_bitexact(oracle, name, variant):
    g = load_golden(name)
    W = tcsc_of(g)
    Y = oracle.sgemm(variant, g["X"], W, g["B"], float(g["a"]))
    ref = g["Y_" + variant]
    assert Y.shape == ref.shape
    # bit-exact, NaN == NaN
    np.testing.assert_array_equal(Y.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_sparse_gemm_omp_and_dense(oracle, name):
    g = load_golden(name)
    W = tcsc_of(g)
    a = float(g["a"])
    np.testing.assert_array_equal(oracle.sparse_gemm_omp(g["X"], W, g["B"]).view(np.uint32),
                                  g["Y_sparsegemm"].view(np.uint32))
    np.testing.assert_array_equal(oracle.sparse_gemm_omp(g["X"], W, g["B"], prelu=True, a=a).view(np.uint32),
                                  g["Y_sparsegemm_prelu"].view(np.uint32))
    if g["meta"]["kind"] != "special":
        np.testing.assert_array_equal(oracle.gemm_basic(g["X"], g["Wd"].astype(np.float32), g["B"]),
                                      g["Y_gemm"])


def test_sparseformat_matches_reference(oracle):
    g = load_golden("sparseformat_48x40")
    W = oracle.sparseformat(g["mat"])
    assert np.array_equal(W.col_start_pos, g["csp"]) and np.array_equal(W.row_index_neg, g["rin"])
    assert np.array_equal(W.col_start_neg, g["csn"]) and np.array_equal(W.row_index_pos, g["rip"])
    # SparseFormat == tcsc_from_dense on ternary input
    W2 = oracle.tcsc_from_dense(g["mat"].astype(np.float32))
    assert W.equal(W2)


@pytest.mark.parametrize("name", ["cfg1", "cfg1_int", "grid_m16_k512_n1024_nz8", "edge_long_k"])
def test_reference_within_tolerance_of_f64(oracle, name):
    """The tolerance used for the GPU (pyoracle.TOL_REL) is met by every
    reference variant itself -- i.e. it is not tighter than the reference."""
    g = load_golden(name)
    W = tcsc_of(g)
    Y64, S64 = oracle.f64_rows(g["X"], W, g["B"])
    for v in pyoracle.VARIANTS:
        a = float(g["a"]) if v in pyoracle.PRELU_VARIANTS else None
        ok, ratio = pyoracle.check_close(g["Y_" + v], Y64, S64, a)
        assert ok, (v, ratio)
        assert ratio < 0.5, (v, ratio)


def test_integer_fixtures_are_order_independent(oracle):
    """Integer X: every summation order is exact, so all 5 variants agree
    bit-for-bit before PReLU -- the GPU must match them exactly."""
    g = load_golden("cfg1_int")
    assert np.array_equal(g["Y_basic"], g["Y_optimized"])
    assert np.array_equal(g["Y_prelu_basic"], g["Y_prelu_separate"])
    assert np.array_equal(g["Y_prelu_basic"], g["Y_prelu_onthego"])
    Y64, _ = oracle.f64_rows(g["X"], tcsc_of(g), g["B"])
    assert np.array_equal(g["Y_basic"].astype(np.float64), Y64)


def test_generators_deterministic(oracle):
    a = oracle.uniform((1000,), 123)
    b = oracle.uniform((1000,), 123)
    assert np.array_equal(a, b) and a.min() >= -1 and a.max() < 1
    t = oracle.ternary((200, 300), 0.02, 5)
    assert set(np.unique(t)) <= {-1.0, 0.0, 1.0}
    d = float(np.count_nonzero(t)) / t.size
    assert 0.01 < d < 0.03


def test_reference_live_matches_oracle_random(oracle):
    """Fresh random case (not a fixture) through the live reference build."""
    ref = pyoracle.load_reference()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference on this host)")
    X = oracle.uniform((33, 517), 99)
    Wd = oracle.ternary((517, 91), 0.07, 98)
    B = oracle.uniform((91,), 97)
    W = oracle.tcsc_from_dense(Wd)
    assert W.equal(ref.tcsc_from_dense(Wd))
    for v in pyoracle.VARIANTS:
        np.testing.assert_array_equal(oracle.sgemm(v, X, W, B, 0.3), ref.sgemm(v, X, W, B, 0.3))


def test_column_slice_rebase(oracle):
    g = load_golden("cfg1")
    W = tcsc_of(g)
    Y = oracle.sgemm("prelu_basic", g["X"], W, g["B"], 0.2)
    for c0, c1 in [(0, 10), (10, 100), (100, 256), (37, 38), (5, 5)]:
        S = W.column_slice(c0, c1)
        Ys = oracle.sgemm("prelu_basic", g["X"], S, g["B"][c0:c1], 0.2)
        np.testing.assert_array_equal(Ys, Y[:, c0:c1])
