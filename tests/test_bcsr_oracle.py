"""BCSR path, checked without a GPU.

* The oracle (oracle/bcsr_oracle.c) reproduces the reference's own outputs
  (tests/golden/bcsr/*.npz, made by the reference's bcsr.c via oracle/_ref)
  BIT FOR BIT: bcsr_from_dense arrays and every variant's Y, NaN payloads
  included.
* The library's host bcsr_from_dense (libtcsc_amd.so) builds the same arrays.
* The reference's variants agree with each other where the reference says
  they must (ternary W: mul + add == fma) and differ where rounding says
  they may (non-ternary W).
"""
import ctypes

import numpy as np
import pytest

import pyoracle
from conftest import BCSR_GOLDEN_NAMES, load_bcsr_golden, bcsr_of

import tcsc_amd
from tcsc_amd import bcsr


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.mark.parametrize("name", BCSR_GOLDEN_NAMES)
def test_oracle_bcsr_from_dense_bitexact(oracle, name):
    g = load_bcsr_golden(name)
    W = oracle.bcsr_from_dense(g["Wd"].astype(np.float32), int(g["r"]), int(g["c"]))
    assert W.equal(bcsr_of(g)), name
    # the reference's written prefix is followed by k (convention of include/sparse/bcsr.h)
    w = int(g["written"])
    assert np.all(g["rs"][w:] == W.k)


@pytest.mark.parametrize("name", BCSR_GOLDEN_NAMES)
def test_oracle_bcsr_kernels_bitexact(oracle, name):
    g = load_bcsr_golden(name)
    W = bcsr_of(g)
    for v in pyoracle.BCSR_VARIANTS:
        if "Y_" + v not in g:
            continue
        Y = oracle.bcsr_sgemm(v, g["X"], W, g["B"], float(g["a"]))
        np.testing.assert_array_equal(bits(Y), bits(g["Y_" + v]), err_msg=f"{name}/{v}")


@pytest.mark.parametrize("name", BCSR_GOLDEN_NAMES)
def test_library_host_bcsr_from_dense_bitexact(name):
    tcsc_amd.build()
    g = load_bcsr_golden(name)
    W = bcsr.BcsrMatrix.from_dense(g["Wd"].astype(np.float32), int(g["r"]), int(g["c"]))
    ref = bcsr_of(g)
    assert (W.r, W.c, W.br, W.bc, W.k) == (ref.r, ref.c, ref.br, ref.bc, ref.k)
    for a, b in zip(W.arrays(), ref.arrays()):
        np.testing.assert_array_equal(np.ascontiguousarray(a).view(np.uint32),
                                      np.ascontiguousarray(b).view(np.uint32))
    W.free()


def test_variant_relations_in_reference_outputs():
    """Ternary W: every product is exact, so the mul+add variants and the
    fma variants are bit-identical; the non-ternary fixture exercises the
    difference (the GPU must match each variant separately)."""
    g = load_bcsr_golden("m16_k256_n256_8x8")
    assert np.array_equal(bits(g["Y_basic"]), bits(g["Y_avx"]))
    assert np.array_equal(bits(g["Y_basic"]), bits(g["Y_avx2"]))
    assert np.array_equal(bits(g["Y_prelu_basic"]), bits(g["Y_prelu_avx"]))
    n = load_bcsr_golden("nonternary_2x8")
    fin = np.isfinite(n["Y_basic"]) & np.isfinite(n["Y_avx"])
    assert not np.array_equal(n["Y_basic"][fin], n["Y_avx"][fin])


def test_empty_block_rows_compaction_fixture():
    """bcsr.c:114-117: b_row_start holds one entry per NON-empty block row,
    so with block rows 2 and 5 empty the array is shifted (and the
    reference's kernels read the shifted ranges)."""
    g = load_bcsr_golden("empty_block_rows_4x8")
    assert int(g["written"]) == (40 // 4) - 2 + 1
    W = bcsr_of(g)
    assert W.b_row_start[-1] == W.k and W.b_row_start[-2] == W.k


def test_prelu_every_step_semantics(oracle):
    """prelu_basic applies (v>0 ? v : a*v) after EVERY update (bcsr.c:208-209),
    not once: a column with one stored block of two rows gives
    f(f(b + x0*w0) + x1*w1), f(v) = v>0 ? v : a v."""
    Wd = np.zeros((2, 8), np.float32)
    Wd[0, 0], Wd[1, 0] = 1.0, -1.0
    W = oracle.bcsr_from_dense(Wd, 2, 8)
    X = np.array([[-3.0, 1.0]], np.float32)
    B = np.zeros(8, np.float32)
    B[0] = 1.0
    Y = oracle.bcsr_sgemm("prelu_basic", X, W, B, 0.5)
    f = lambda v: v if v > 0 else np.float32(0.5) * v  # noqa: E731
    assert Y[0, 0] == f(f(np.float32(1.0) - 3.0) - 1.0)  # f(-2) = -1, then f(-2) = -1
    assert Y[0, 1] == f(f(0.0))


def test_reference_live_random(oracle):
    ref = pyoracle.load_reference()
    if ref is None:
        pytest.skip("oracle/_ref not built (no /root/reference on this host)")
    X = oracle.uniform((11, 96), 41)
    Wd = oracle.ternary((96, 64), 0.03, 42)
    B = oracle.uniform((64,), 43)
    for r, c in ((1, 8), (8, 8), (3, 8), (4, 4)):
        W = oracle.bcsr_from_dense(Wd, r, c)
        R, _ = ref.bcsr_from_dense(Wd, r, c)
        assert W.equal(R)
        for v in pyoracle.BCSR_VARIANTS:
            if pyoracle.bcsr_variant_allowed(v, r, c, 64):
                np.testing.assert_array_equal(bits(oracle.bcsr_sgemm(v, X, W, B, 0.3)),
                                              bits(ref.bcsr_sgemm(v, X, R, B, 0.3)))


def test_bcsr_struct_layout_matches_reference():
    """bcsr_t keeps the reference's field order (sparse/bcsr.h:7-12): 5 ints
    then 3 pointers, 48 bytes on LP64 (passed by value in memory)."""
    assert ctypes.sizeof(bcsr.bcsr_t) == 48
    assert [f[0] for f in bcsr.bcsr_t._fields_] == ["r", "c", "br", "bc", "k", "b_row_start", "b_col_idx",
                                                   "b_values"]


def test_host_api_fails_loudly_without_device():
    tcsc_amd.build()
    if tcsc_amd.device_count() > 0:
        pytest.skip("GPU present")
    import subprocess
    import sys

    from conftest import PKG

    code = ("import sys, numpy as np; sys.path.insert(0, %r); import tcsc_amd; from tcsc_amd import bcsr;"
            "W = bcsr.BcsrMatrix.from_dense(np.eye(8, dtype=np.float32), 1, 8);"
            "bcsr.sgemm('basic', np.ones((2,8),np.float32), W, np.zeros(8,np.float32))" % PKG)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "no HIP device" in r.stderr
