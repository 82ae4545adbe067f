"""TEST INFRASTRUCTURE ONLY -- ctypes front-end to the parity checkers.

* ``Oracle``: oracle/liboracle.so, the C restatement of the reference's TCSC
  path (oracle/tcsc_oracle.c; every function cites the reference line it
  follows).
* ``Reference``: oracle/_ref/libtcsc_ref.so, the reference's own
  sparse/tcsc.c + dense/dense.c compiled in place (oracle/Makefile).  Only
  present where it was built; absent -> ``load_reference()`` returns None.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (sparse-matrix-multiplication-benchmark_amd/) never
does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libtcsc_ref.so")
# the same sources built with the reference's own optimisation flags
# (build_and_run_m1.sh:77: -O3 -ffast-math, -march=native pinned to AVX2+FMA):
# a timing baseline only, never a parity oracle (fast-math re-associates)
REF_FAST_SO = os.path.join(HERE, "_ref", "libtcsc_ref_fast.so")

VARIANTS = ("basic", "optimized", "prelu_basic", "prelu_separate", "prelu_onthego")
# the five bcsr_sgemm_* of sparse/bcsr.h:16-39, in the variant-id order of include/bcsr_gpu.h
BCSR_VARIANTS = ("basic", "prelu_basic", "avx", "prelu_avx", "avx2")
BCSR_PRELU_VARIANTS = ("prelu_basic", "prelu_avx")
PRELU_VARIANTS = ("prelu_basic", "prelu_separate", "prelu_onthego")

_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


@dataclass
class TCSC:
    """Host TCSC arrays (the fields of tcsc_t, sparse/tcsc.h:6-17)."""

    rows: int
    cols: int
    col_start_pos: np.ndarray
    col_start_neg: np.ndarray
    row_index_pos: np.ndarray
    row_index_neg: np.ndarray

    @property
    def n_pos(self) -> int:
        return int(self.col_start_pos[-1])

    @property
    def n_neg(self) -> int:
        return int(self.col_start_neg[-1])

    @property
    def nnz(self) -> int:
        return self.n_pos + self.n_neg

    def arrays(self):
        return (self.col_start_pos, self.col_start_neg, self.row_index_pos, self.row_index_neg)

    def equal(self, other: "TCSC") -> bool:
        return (
            self.rows == other.rows
            and self.cols == other.cols
            and all(np.array_equal(a, b) for a, b in zip(self.arrays(), other.arrays()))
        )

    def column_slice(self, c0: int, c1: int) -> "TCSC":
        """Columns [c0, c1), rebased (SURVEY.md §8e partitioning)."""
        p0, p1 = int(self.col_start_pos[c0]), int(self.col_start_pos[c1])
        q0, q1 = int(self.col_start_neg[c0]), int(self.col_start_neg[c1])
        return TCSC(
            self.rows,
            c1 - c0,
            (self.col_start_pos[c0 : c1 + 1] - p0).astype(np.int32),
            (self.col_start_neg[c0 : c1 + 1] - q0).astype(np.int32),
            np.ascontiguousarray(self.row_index_pos[p0:p1]),
            np.ascontiguousarray(self.row_index_neg[q0:q1]),
        )


@dataclass
class BCSR:
    """Host BCSR arrays (the fields of bcsr_t, sparse/bcsr.h:7-12).
    b_row_start has br+1 entries; the ones past the reference's written
    prefix (non-empty block rows + 1, bcsr.c:114-117,137) are k."""

    r: int
    c: int
    br: int
    bc: int
    b_row_start: np.ndarray
    b_col_idx: np.ndarray
    b_values: np.ndarray  # k*r*c float32

    @property
    def k(self) -> int:
        return int(self.b_col_idx.size)

    def arrays(self):
        return (self.b_row_start, self.b_col_idx, self.b_values)

    def equal(self, other: "BCSR") -> bool:
        return ((self.r, self.c, self.br, self.bc) == (other.r, other.c, other.br, other.bc)
                and np.array_equal(self.b_row_start, other.b_row_start)
                and np.array_equal(self.b_col_idx, other.b_col_idx)
                and np.array_equal(self.b_values.view(np.uint32), other.b_values.view(np.uint32)))


def bcsr_variant_allowed(variant: str, r: int, c: int, N: int) -> bool:
    """Shapes each reference variant is defined for (and runs without
    faulting: the avx forms use aligned 8-float loads, bcsr.c:229,250-256)."""
    if variant in ("basic", "prelu_basic"):
        return True
    if c != 8 or N % 8:
        return False
    return variant != "avx2" or r == 8


def _nz(a: np.ndarray) -> np.ndarray:
    """ctypes ndpointer rejects size-0 arrays' NULL data on some numpy builds."""
    return a if a.size else np.zeros(1, dtype=a.dtype)


def build_oracle(force: bool = False) -> None:
    if force or not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", HERE, "liboracle.so"])


class Oracle:
    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            build_oracle()
        L = C.CDLL(path)
        self.lib = L
        L.oracle_tcsc_count.argtypes = [_f32p, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.oracle_tcsc_fill.argtypes = [_f32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p]
        L.oracle_tcsc_fill_rowmajor.argtypes = [_f32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p]
        L.oracle_sparseformat_fill.argtypes = [_i32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p,
                                               C.POINTER(C.c_int), C.POINTER(C.c_int)]
        k_args = [_f32p, _i32p, _i32p, _i32p, _i32p, _f32p]
        for name in ("oracle_sgemm_basic", "oracle_sgemm_optimized"):
            getattr(L, name).argtypes = k_args + [_f32p, C.c_int, C.c_int, C.c_int]
        for name in ("oracle_sgemm_prelu_basic", "oracle_sgemm_prelu_separate", "oracle_sgemm_prelu_onthego"):
            getattr(L, name).argtypes = k_args + [C.c_float, _f32p, C.c_int, C.c_int, C.c_int]
        L.oracle_sparse_gemm_omp.argtypes = k_args + [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_int]
        L.oracle_omp_max_threads.restype = C.c_int
        L.oracle_gemm_basic.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.oracle_sgemm_f64_rows.argtypes = k_args + [_i32p, C.c_int, _f64p, _f64p, C.c_int, C.c_int]
        L.oracle_fill_uniform.argtypes = [_f32p, C.c_size_t, C.c_uint64]
        L.oracle_fill_int.argtypes = [_f32p, C.c_size_t, C.c_uint64, C.c_int]
        L.oracle_fill_ternary.argtypes = [_f32p, C.c_size_t, C.c_uint64, C.c_double]
        L.oracle_bcsr_count.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int),
                                        C.POINTER(C.c_int)]
        L.oracle_bcsr_fill.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p, _f32p]
        L.oracle_bcsr_sgemm.argtypes = [C.c_int, _f32p, C.c_int, C.c_int, C.c_int, _i32p, _i32p, _f32p, _f32p,
                                        C.c_float, _f32p, C.c_int, C.c_int, C.c_int]

    # -- generators -------------------------------------------------------
    def uniform(self, shape, seed: int) -> np.ndarray:
        out = np.empty(shape, dtype=np.float32)
        self.lib.oracle_fill_uniform(out.reshape(-1), out.size, seed)
        return out

    def integers(self, shape, seed: int, rng: int = 512) -> np.ndarray:
        out = np.empty(shape, dtype=np.float32)
        self.lib.oracle_fill_int(out.reshape(-1), out.size, seed, rng)
        return out

    def ternary(self, shape, density: float, seed: int) -> np.ndarray:
        out = np.empty(shape, dtype=np.float32)
        self.lib.oracle_fill_ternary(out.reshape(-1), out.size, seed, density)
        return out

    # -- format -------------------------------------------------------------
    def tcsc_from_dense(self, dense: np.ndarray, rowmajor: bool = False) -> TCSC:
        """tcsc.c:6-66; rowmajor=True uses the fast two-pass restatement
        (same output, pinned by tests/test_oracle.py)."""
        dense = np.ascontiguousarray(dense, dtype=np.float32)
        rows, cols = dense.shape
        p, q = C.c_int(), C.c_int()
        self.lib.oracle_tcsc_count(_nz(dense.reshape(-1)), rows, cols, C.byref(p), C.byref(q))
        csp = np.empty(cols + 1, np.int32)
        csn = np.empty(cols + 1, np.int32)
        rip = np.empty(max(p.value, 1), np.int32)
        rin = np.empty(max(q.value, 1), np.int32)
        fill = self.lib.oracle_tcsc_fill_rowmajor if rowmajor else self.lib.oracle_tcsc_fill
        fill(_nz(dense.reshape(-1)), rows, cols, csp, csn, rip, rin)
        return TCSC(rows, cols, csp, csn, rip[: p.value].copy(), rin[: q.value].copy())

    def sparseformat(self, mat: np.ndarray) -> TCSC:
        mat = np.ascontiguousarray(mat, dtype=np.int32)
        K, N = mat.shape
        csp = np.empty(N + 1, np.int32)
        csn = np.empty(N + 1, np.int32)
        rip = np.empty(max(mat.size, 1), np.int32)
        rin = np.empty(max(mat.size, 1), np.int32)
        p, q = C.c_int(), C.c_int()
        self.lib.oracle_sparseformat_fill(mat.reshape(-1), K, N, csp, csn, rip, rin, C.byref(p), C.byref(q))
        return TCSC(K, N, csp, csn, rip[: p.value].copy(), rin[: q.value].copy())

    # -- kernels ------------------------------------------------------------
    def sgemm(self, variant: str, X: np.ndarray, W: TCSC, B: np.ndarray, a: float = 0.2) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        M, K = X.shape
        N = W.cols
        Y = np.empty((M, N), np.float32)
        args = (_nz(X.reshape(-1)), W.col_start_pos, W.col_start_neg, _nz(W.row_index_pos),
                _nz(W.row_index_neg), _nz(np.ascontiguousarray(B, np.float32)))
        yv = _nz(Y.reshape(-1))
        if variant in PRELU_VARIANTS:
            getattr(self.lib, "oracle_sgemm_" + variant)(*args, a, yv, M, N, K)
        else:
            getattr(self.lib, "oracle_sgemm_" + variant)(*args, yv, M, N, K)
        return Y

    def sparse_gemm_omp(self, X, W: TCSC, B, prelu=False, a=0.2, threads=0) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        M, K = X.shape
        Y = np.empty((M, W.cols), np.float32)
        self.lib.oracle_sparse_gemm_omp(_nz(X.reshape(-1)), W.col_start_pos, W.col_start_neg,
                                        _nz(W.row_index_pos), _nz(W.row_index_neg),
                                        _nz(np.ascontiguousarray(B, np.float32)), _nz(Y.reshape(-1)),
                                        M, W.cols, K, int(prelu), a, threads)
        return Y

    def gemm_basic(self, X, Wd, B) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        Wd = np.ascontiguousarray(Wd, np.float32)
        M, K = X.shape
        N = Wd.shape[1]
        Y = np.empty((M, N), np.float32)
        self.lib.oracle_gemm_basic(_nz(X.reshape(-1)), _nz(Wd.reshape(-1)), _nz(np.ascontiguousarray(B, np.float32)),
                                   _nz(Y.reshape(-1)), M, N, K)
        return Y

    def f64_rows(self, X, W: TCSC, B, rows=None):
        """Exact (fp64) outputs and error scales for the given rows of X."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        M, K = X.shape
        rows = np.arange(M, dtype=np.int32) if rows is None else np.ascontiguousarray(rows, np.int32)
        Y64 = np.empty((len(rows), W.cols), np.float64)
        S64 = np.empty_like(Y64)
        self.lib.oracle_sgemm_f64_rows(_nz(X.reshape(-1)), W.col_start_pos, W.col_start_neg,
                                       _nz(W.row_index_pos), _nz(W.row_index_neg),
                                       _nz(np.ascontiguousarray(B, np.float32)), _nz(rows), len(rows),
                                       _nz(Y64.reshape(-1)), _nz(S64.reshape(-1)), W.cols, K)
        return Y64, S64

    def omp_max_threads(self) -> int:
        return int(self.lib.oracle_omp_max_threads())

    def set_omp_threads(self, n: int) -> None:
        """omp_set_num_threads for this thread: libgomp is one shared library,
        so it also sets the team size of the reference's own OpenMP loops."""
        C.CDLL("libgomp.so.1").omp_set_num_threads(int(n))

    # -- BCSR (oracle/bcsr_oracle.c) -------------------------------------------
    def bcsr_from_dense(self, dense: np.ndarray, r: int, c: int) -> BCSR:
        """bcsr.c:19-139."""
        dense = np.ascontiguousarray(dense, dtype=np.float32)
        rows, cols = dense.shape
        k, ne = C.c_int(), C.c_int()
        self.lib.oracle_bcsr_count(_nz(dense.reshape(-1)), rows, cols, r, c, C.byref(k), C.byref(ne))
        br, bc = rows // r, cols // c
        rs = np.empty(br + 1, np.int32)
        ci = np.empty(max(k.value, 1), np.int32)
        vals = np.empty(max(k.value * r * c, 1), np.float32)
        self.lib.oracle_bcsr_fill(_nz(dense.reshape(-1)), rows, cols, r, c, rs, ci, vals)
        return BCSR(r, c, br, bc, rs, ci[: k.value].copy(), vals[: k.value * r * c].copy())

    def bcsr_sgemm(self, variant: str, X: np.ndarray, W: BCSR, B: np.ndarray, a: float = 0.2,
                   N: int | None = None) -> np.ndarray:
        """bcsr_sgemm_<variant> (bcsr.c:141-385); N defaults to len(B)."""
        X = np.ascontiguousarray(X, dtype=np.float32)
        M, K = X.shape
        B = np.ascontiguousarray(B, np.float32).reshape(-1)
        N = B.size if N is None else N
        Y = np.empty((M, N), np.float32)
        self.lib.oracle_bcsr_sgemm(BCSR_VARIANTS.index(variant), _nz(X.reshape(-1)), W.r, W.c, W.br, W.b_row_start,
                                   _nz(W.b_col_idx), _nz(W.b_values), _nz(B), a, _nz(Y.reshape(-1)), M, N, K)
        return Y


class Reference:
    """The reference's own code (compiled from /root/reference)."""

    def __init__(self, path: str = REF_SO):
        L = C.CDLL(path)
        self.lib = L
        L.ref_tcsc_from_dense.argtypes = [_f32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p,
                                          C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]
        L.ref_tcsc_sgemm.argtypes = [C.c_int, _f32p, _i32p, _i32p, _i32p, _i32p, _f32p, C.c_float, _f32p,
                                     C.c_int, C.c_int, C.c_int]
        L.ref_gemm_basic.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int]
        L.ref_compare.argtypes = [_f32p, _f32p, C.c_int, C.c_int]
        L.ref_compare.restype = C.c_int
        L.ref_sparseformat.argtypes = [_i32p, C.c_int, C.c_int, _i32p, _i32p, _i32p, _i32p,
                                       C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.ref_sparse_gemm.argtypes = [_f32p, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, C.c_int, C.c_int,
                                      C.c_int, C.c_int, C.c_float]
        L.ref_gemm_prelu.argtypes = [_f32p, _f32p, _f32p, _f32p, C.c_int, C.c_int, C.c_int, C.c_float]
        L.ref_bcsr_from_dense.argtypes = [_f32p, C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p, _f32p,
                                          C.POINTER(C.c_int), C.POINTER(C.c_int), C.c_int]
        L.ref_bcsr_sgemm.argtypes = [C.c_int, _f32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _i32p, _i32p,
                                     _f32p, _f32p, C.c_float, _f32p, C.c_int, C.c_int, C.c_int]

    def tcsc_from_dense(self, dense: np.ndarray) -> TCSC:
        dense = np.ascontiguousarray(dense, np.float32)
        rows, cols = dense.shape
        p, q = C.c_int(), C.c_int()
        dummy = np.zeros(1, np.int32)
        self.lib.ref_tcsc_from_dense(_nz(dense.reshape(-1)), rows, cols, dummy, dummy, dummy, dummy,
                                     C.byref(p), C.byref(q), 1)
        csp = np.empty(cols + 1, np.int32)
        csn = np.empty(cols + 1, np.int32)
        rip = np.empty(max(p.value, 1), np.int32)
        rin = np.empty(max(q.value, 1), np.int32)
        self.lib.ref_tcsc_from_dense(_nz(dense.reshape(-1)), rows, cols, csp, csn, rip, rin,
                                     C.byref(p), C.byref(q), 0)
        return TCSC(rows, cols, csp, csn, rip[: p.value].copy(), rin[: q.value].copy())

    def sgemm(self, variant: str, X, W: TCSC, B, a: float = 0.2) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        M, K = X.shape
        Y = np.empty((M, W.cols), np.float32)
        self.lib.ref_tcsc_sgemm(VARIANTS.index(variant), _nz(X.reshape(-1)), W.col_start_pos.copy(),
                                W.col_start_neg.copy(), _nz(W.row_index_pos.copy()), _nz(W.row_index_neg.copy()),
                                _nz(np.ascontiguousarray(B, np.float32).copy()), a, _nz(Y.reshape(-1)),
                                M, W.cols, K)
        return Y

    def sgemm_call(self, variant: str, X, W: TCSC, B, a: float = 0.2):
        """A zero-argument callable running the reference's tcsc_sgemm_<variant>
        on fixed arrays (copied once here, not per call): what bench.py's CPU
        baseline times with the harness's own call loop (main.cpp:54-113)."""
        X = np.ascontiguousarray(X, np.float32).copy()
        M, K = X.shape
        Y = np.empty((M, W.cols), np.float32)
        keep = (X, W.col_start_pos.copy(), W.col_start_neg.copy(), _nz(W.row_index_pos.copy()),
                _nz(W.row_index_neg.copy()), _nz(np.ascontiguousarray(B, np.float32).copy()), Y)
        fn, vid, N = self.lib.ref_tcsc_sgemm, VARIANTS.index(variant), W.cols
        xv, yv = _nz(keep[0].reshape(-1)), _nz(Y.reshape(-1))

        def call():
            fn(vid, xv, keep[1], keep[2], keep[3], keep[4], keep[5], a, yv, M, N, K)

        call.keep = keep
        return call

    def gemm_basic(self, X, Wd, B) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        M, K = X.shape
        N = Wd.shape[1]
        Y = np.empty((M, N), np.float32)
        self.lib.ref_gemm_basic(_nz(X.reshape(-1).copy()), _nz(np.ascontiguousarray(Wd, np.float32).reshape(-1).copy()),
                                _nz(np.ascontiguousarray(B, np.float32).copy()), _nz(Y.reshape(-1)), M, N, K)
        return Y

    def gemm_prelu(self, X, Wd, B, a) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        M, K = X.shape
        N = Wd.shape[1]
        Y = np.empty((M, N), np.float32)
        self.lib.ref_gemm_prelu(_nz(X.reshape(-1).copy()), _nz(np.ascontiguousarray(Wd, np.float32).reshape(-1).copy()),
                                _nz(np.ascontiguousarray(B, np.float32).copy()), _nz(Y.reshape(-1)), M, N, K, a)
        return Y

    def sparseformat(self, mat) -> TCSC:
        mat = np.ascontiguousarray(mat, np.int32)
        K, N = mat.shape
        csp = np.empty(N + 1, np.int32)
        csn = np.empty(N + 1, np.int32)
        rip = np.empty(max(mat.size, 1), np.int32)
        rin = np.empty(max(mat.size, 1), np.int32)
        p, q = C.c_int(), C.c_int()
        self.lib.ref_sparseformat(_nz(mat.reshape(-1).copy()), K, N, csp, csn, rip, rin, C.byref(p), C.byref(q))
        return TCSC(K, N, csp, csn, rip[: p.value].copy(), rin[: q.value].copy())

    def sparse_gemm(self, X, W: TCSC, B, prelu=False, a=0.2) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        M, K = X.shape
        Y = np.empty((M, W.cols), np.float32)
        self.lib.ref_sparse_gemm(_nz(X.reshape(-1).copy()), W.col_start_pos.copy(), W.col_start_neg.copy(),
                                 _nz(W.row_index_pos.copy()), _nz(W.row_index_neg.copy()),
                                 _nz(np.ascontiguousarray(B, np.float32).copy()), _nz(Y.reshape(-1)),
                                 M, W.cols, K, int(prelu), a)
        return Y


    def bcsr_from_dense(self, dense: np.ndarray, r: int, c: int):
        """Returns (BCSR, written): `written` = entries of b_row_start the
        reference itself writes (the rest are set to k)."""
        dense = np.ascontiguousarray(dense, np.float32)
        rows, cols = dense.shape
        k, w = C.c_int(), C.c_int()
        d = np.zeros(1, np.int32)
        self.lib.ref_bcsr_from_dense(_nz(dense.reshape(-1)), rows, cols, r, c, d, d, np.zeros(1, np.float32),
                                     C.byref(k), C.byref(w), 1)
        br, bc = rows // r, cols // c
        rs = np.empty(br + 1, np.int32)
        ci = np.empty(max(k.value, 1), np.int32)
        vals = np.empty(max(k.value * r * c, 1), np.float32)
        self.lib.ref_bcsr_from_dense(_nz(dense.reshape(-1)), rows, cols, r, c, rs, ci, vals, C.byref(k),
                                     C.byref(w), 0)
        return BCSR(r, c, br, bc, rs, ci[: k.value].copy(), vals[: k.value * r * c].copy()), w.value

    def bcsr_sgemm(self, variant: str, X, W: BCSR, B, a: float = 0.2, N: int | None = None) -> np.ndarray:
        X = np.ascontiguousarray(X, np.float32)
        M, K = X.shape
        B = np.ascontiguousarray(B, np.float32).reshape(-1)
        N = B.size if N is None else N
        Y = np.empty((M, N), np.float32)
        self.lib.ref_bcsr_sgemm(BCSR_VARIANTS.index(variant), _nz(X.reshape(-1).copy()), W.r, W.c, W.br, W.bc, W.k,
                                W.b_row_start.copy(), _nz(W.b_col_idx.copy()), _nz(W.b_values.copy()), _nz(B.copy()),
                                a, _nz(Y.reshape(-1)), M, N, K)
        return Y


_ORACLE: Oracle | None = None


def load_oracle() -> Oracle:
    global _ORACLE
    if _ORACLE is None:
        _ORACLE = Oracle()
    return _ORACLE


def load_reference(fast: bool = False) -> Reference | None:
    path = REF_FAST_SO if fast else REF_SO
    if not os.path.exists(path):
        return None
    return Reference(path)


def prelu(v: np.ndarray, a: float) -> np.ndarray:
    return np.where(v < 0, np.float32(a) * v, v).astype(np.float32)


# Tolerance used by every float parity check: per element
#   |y - y64| <= TOL_REL * (|b| + sum_{P u Q} |x|)  (+ TOL_ABS for denormals)
# 2^-20 = 16 fp32 units of roundoff of the worst-case sum magnitude; the
# reference's own kernels measure 0.6-2.2 units on the BASELINE configs.
TOL_REL = 2.0 ** -20
TOL_ABS = 1e-30


def check_close(Y: np.ndarray, Y64: np.ndarray, S64: np.ndarray, prelu_a: float | None = None):
    """Return (ok, worst_ratio).  For PReLU outputs the bound is scaled by
    max(1, a) (PReLU is max(1,a)-Lipschitz) and Y64 is activated first."""
    ref = Y64
    scale = 1.0
    if prelu_a is not None:
        ref = np.where(Y64 < 0, prelu_a * Y64, Y64)
        scale = max(1.0, abs(prelu_a))
    bound = scale * (TOL_REL * S64) + TOL_ABS
    err = np.abs(Y.astype(np.float64) - ref)
    ratio = float(np.max(err / bound)) if err.size else 0.0
    return bool(np.all(err <= bound)), ratio


def assert_builder_matches(oracle: Oracle, dense: np.ndarray, csp, csn, rip, rin) -> None:
    """Pin a device-built TCSC (the library's tcsc_gpu_from_dense) to the
    oracle's tcsc_from_dense (tcsc.c:6-66, row-major restatement) of the same
    dense matrix: all four arrays bit for bit.  Raises AssertionError naming
    the first differing array and position."""
    ref = oracle.tcsc_from_dense(dense, rowmajor=True)
    got = [np.asarray(a, dtype=np.int32) for a in (csp, csn, rip, rin)]
    for name, g, r in zip(("col_start_pos", "col_start_neg", "row_index_pos", "row_index_neg"), got, ref.arrays()):
        if g.shape != r.shape:
            raise AssertionError(f"device builder: {name} has {g.size} entries, the oracle {r.size}")
        bad = np.flatnonzero(g != r)
        if bad.size:
            i = int(bad[0])
            raise AssertionError(f"device builder: {name} differs at {bad.size} entries, first [{i}]: "
                                 f"{int(g[i])} vs oracle {int(r[i])}")
