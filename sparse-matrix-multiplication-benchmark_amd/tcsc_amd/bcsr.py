"""Python mirror of the BCSR drop-in API (ctypes over libtcsc_amd.so).

Names and argument meaning follow the reference's sparse/bcsr.h:14-39
(W passed by value, argument order (M, N, K) handled here); the device API
of include/bcsr_gpu.h is :class:`BcsrPlan`.  No CPU fallback: every compute
call needs the gfx950 library and a device (TcscError otherwise).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import TcscError, _check, _ptr, lib

VARIANTS = ("basic", "prelu_basic", "avx", "prelu_avx", "avx2")
VARIANT_ID = {v: i for i, v in enumerate(VARIANTS)}
PRELU_VARIANTS = frozenset(("prelu_basic", "prelu_avx"))


class bcsr_t(C.Structure):
    """Layout of bcsr_t (include/sparse/bcsr.h; reference sparse/bcsr.h:7-12)."""

    _fields_ = [
        ("r", C.c_int), ("c", C.c_int), ("br", C.c_int), ("bc", C.c_int), ("k", C.c_int),
        ("b_row_start", C.POINTER(C.c_int)), ("b_col_idx", C.POINTER(C.c_int)),
        ("b_values", C.POINTER(C.c_float)),
    ]


_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")


def bind(L) -> None:
    P = C.POINTER(bcsr_t)
    vp, i, f = C.c_void_p, C.c_int, C.c_float
    L.bcsr_from_dense.argtypes = [_f32p, i, i, i, i]
    L.bcsr_from_dense.restype = P
    for n in ("bcsr_sgemm_basic", "bcsr_sgemm_avx", "bcsr_sgemm_avx2"):
        getattr(L, n).argtypes = [_f32p, bcsr_t, _f32p, _f32p, i, i, i]
        getattr(L, n).restype = None
    for n in ("bcsr_sgemm_prelu_basic", "bcsr_sgemm_prelu_avx"):
        getattr(L, n).argtypes = [_f32p, bcsr_t, _f32p, f, _f32p, i, i, i]
        getattr(L, n).restype = None
    L.bcsr_free.argtypes = [P]
    L.bcsr_free.restype = None
    L.bcsr_gpu_plan_create.argtypes = [P, i, vp, C.POINTER(vp)]
    L.bcsr_gpu_plan_stats.argtypes = [vp, C.POINTER(C.c_longlong), C.POINTER(C.c_size_t)]
    L.bcsr_gpu_plan_reserve.argtypes = [vp, i, i]
    L.bcsr_gpu_plan_destroy.argtypes = [vp]
    L.bcsr_gpu_plan_destroy.restype = None
    L.bcsr_gpu_sgemm.argtypes = [vp, vp, vp, vp, i, i, i, i, i, f, vp]
    L.bcsr_gpu_prepare_x.argtypes = [vp, vp, i, i, vp]
    L.bcsr_gpu_sgemm_prepared.argtypes = [vp, vp, vp, i, i, i, i, i, f, vp]


class BcsrMatrix:
    """Owns a ``bcsr_t*`` (bcsr_from_dense, sparse/bcsr.h:14; freed with bcsr_free)."""

    def __init__(self, ptr):
        if not ptr:
            raise TcscError("bcsr_from_dense returned NULL")
        self.ptr = ptr

    @classmethod
    def from_dense(cls, dense: np.ndarray, r: int, c: int) -> "BcsrMatrix":
        dense = np.ascontiguousarray(dense, dtype=np.float32)
        rows, cols = dense.shape
        buf = dense.reshape(-1) if dense.size else np.zeros(1, np.float32)
        return cls(lib().bcsr_from_dense(buf, rows, cols, int(r), int(c)))

    @property
    def struct(self) -> bcsr_t:
        return self.ptr.contents

    def __getattr__(self, name):
        if name in ("r", "c", "br", "bc", "k"):
            return getattr(self.ptr.contents, name)
        raise AttributeError(name)

    def arrays(self):
        """(b_row_start, b_col_idx, b_values) copies."""
        t = self.ptr.contents

        def take(p, n, dt):
            return np.ctypeslib.as_array(p, shape=(n,)).copy() if n > 0 else np.zeros(0, dt)

        return (take(t.b_row_start, t.br + 1, np.int32), take(t.b_col_idx, t.k, np.int32),
                take(t.b_values, t.k * t.r * t.c, np.float32))

    def free(self) -> None:
        if self.ptr:
            lib().bcsr_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def struct_from_arrays(r, c, br, bc, rs, ci, vals):
    """A bcsr_t view of numpy arrays (kept alive by the caller)."""
    t = bcsr_t()
    t.r, t.c, t.br, t.bc, t.k = int(r), int(c), int(br), int(bc), int(ci.size)
    t.b_row_start = rs.ctypes.data_as(C.POINTER(C.c_int))
    t.b_col_idx = ci.ctypes.data_as(C.POINTER(C.c_int))
    t.b_values = vals.ctypes.data_as(C.POINTER(C.c_float))
    return t


def sgemm(variant: str, X: np.ndarray, W, B: np.ndarray, a: float = 0.2, N: int | None = None,
          Y: np.ndarray | None = None) -> np.ndarray:
    """Host-pointer call of bcsr_sgemm_<variant> (sparse/bcsr.h:16-39).
    W: a BcsrMatrix or a bcsr_t; N defaults to len(B)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    M, K = X.shape
    B = np.ascontiguousarray(B, dtype=np.float32).reshape(-1)
    N = B.size if N is None else N
    if Y is None:
        Y = np.empty((M, N), np.float32)
    st = W.struct if isinstance(W, BcsrMatrix) else W
    nz = lambda a_: a_.reshape(-1) if a_.size else np.zeros(1, np.float32)  # noqa: E731
    fn = getattr(lib(), "bcsr_sgemm_" + variant)
    if variant in PRELU_VARIANTS:
        fn(nz(X), st, nz(B), a, nz(Y), M, N, K)
    else:
        fn(nz(X), st, nz(B), nz(Y), M, N, K)
    return Y


class BcsrPlan:
    """Device plan of one bcsr_t (include/bcsr_gpu.h)."""

    def __init__(self, W, device: int = 0, stream: int = 0):
        h = C.c_void_p()
        ptr = W.ptr if isinstance(W, BcsrMatrix) else C.pointer(W)
        _check(lib().bcsr_gpu_plan_create(ptr, device, C.c_void_p(stream), C.byref(h)), "bcsr_gpu_plan_create")
        self.handle = h

    def stats(self) -> dict:
        v, b = C.c_longlong(), C.c_size_t()
        _check(lib().bcsr_gpu_plan_stats(self.handle, C.byref(v), C.byref(b)), "bcsr_gpu_plan_stats")
        return {"block_visits": v.value, "device_bytes": b.value}

    def reserve(self, max_M: int, K: int) -> None:
        _check(lib().bcsr_gpu_plan_reserve(self.handle, int(max_M), int(K)), "bcsr_gpu_plan_reserve")

    def sgemm(self, X, B, Y, M: int, N: int, K: int, ldy: int, variant: str = "basic", a: float = 0.2,
              stream: int = 0) -> None:
        _check(lib().bcsr_gpu_sgemm(self.handle, C.c_void_p(_ptr(X)), C.c_void_p(_ptr(B)), C.c_void_p(_ptr(Y)),
                                    int(M), int(N), int(K), int(ldy), VARIANT_ID[variant], float(a),
                                    C.c_void_p(stream)), "bcsr_gpu_sgemm")

    def prepare_x(self, X, M: int, K: int, stream: int = 0) -> None:
        _check(lib().bcsr_gpu_prepare_x(self.handle, C.c_void_p(_ptr(X)), int(M), int(K), C.c_void_p(stream)),
               "bcsr_gpu_prepare_x")

    def sgemm_prepared(self, B, Y, M: int, N: int, K: int, ldy: int, variant: str = "basic", a: float = 0.2,
                       stream: int = 0) -> None:
        _check(lib().bcsr_gpu_sgemm_prepared(self.handle, C.c_void_p(_ptr(B)), C.c_void_p(_ptr(Y)), int(M), int(N),
                                             int(K), int(ldy), VARIANT_ID[variant], float(a), C.c_void_p(stream)),
               "bcsr_gpu_sgemm_prepared")

    def destroy(self) -> None:
        if getattr(self, "handle", None):
            lib().bcsr_gpu_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass
