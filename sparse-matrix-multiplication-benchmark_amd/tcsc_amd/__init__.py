"""Python mirror of the TCSC drop-in API (ctypes over libtcsc_amd.so).

Names and argument order follow the reference's C API (sparse/tcsc.h:19-48,
argument order (M, N, K) handled internally); numpy arrays stand in for
``dense_t`` and :class:`TcscMatrix` owns a ``tcsc_t*`` created by the
library's ``tcsc_from_dense``.  The device API of include/tcsc_gpu.h is
exposed through :class:`Plan`, which takes raw device pointers (ints) or
torch tensors.

There is no CPU fallback: importing works without a GPU (so the ABI can be
checked on a build host), but every compute call needs the gfx950 HIP
library and a visible device, and raises :class:`TcscError` otherwise.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# TCSC_AMD_LIB points at an alternative build (e.g. the timing-only ablation
# builds of `make ablation`); default: the in-tree library.
LIB_PATH = os.environ.get("TCSC_AMD_LIB") or os.path.join(PKG_DIR, "lib", "libtcsc_amd.so")

VARIANTS = ("basic", "optimized", "prelu_basic", "prelu_separate", "prelu_onthego")
VARIANT_ID = {v: i for i, v in enumerate(VARIANTS)}
# SparseGEMM.h's sparseGEMM<float> (include/tcsc_gpu.h TCSC_VARIANT_SPARSE_GEMM):
# bias last, no activation; accepted by the device API (Plan.sgemm)
VARIANT_ID["sparse_gemm"] = 5
PRELU_VARIANTS = frozenset(VARIANTS[2:])

# every symbol include/*.h declares (checked by tests/test_abi.py)
EXPORTED_SYMBOLS = (
    # include/sparse/tcsc.h
    "tcsc_from_dense", "tcsc_sgemm_basic", "tcsc_sgemm_optimized", "tcsc_sgemm_prelu_basic",
    "tcsc_sgemm_prelu_optimized_separate", "tcsc_sgemm_prelu_optimized_onthego", "tcsc_free",
    # include/dense/dense.h
    "dense_random", "init_rand_dense", "init_rand_sparse", "compare", "gemm_basic", "gemm_prelu_basic",
    "tcsc_set_seed",
    # include/tcsc_gpu.h
    "tcsc_gpu_device_count", "tcsc_gpu_plan_create", "tcsc_gpu_plan_create_device", "tcsc_gpu_plan_get_info",
    "tcsc_gpu_plan_reserve", "tcsc_gpu_plan_destroy", "tcsc_gpu_sgemm", "tcsc_gpu_prepare_x",
    "tcsc_gpu_sgemm_prepared", "tcsc_gpu_from_dense", "tcsc_gpu_dense_sgemm", "tcsc_gpu_last_error",
    "tcsc_gpu_cache_clear", "tcsc_gpu_num_shards", "tcsc_gpu_set_num_shards", "tcsc_gpu_set_order",
    "tcsc_gpu_get_order", "tcsc_gpu_launch_info", "tcsc_gpu_launch_combine", "tcsc_gpu_build_flags",
    # include/sparse/bcsr.h
    "bcsr_from_dense", "bcsr_sgemm_basic", "bcsr_sgemm_prelu_basic", "bcsr_sgemm_avx", "bcsr_sgemm_prelu_avx",
    "bcsr_sgemm_avx2", "bcsr_free",
    # include/bcsr_gpu.h
    "bcsr_gpu_plan_create", "bcsr_gpu_plan_stats", "bcsr_gpu_plan_reserve", "bcsr_gpu_plan_destroy",
    "bcsr_gpu_sgemm", "bcsr_gpu_prepare_x", "bcsr_gpu_sgemm_prepared",
    # include/sparse_gemm.h (SparseGEMM.h's raw-array API)
    "tcsc_sparse_format", "tcsc_sparse_gemm", "tcsc_sparse_gemm_prelu", "tcsc_dense_gemm", "tcsc_dense_gemm_prelu",
)


class TcscError(RuntimeError):
    pass


class tcsc_t(C.Structure):
    """Layout of tcsc_t (include/sparse/tcsc.h; reference sparse/tcsc.h:6-17)."""

    _fields_ = [
        ("rows", C.c_int), ("cols", C.c_int), ("n_elem_pos", C.c_int), ("n_elem_neg", C.c_int),
        ("col_start_pos", C.POINTER(C.c_int)), ("col_start_neg", C.POINTER(C.c_int)),
        ("row_index_pos", C.POINTER(C.c_int)), ("row_index_neg", C.POINTER(C.c_int)),
    ]


class plan_info_t(C.Structure):
    _fields_ = [
        ("device", C.c_int), ("rows", C.c_int), ("cols", C.c_int), ("col_begin", C.c_int),
        ("nnz", C.c_longlong), ("n_pos", C.c_longlong), ("n_neg", C.c_longlong),
        ("chunk_k", C.c_int), ("n_chunks", C.c_int), ("device_bytes", C.c_size_t), ("order", C.c_int),
        ("mfma_min_M", C.c_int),
    ]


_f32p = np.ctypeslib.ndpointer(dtype=np.float32, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")
_lib = None


def build(force: bool = False) -> str:
    """Compile lib/libtcsc_amd.so (hipcc --offload-arch=gfx950)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", PKG_DIR, "-j8"])
    return LIB_PATH


def lib():
    """Load the library (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise TcscError(f"{LIB_PATH} missing: build it with `make -C {PKG_DIR}`")
    # One HIP runtime per process: torch ships its own libamdhip64 (SONAME
    # libamdhip64.so.7, the one the library needs too).  Loaded first, it is
    # the one the library binds to; loaded after the library's
    # /opt/rocm copy, torch sees two runtimes and reports no device
    # (torch.cuda.is_available() False).  So bring torch in first when it is
    # installed; the library itself never calls into torch.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(LIB_PATH)
    # the timing-only diagnostic builds of tools/ab.mk compute wrong results by
    # design: never under a parity test or a bench line unless asked for
    L.tcsc_gpu_build_flags.restype = C.c_int
    flags = int(L.tcsc_gpu_build_flags())
    if flags and os.environ.get("TCSC_ALLOW_DIAG") != "1":
        raise TcscError(f"{LIB_PATH} is a diagnostic build (flags {flags:#x}: ablation/no-DMA/stamps/trace, "
                        "results wrong by design); set TCSC_ALLOW_DIAG=1 to load it anyway")
    vp, i, f = C.c_void_p, C.c_int, C.c_float
    P = C.POINTER(tcsc_t)
    L.tcsc_from_dense.argtypes = [_f32p, i, i]
    L.tcsc_from_dense.restype = P
    for n in ("tcsc_sgemm_basic", "tcsc_sgemm_optimized"):
        getattr(L, n).argtypes = [_f32p, P, _f32p, _f32p, i, i, i]
        getattr(L, n).restype = None
    for n in ("tcsc_sgemm_prelu_basic", "tcsc_sgemm_prelu_optimized_separate",
              "tcsc_sgemm_prelu_optimized_onthego"):
        getattr(L, n).argtypes = [_f32p, P, _f32p, f, _f32p, i, i, i]
        getattr(L, n).restype = None
    L.tcsc_free.argtypes = [P]
    L.tcsc_free.restype = None
    L.tcsc_set_seed.argtypes = [C.c_ulonglong]
    L.tcsc_gpu_device_count.restype = i
    L.tcsc_gpu_last_error.restype = C.c_char_p
    L.tcsc_gpu_plan_create.argtypes = [P, i, i, i, vp, C.POINTER(vp)]
    L.tcsc_gpu_plan_create_device.argtypes = [i, i, vp, vp, vp, vp, i, i, i, vp, C.POINTER(vp)]
    L.tcsc_gpu_plan_get_info.argtypes = [vp, C.POINTER(plan_info_t)]
    L.tcsc_gpu_launch_info.argtypes = [vp, i, C.POINTER(i), C.POINTER(i)]
    L.tcsc_gpu_launch_combine.argtypes = [vp, i, C.POINTER(i)]
    L.tcsc_gpu_plan_reserve.argtypes = [vp, i]
    L.tcsc_gpu_plan_destroy.argtypes = [vp]
    L.tcsc_gpu_plan_destroy.restype = None
    L.tcsc_gpu_sgemm.argtypes = [vp, vp, vp, vp, i, i, i, f, vp]
    L.tcsc_gpu_prepare_x.argtypes = [vp, vp, i, vp]
    L.tcsc_gpu_sgemm_prepared.argtypes = [vp, vp, vp, i, i, i, f, vp]
    L.tcsc_gpu_from_dense.argtypes = [vp, i, i, vp, vp, vp, vp, C.POINTER(i), C.POINTER(i), vp]
    L.tcsc_gpu_dense_sgemm.argtypes = [vp, vp, vp, vp, i, i, i, i, i, f, vp]
    L.tcsc_gpu_num_shards.restype = i
    L.tcsc_gpu_set_num_shards.argtypes = [i]
    L.tcsc_gpu_set_num_shards.restype = None
    L.tcsc_gpu_cache_clear.restype = None
    L.tcsc_gpu_set_order.argtypes = [i]
    L.tcsc_gpu_set_order.restype = None
    L.tcsc_gpu_get_order.restype = i
    ip = C.POINTER(i)
    L.tcsc_sparse_format.argtypes = [_i32p, i, i, _i32p, _i32p, vp, vp, ip, ip]
    L.tcsc_sparse_format.restype = i
    L.tcsc_sparse_gemm.argtypes = [_f32p, _i32p, _i32p, _i32p, _i32p, _f32p, _f32p, i, i, i]
    L.tcsc_sparse_gemm.restype = None
    L.tcsc_sparse_gemm_prelu.argtypes = L.tcsc_sparse_gemm.argtypes + [f]
    L.tcsc_sparse_gemm_prelu.restype = None
    L.tcsc_dense_gemm.argtypes = [_f32p, _f32p, _f32p, _f32p, i, i, i]
    L.tcsc_dense_gemm.restype = None
    L.tcsc_dense_gemm_prelu.argtypes = L.tcsc_dense_gemm.argtypes + [f]
    L.tcsc_dense_gemm_prelu.restype = None
    from . import bcsr as _bcsr

    _bcsr.bind(L)
    _lib = L
    return L


def last_error() -> str:
    return lib().tcsc_gpu_last_error().decode(errors="replace")


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise TcscError(f"{what} failed (status {rc}): {last_error()}")


def device_count() -> int:
    return int(lib().tcsc_gpu_device_count())


def require_gpu() -> None:
    if device_count() <= 0:
        raise TcscError("no HIP device visible: the TCSC kernels need a gfx950 (MI355X) GPU")


class TcscMatrix:
    """Owns a ``tcsc_t*`` (tcsc_from_dense / tcsc_free, sparse/tcsc.h:19,48)."""

    def __init__(self, ptr):
        if not ptr:
            raise TcscError("tcsc_from_dense returned NULL")
        self.ptr = ptr

    @classmethod
    def from_dense(cls, dense: np.ndarray) -> "TcscMatrix":
        dense = np.ascontiguousarray(dense, dtype=np.float32)
        rows, cols = dense.shape
        buf = dense.reshape(-1) if dense.size else np.zeros(1, np.float32)
        return cls(lib().tcsc_from_dense(buf, rows, cols))

    @classmethod
    def from_arrays(cls, rows: int, cols: int, col_start_pos, col_start_neg, row_index_pos,
                    row_index_neg) -> "TcscMatrix":
        """A hand-built ``tcsc_t`` (the struct of sparse/tcsc.h:6-17) from four
        index arrays, in malloc'd memory so that ``tcsc_free`` releases it as
        it releases ``tcsc_from_dense``'s.  No checks here: the library's
        plan build validates (rows in [0, rows), order) as the tests need."""
        libc = C.CDLL(None)
        libc.malloc.restype = C.c_void_p
        libc.malloc.argtypes = [C.c_size_t]

        def put(a):
            a = np.ascontiguousarray(a, dtype=np.int32).reshape(-1)
            p = libc.malloc(max(a.nbytes, 4))
            if not p:
                raise MemoryError("malloc failed")
            if a.size:
                C.memmove(p, a.ctypes.data, a.nbytes)
            return C.cast(p, C.POINTER(C.c_int)), a.size

        t = libc.malloc(C.sizeof(tcsc_t))
        if not t:
            raise MemoryError("malloc failed")
        s = C.cast(t, C.POINTER(tcsc_t))
        s.contents.rows, s.contents.cols = int(rows), int(cols)
        s.contents.col_start_pos, _ = put(col_start_pos)
        s.contents.col_start_neg, _ = put(col_start_neg)
        s.contents.row_index_pos, s.contents.n_elem_pos = put(row_index_pos)
        s.contents.row_index_neg, s.contents.n_elem_neg = put(row_index_neg)
        return cls(s)

    def row_index(self, sign: str) -> np.ndarray:
        """Writable view of row_index_pos ('pos') or row_index_neg ('neg'):
        lets tests rebuild the arrays in place, as a caller may."""
        t = self.ptr.contents
        p, n = (t.row_index_pos, t.n_elem_pos) if sign == "pos" else (t.row_index_neg, t.n_elem_neg)
        return np.ctypeslib.as_array(p, shape=(n,)) if n > 0 else np.zeros(0, np.int32)

    @property
    def rows(self) -> int:
        return self.ptr.contents.rows

    @property
    def cols(self) -> int:
        return self.ptr.contents.cols

    @property
    def nnz(self) -> int:
        t = self.ptr.contents
        return t.n_elem_pos + t.n_elem_neg

    def arrays(self):
        """(col_start_pos, col_start_neg, row_index_pos, row_index_neg) copies."""
        t = self.ptr.contents

        def take(p, n):
            return np.ctypeslib.as_array(p, shape=(n,)).copy() if n > 0 else np.zeros(0, np.int32)

        return (take(t.col_start_pos, t.cols + 1), take(t.col_start_neg, t.cols + 1),
                take(t.row_index_pos, t.n_elem_pos), take(t.row_index_neg, t.n_elem_neg))

    def free(self) -> None:
        if self.ptr:
            lib().tcsc_free(self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def sgemm(variant: str, X: np.ndarray, W: TcscMatrix, B: np.ndarray, a: float = 0.2,
          Y: np.ndarray | None = None) -> np.ndarray:
    """Host-pointer call of tcsc_sgemm_<variant> (sparse/tcsc.h:21-46).

    The C entry points trust their sizes as the reference's do (they read N
    floats of B and write M rows of pitch N into Y), so the shapes are checked
    here and a mismatch raises :class:`TcscError` instead of reaching the
    library as an out-of-bounds host read or write."""
    if variant not in VARIANTS:
        raise TcscError(f"unknown variant {variant!r} (one of {', '.join(VARIANTS)})")
    if not getattr(W, "ptr", None):
        raise TcscError("W is freed or not a TcscMatrix")
    X = np.ascontiguousarray(X, dtype=np.float32)
    if X.ndim != 2:
        raise TcscError(f"X must be 2-D (M x K), got shape {X.shape}")
    M, K = X.shape
    N = W.cols
    if K != W.rows:
        raise TcscError(f"X has K={K} columns but W has {W.rows} rows")
    B = np.ascontiguousarray(B, dtype=np.float32).reshape(-1)
    if B.size != N:
        raise TcscError(f"B has {B.size} elements, W has N={N} columns")
    if Y is None:
        Y = np.empty((M, N), np.float32)
    elif (not isinstance(Y, np.ndarray) or Y.shape != (M, N) or Y.dtype != np.float32
          or not Y.flags["C_CONTIGUOUS"]):
        raise TcscError(f"Y must be a C-contiguous float32 array of shape ({M}, {N})")
    L = lib()
    nz = lambda a_: a_.reshape(-1) if a_.size else np.zeros(1, np.float32)  # noqa: E731
    if variant in PRELU_VARIANTS:
        name = "tcsc_sgemm_prelu_basic" if variant == "prelu_basic" else "tcsc_sgemm_" + variant.replace(
            "prelu_", "prelu_optimized_")
        getattr(L, name)(nz(X), W.ptr, nz(B), a, nz(Y), M, N, K)
    else:
        getattr(L, "tcsc_sgemm_" + variant)(nz(X), W.ptr, nz(B), nz(Y), M, N, K)
    return Y


# --- SparseGEMM.h's raw-array API (include/sparse_gemm.h) -------------------

def sparse_format(matrix: np.ndarray):
    """SparseFormat(int* matrix, K, N) (SparseGEMM.h:20-39): an int K x N
    matrix -> (col_start_pos, col_start_neg, row_index_pos, row_index_neg);
    >= 1 is +1, <= -1 is -1.  Host code in the library (no GPU needed)."""
    m = np.ascontiguousarray(matrix, dtype=np.int32)
    if m.ndim != 2:
        raise TcscError(f"matrix must be 2-D (K x N), got shape {m.shape}")
    K, N = m.shape
    flat = m.reshape(-1) if m.size else np.zeros(1, np.int32)
    csp, csn = np.zeros(N + 1, np.int32), np.zeros(N + 1, np.int32)
    p, q = C.c_int(0), C.c_int(0)
    L = lib()
    _check(L.tcsc_sparse_format(flat, K, N, csp, csn, None, None, C.byref(p), C.byref(q)), "tcsc_sparse_format")
    rip, rin = np.zeros(max(p.value, 1), np.int32), np.zeros(max(q.value, 1), np.int32)
    _check(L.tcsc_sparse_format(flat, K, N, csp, csn, rip.ctypes.data, rin.ctypes.data, C.byref(p), C.byref(q)),
           "tcsc_sparse_format")
    return csp, csn, rip[:p.value].copy(), rin[:q.value].copy()


def sparse_gemm(X: np.ndarray, col_start_pos, col_start_neg, row_index_pos, row_index_neg, b: np.ndarray,
                a: float | None = None, Y: np.ndarray | None = None) -> np.ndarray:
    """sparseGEMM<float> (a None) or sparseGEMM_PReLU<float> (SparseGEMM.h:104-119,
    151-168) on host arrays: Y = act(X . W + b), W given by its four TCSC
    arrays.  Shapes are checked here (the C entry points trust them)."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    if X.ndim != 2:
        raise TcscError(f"X must be 2-D (M x K), got shape {X.shape}")
    M, K = X.shape
    arrs = [np.ascontiguousarray(v, dtype=np.int32).reshape(-1)
            for v in (col_start_pos, col_start_neg, row_index_pos, row_index_neg)]
    csp, csn, rip, rin = arrs
    N = csp.size - 1
    if N < 0 or csn.size != N + 1:
        raise TcscError("col_start_pos / col_start_neg must both have N+1 entries")
    if rip.size < csp[-1] or rin.size < csn[-1]:
        raise TcscError("row_index arrays shorter than col_start[N]")
    b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
    if b.size != N:
        raise TcscError(f"b has {b.size} elements, W has N={N} columns")
    if Y is None:
        Y = np.empty((M, N), np.float32)
    elif Y.shape != (M, N) or Y.dtype != np.float32 or not Y.flags["C_CONTIGUOUS"]:
        raise TcscError(f"Y must be a C-contiguous float32 array of shape ({M}, {N})")
    nz = lambda v, t: v if v.size else np.zeros(1, t)  # noqa: E731
    args = [nz(X.reshape(-1), np.float32), csp, csn, nz(rip, np.int32), nz(rin, np.int32), nz(b, np.float32),
            nz(Y.reshape(-1), np.float32), M, N, K]
    if a is None:
        lib().tcsc_sparse_gemm(*args)
    else:
        lib().tcsc_sparse_gemm_prelu(*args, float(a))
    return Y


def dense_gemm(X: np.ndarray, W: np.ndarray, b: np.ndarray, a: float | None = None) -> np.ndarray:
    """GEMM<float> / GEMM_PReLU<float> (SparseGEMM.h:121-149) on host arrays,
    computed by the GPU's fp32 rocBLAS product + bias/PReLU epilogue."""
    X = np.ascontiguousarray(X, dtype=np.float32)
    W = np.ascontiguousarray(W, dtype=np.float32)
    if X.ndim != 2 or W.ndim != 2 or X.shape[1] != W.shape[0]:
        raise TcscError(f"X {X.shape} and W {W.shape} do not chain")
    M, K = X.shape
    N = W.shape[1]
    b = np.ascontiguousarray(b, dtype=np.float32).reshape(-1)
    if b.size != N:
        raise TcscError(f"b has {b.size} elements, W has N={N} columns")
    Y = np.empty((M, N), np.float32)
    nz = lambda v: v.reshape(-1) if v.size else np.zeros(1, np.float32)  # noqa: E731
    if a is None:
        lib().tcsc_dense_gemm(nz(X), nz(W), nz(b), nz(Y), M, N, K)
    else:
        lib().tcsc_dense_gemm_prelu(nz(X), nz(W), nz(b), nz(Y), M, N, K, float(a))
    return Y


ORDERS = {"fast": 0, "reference": 1}


def set_order(order: str) -> None:
    """Summation order of plans created from now on (include/tcsc_gpu.h
    tcsc_order): "fast" (merged +1/-1, tolerance parity) or "reference"
    (each variant's own order: float outputs bit-identical to the reference)."""
    lib().tcsc_gpu_set_order(ORDERS[order])


def get_order() -> str:
    return {v: k for k, v in ORDERS.items()}[int(lib().tcsc_gpu_get_order())]


def set_num_shards(n: int) -> None:
    lib().tcsc_gpu_set_num_shards(int(n))


def num_shards() -> int:
    return int(lib().tcsc_gpu_num_shards())


def cache_clear() -> None:
    lib().tcsc_gpu_cache_clear()


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):  # torch tensor
        return int(x.data_ptr())
    raise TypeError(f"expected a device pointer or tensor, got {type(x)}")


class Plan:
    """Device plan for columns [col_begin, col_end) of W (include/tcsc_gpu.h)."""

    def __init__(self, W: TcscMatrix, col_begin: int = 0, col_end: int | None = None, device: int = 0,
                 stream: int = 0):
        col_end = W.cols if col_end is None else col_end
        h = C.c_void_p()
        _check(lib().tcsc_gpu_plan_create(W.ptr, col_begin, col_end, device, C.c_void_p(stream), C.byref(h)),
               "tcsc_gpu_plan_create")
        self.handle = h

    @classmethod
    def from_device(cls, rows, cols, csp, csn, rip, rin, col_begin=0, col_end=None, device=0, stream=0):
        self = cls.__new__(cls)
        col_end = cols if col_end is None else col_end
        h = C.c_void_p()
        _check(lib().tcsc_gpu_plan_create_device(rows, cols, C.c_void_p(_ptr(csp)), C.c_void_p(_ptr(csn)),
                                                 C.c_void_p(_ptr(rip)), C.c_void_p(_ptr(rin)), col_begin,
                                                 col_end, device, C.c_void_p(stream), C.byref(h)),
               "tcsc_gpu_plan_create_device")
        self.handle = h
        return self

    def info(self) -> dict:
        inf = plan_info_t()
        _check(lib().tcsc_gpu_plan_get_info(self.handle, C.byref(inf)), "tcsc_gpu_plan_get_info")
        return {k: getattr(inf, k) for k, _ in plan_info_t._fields_}

    def launch_info(self, M: int) -> tuple[str, int]:
        """(path, K slices) of a launch of M rows: path is 'gather' (k_transpose +
        k_stream), 'mfma' or 'small' (include/tcsc_gpu.h tcsc_gpu_launch_info; value 1,
        the retired persistent k_fused, is never returned)."""
        path, slices = C.c_int(), C.c_int()
        _check(lib().tcsc_gpu_launch_info(self.handle, int(M), C.byref(path), C.byref(slices)),
               "tcsc_gpu_launch_info")
        return ("gather", "fused", "mfma", "small")[path.value], slices.value

    def launch_combine(self, M: int) -> bool:
        """True when a gather launch of M rows combines its split-K slabs inside
        k_stream instead of a k_reduce launch (tcsc_gpu_launch_combine)."""
        return self.combine_mode(M) is not None

    def combine_mode(self, M: int):
        """How a gather launch of M rows combines its split-K slabs: 'pairwise'
        (2 slices, inside k_stream, any grid), 'pairwise-split' (2 slices, split
        halves, a resident grid), 'bands' (>= 3 slices, inside k_stream) or None
        (k_reduce4 after it, or no split) -- tcsc_gpu_launch_combine."""
        v = C.c_int()
        _check(lib().tcsc_gpu_launch_combine(self.handle, int(M), C.byref(v)), "tcsc_gpu_launch_combine")
        return {2: "bands", 3: "pairwise", 4: "pairwise-split"}.get(v.value)

    def reserve(self, max_M: int) -> None:
        """Allocate the workspace (X^T + split-K slabs) for launches of up to max_M rows."""
        _check(lib().tcsc_gpu_plan_reserve(self.handle, int(max_M)), "tcsc_gpu_plan_reserve")

    def sgemm(self, X, B, Y, M: int, ldy: int, variant: str = "prelu_basic", a: float = 0.2,
              stream: int = 0) -> None:
        _check(lib().tcsc_gpu_sgemm(self.handle, C.c_void_p(_ptr(X)), C.c_void_p(_ptr(B)), C.c_void_p(_ptr(Y)),
                                    int(M), int(ldy), VARIANT_ID[variant], float(a), C.c_void_p(stream)),
               "tcsc_gpu_sgemm")

    def prepare_x(self, X, M: int, stream: int = 0) -> None:
        """First half of sgemm: stage X^T in the plan's workspace (k_transpose)."""
        _check(lib().tcsc_gpu_prepare_x(self.handle, C.c_void_p(_ptr(X)), int(M), C.c_void_p(stream)),
               "tcsc_gpu_prepare_x")

    def sgemm_prepared(self, B, Y, M: int, ldy: int, variant: str = "prelu_basic", a: float = 0.2,
                       stream: int = 0) -> None:
        """Second half of sgemm: the gather on the staged X^T (k_stream)."""
        _check(lib().tcsc_gpu_sgemm_prepared(self.handle, C.c_void_p(_ptr(B)), C.c_void_p(_ptr(Y)), int(M), int(ldy),
                                             VARIANT_ID[variant], float(a), C.c_void_p(stream)),
               "tcsc_gpu_sgemm_prepared")

    def destroy(self) -> None:
        if getattr(self, "handle", None):
            lib().tcsc_gpu_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass


def dense_sgemm(X, Wd, B, Y, M: int, N: int, K: int, ldy: int, variant: str = "prelu_basic", a: float = 0.2,
                stream: int = 0) -> None:
    """Dense baseline on the device (gemm_basic, dense/dense.c:64-77): Y = act(X Wd + B), rocBLAS fp32 SGEMM
    plus the bias/PReLU epilogue kernel.  X, Wd, B, Y are device buffers (torch tensors or raw pointers)."""
    _check(lib().tcsc_gpu_dense_sgemm(C.c_void_p(_ptr(X)), C.c_void_p(_ptr(Wd)), C.c_void_p(_ptr(B)),
                                      C.c_void_p(_ptr(Y)), int(M), int(N), int(K), int(ldy), VARIANT_ID[variant],
                                      float(a), C.c_void_p(stream)), "tcsc_gpu_dense_sgemm")


def gpu_from_dense(d_dense, rows: int, cols: int, d_csp, d_csn, d_rip=None, d_rin=None, stream: int = 0):
    """Device tcsc_from_dense; returns (n_pos, n_neg)."""
    p, q = C.c_int(), C.c_int()
    _check(lib().tcsc_gpu_from_dense(C.c_void_p(_ptr(d_dense)), rows, cols, C.c_void_p(_ptr(d_csp)),
                                     C.c_void_p(_ptr(d_csn)), C.c_void_p(_ptr(d_rip)), C.c_void_p(_ptr(d_rin)),
                                     C.byref(p), C.byref(q), C.c_void_p(stream)), "tcsc_gpu_from_dense")
    return p.value, q.value
