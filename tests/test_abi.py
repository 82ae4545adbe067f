"""The drop-in boundary, checked without a GPU: the C-ABI library loads and
exports every symbol include/*.h declares, the headers are valid C and C++,
and the host-side format builder is bit-exact with the reference."""
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN_NAMES, PKG, ROOT, load_golden, tcsc_of

import tcsc_amd


@pytest.fixture(scope="module")
def built_lib():
    tcsc_amd.build()
    return tcsc_amd.lib()


def declared_functions():
    names = set()
    for h in ("include/sparse/tcsc.h", "include/dense/dense.h", "include/tcsc_gpu.h", "include/sparse/bcsr.h",
              "include/bcsr_gpu.h", "include/sparse_gemm.h"):
        src = open(os.path.join(ROOT, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", src):
            name = m.group(1)
            if name not in ("if", "sizeof", "defined") and not name.isupper():
                names.add(name)
    return names


def test_every_declared_symbol_is_exported(built_lib):
    declared = declared_functions()
    assert declared == set(tcsc_amd.EXPORTED_SYMBOLS), declared ^ set(tcsc_amd.EXPORTED_SYMBOLS)
    out = subprocess.check_output(["nm", "-D", "--defined-only", tcsc_amd.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    missing = declared - exported
    assert not missing, missing
    for name in declared:
        assert hasattr(built_lib, name)


def test_reference_signatures_have_c_linkage():
    """main.cpp's function-pointer types (main.cpp:54,116) bind to these
    unmangled symbols when recompiled against include/."""
    out = subprocess.check_output(["nm", "-D", "--defined-only", tcsc_amd.LIB_PATH], text=True)
    for s in ("tcsc_sgemm_basic", "tcsc_sgemm_prelu_optimized_onthego", "tcsc_from_dense", "tcsc_free"):
        assert re.search(rf"\bT {s}$", out, re.M), s


HEADER_PROBE = r"""
#include <sparse/tcsc.h>
#include <tcsc_gpu.h>
#include <sparse/bcsr.h>
#include <bcsr_gpu.h>
#include <sparse_gemm.h>
typedef void (*gemm_fn)(const dense_t, const tcsc_t *, const dense_t, dense_t, int, int, int);
typedef void (*prelu_fn)(const dense_t, const tcsc_t *, const dense_t, float, dense_t, int, int, int);
typedef void (*bgemm_fn)(const dense_t, const bcsr_t, const dense_t, dense_t, int, int, int);
typedef void (*bprelu_fn)(const dense_t, const bcsr_t, const dense_t, float, dense_t, int, int, int);
int main(void) {
    gemm_fn g[2] = {tcsc_sgemm_basic, tcsc_sgemm_optimized};
    prelu_fn p[3] = {tcsc_sgemm_prelu_basic, tcsc_sgemm_prelu_optimized_separate,
                     tcsc_sgemm_prelu_optimized_onthego};
    bgemm_fn bg[3] = {bcsr_sgemm_basic, bcsr_sgemm_avx, bcsr_sgemm_avx2};
    bprelu_fn bp[2] = {bcsr_sgemm_prelu_basic, bcsr_sgemm_prelu_avx};
    void (*sg)(const float *, const int *, const int *, const int *, const int *, const float *, float *,
               int, int, int) = tcsc_sparse_gemm;
    void (*dg)(const float *, const float *, const float *, float *, int, int, int, float) =
        tcsc_dense_gemm_prelu;
    tcsc_gpu_plan_info info;
    (void)info; (void)g; (void)p; (void)bg; (void)bp; (void)sg; (void)dg;
    return tcsc_gpu_device_count() < 0;
}
"""


@pytest.mark.parametrize("lang", ["c", "c++"])
def test_headers_compile_and_link(tmp_path, built_lib, lang):
    src = tmp_path / ("probe.c" if lang == "c" else "probe.cpp")
    src.write_text(HEADER_PROBE)
    exe = tmp_path / "probe"
    cc = "gcc" if lang == "c" else "g++"
    std = "-std=c99" if lang == "c" else "-std=c++17"
    subprocess.check_call([cc, std, "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o",
                           str(exe), "-L", os.path.dirname(tcsc_amd.LIB_PATH), "-ltcsc_amd",
                           "-Wl,-rpath," + os.path.dirname(tcsc_amd.LIB_PATH)])
    assert exe.exists()


@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_host_tcsc_from_dense_bitexact(built_lib, name, monkeypatch):
    monkeypatch.setenv("TCSC_BUILDER", "host")
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    ref = tcsc_of(g)
    got = W.arrays()
    for a, b in zip(got, ref.arrays()):
        np.testing.assert_array_equal(a, b)
    assert W.rows == ref.rows and W.cols == ref.cols
    W.free()


def test_device_count_without_gpu_is_zero_or_more(built_lib):
    assert tcsc_amd.device_count() >= 0


def test_product_library_is_not_a_diagnostic_build(built_lib):
    """tcsc_gpu_build_flags() is 0 for the product build; tcsc_amd refuses a
    nonzero one (the timing-only ablation / stamps / trace builds of
    tools/ab.mk) unless TCSC_ALLOW_DIAG=1."""
    assert built_lib.tcsc_gpu_build_flags() == 0
    src = open(os.path.join(PKG, "tcsc_amd", "__init__.py")).read()
    assert 'os.environ.get("TCSC_ALLOW_DIAG") != "1"' in src


def test_plan_create_rejects_bad_range(built_lib):
    g = load_golden("cfg1")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.Plan(W, 10, 5)
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.Plan(W, 0, W.cols + 1)


def test_gpu_entry_points_fail_loudly_without_device(built_lib):
    if tcsc_amd.device_count() > 0:
        pytest.skip("GPU present")
    g = load_golden("cfg1")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.Plan(W)
    # host-pointer API: no silent CPU fallback -- it reports and aborts
    code = (
        "import sys, numpy as np; sys.path.insert(0, %r); import tcsc_amd;"
        "W = tcsc_amd.TcscMatrix.from_dense(np.eye(4, dtype=np.float32));"
        "tcsc_amd.sgemm('basic', np.ones((2,4),np.float32), W, np.zeros(4,np.float32))" % PKG
    )
    r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode != 0
    assert "no HIP device" in r.stderr


# g++ (Itanium ABI) names the reference harness's objects reference: the
# reference compiles its .c files as C++ without extern "C" (SURVEY.md §8b,
# "Linkage"), so a link-level drop-in must export exactly these.
REFERENCE_MANGLED = {
    "_Z15tcsc_from_densePfii": "tcsc_from_dense",
    "_Z16tcsc_sgemm_basicPfPK6tcsc_tS_S_iii": "tcsc_sgemm_basic",
    "_Z20tcsc_sgemm_optimizedPfPK6tcsc_tS_S_iii": "tcsc_sgemm_optimized",
    "_Z22tcsc_sgemm_prelu_basicPfPK6tcsc_tS_fS_iii": "tcsc_sgemm_prelu_basic",
    "_Z35tcsc_sgemm_prelu_optimized_separatePfPK6tcsc_tS_fS_iii": "tcsc_sgemm_prelu_optimized_separate",
    "_Z34tcsc_sgemm_prelu_optimized_onthegoPfPK6tcsc_tS_fS_iii": "tcsc_sgemm_prelu_optimized_onthego",
    "_Z9tcsc_freeP6tcsc_t": "tcsc_free",
    "_Z15init_rand_denseii": "init_rand_dense",
    "_Z16init_rand_sparseiii": "init_rand_sparse",
    "_Z7comparePfS_ii": "compare",
    "_Z10gemm_basicPfS_S_S_iii": "gemm_basic",
    # sparse/bcsr.h:14-39 (bcsr_t by value), linked by test/test_bcsr.cpp
    "_Z15bcsr_from_densePfiiii": "bcsr_from_dense",
    "_Z16bcsr_sgemm_basicPf6bcsr_tS_S_iii": "bcsr_sgemm_basic",
    "_Z22bcsr_sgemm_prelu_basicPf6bcsr_tS_fS_iii": "bcsr_sgemm_prelu_basic",
    "_Z14bcsr_sgemm_avxPf6bcsr_tS_S_iii": "bcsr_sgemm_avx",
    "_Z20bcsr_sgemm_prelu_avxPf6bcsr_tS_fS_iii": "bcsr_sgemm_prelu_avx",
    "_Z15bcsr_sgemm_avx2Pf6bcsr_tS_S_iii": "bcsr_sgemm_avx2",
}


def test_reference_mangled_names_are_exported(built_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", tcsc_amd.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = sorted(set(REFERENCE_MANGLED) - exported)
    assert not missing, missing


def test_mangled_aliases_forward_to_c_entry_points(built_lib, monkeypatch):
    """The C++-ABI alias of tcsc_from_dense builds the same TCSC as the C
    name (host builder: no GPU), and compare() agrees."""
    import ctypes

    monkeypatch.setenv("TCSC_BUILDER", "host")
    lib = ctypes.CDLL(tcsc_amd.LIB_PATH)
    g = load_golden("cfg1")
    Wd = np.ascontiguousarray(g["Wd"].astype(np.float32))
    fp = ctypes.POINTER(ctypes.c_float)
    K, N = Wd.shape
    f_c = lib.tcsc_from_dense
    f_x = getattr(lib, "_Z15tcsc_from_densePfii")
    for f in (f_c, f_x):
        f.restype = ctypes.c_void_p
        f.argtypes = [fp, ctypes.c_int, ctypes.c_int]
    pc = f_c(Wd.ctypes.data_as(fp), K, N)
    px = f_x(Wd.ctypes.data_as(fp), K, N)
    assert pc and px

    class T(ctypes.Structure):
        _fields_ = [("rows", ctypes.c_int), ("cols", ctypes.c_int), ("n_pos", ctypes.c_int), ("n_neg", ctypes.c_int),
                    ("csp", ctypes.POINTER(ctypes.c_int)), ("csn", ctypes.POINTER(ctypes.c_int)),
                    ("rip", ctypes.POINTER(ctypes.c_int)), ("rin", ctypes.POINTER(ctypes.c_int))]

    a, b = T.from_address(pc), T.from_address(px)
    assert (a.rows, a.cols, a.n_pos, a.n_neg) == (b.rows, b.cols, b.n_pos, b.n_neg)
    assert np.array_equal(np.ctypeslib.as_array(a.rip, (a.n_pos,)), np.ctypeslib.as_array(b.rip, (b.n_pos,)))
    assert np.array_equal(np.ctypeslib.as_array(a.rin, (a.n_neg,)), np.ctypeslib.as_array(b.rin, (b.n_neg,)))
    free_x = getattr(lib, "_Z9tcsc_freeP6tcsc_t")
    free_x.argtypes = [ctypes.c_void_p]
    free_x(px)
    lib.tcsc_free.argtypes = [ctypes.c_void_p]
    lib.tcsc_free(pc)
    cmp_x = getattr(lib, "_Z7comparePfS_ii")
    cmp_x.restype = ctypes.c_bool
    cmp_x.argtypes = [fp, fp, ctypes.c_int, ctypes.c_int]
    y = np.ones((3, 5), np.float32)
    z = y.copy()
    assert cmp_x(y.ctypes.data_as(fp), z.ctypes.data_as(fp), 3, 5)
    z[1, 2] += 1e-3
    assert not cmp_x(y.ctypes.data_as(fp), z.ctypes.data_as(fp), 3, 5)


def test_python_sgemm_checks_shapes_before_the_library(built_lib):
    """The C entry points trust M, N, K as the reference's do; the Python
    mirror raises on a mismatch instead of letting a short B or Y reach them."""
    W = tcsc_amd.TcscMatrix.from_dense(np.eye(6, 5, dtype=np.float32))
    X = np.ones((3, 6), np.float32)
    with pytest.raises(tcsc_amd.TcscError, match="B has"):
        tcsc_amd.sgemm("basic", X, W, np.zeros(4, np.float32))
    with pytest.raises(tcsc_amd.TcscError, match="Y must be"):
        tcsc_amd.sgemm("basic", X, W, np.zeros(5, np.float32), Y=np.zeros((3, 4), np.float32))
    with pytest.raises(tcsc_amd.TcscError, match="Y must be"):
        tcsc_amd.sgemm("basic", X, W, np.zeros(5, np.float32), Y=np.zeros((3, 5), np.float64))
    with pytest.raises(tcsc_amd.TcscError, match="K=7"):
        tcsc_amd.sgemm("basic", np.ones((3, 7), np.float32), W, np.zeros(5, np.float32))
    with pytest.raises(tcsc_amd.TcscError, match="unknown variant"):
        tcsc_amd.sgemm("fast", X, W, np.zeros(5, np.float32))
    W.free()


def test_hand_built_tcsc_round_trips_and_plan_build_validates_rows(built_lib, oracle):
    """TcscMatrix.from_arrays (a malloc'd tcsc_t, freed by tcsc_free) keeps the
    arrays; the plan build rejects a row outside [0, K) before touching a
    device (the reference would read outside X)."""
    Wd = oracle.ternary((40, 9), 0.2, 3)
    ref = oracle.tcsc_from_dense(Wd)
    W = tcsc_amd.TcscMatrix.from_arrays(40, 9, *ref.arrays())
    for a, b in zip(W.arrays(), ref.arrays()):
        np.testing.assert_array_equal(a, b)
    W.free()
    rip = ref.row_index_pos.copy()
    rip[0] = 40
    bad = tcsc_amd.TcscMatrix.from_arrays(40, 9, ref.col_start_pos, ref.col_start_neg, rip, ref.row_index_neg)
    with pytest.raises(tcsc_amd.TcscError, match="outside"):
        tcsc_amd.Plan(bad)
    bad.free()
    csn = ref.col_start_neg.copy()
    csn[3], csn[4] = csn[4] + 1, csn[3]  # a decreasing col_start
    bad = tcsc_amd.TcscMatrix.from_arrays(40, 9, ref.col_start_pos, csn, ref.row_index_pos, ref.row_index_neg)
    with pytest.raises(tcsc_amd.TcscError, match="col_start_neg"):
        tcsc_amd.Plan(bad)
    bad.free()


@pytest.mark.parametrize("M,K,N,threads", [(1, 512, 2048, None), (37, 300, 129, "1"), (256, 512, 700, "0"),
                                           (64, 300, 200, "3")])
def test_gemm_basic_bit_identical_to_reference(built_lib, oracle, M, K, N, threads, monkeypatch):
    """dense/dense.h gemm_basic -- the harness's dense oracle (dense.c:64-77),
    a CPU function of the library -- against the reference's own gemm_basic
    (compiled in place, IEEE): same bits, single-threaded (the default, as the
    reference) and on the opt-in threaded path ($TCSC_DENSE_THREADS; a row of
    accumulators, k ascending per element)."""
    import pyoracle

    if threads is None:
        monkeypatch.delenv("TCSC_DENSE_THREADS", raising=False)
    else:
        monkeypatch.setenv("TCSC_DENSE_THREADS", threads)

    ref = pyoracle.load_reference()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    X = oracle.uniform((M, K), 301 + M)
    Wd = oracle.ternary((K, N), 0.5, 302 + M)
    Wd[0, :3] = [0.5, -2.0, 3.0]  # gemm_basic multiplies whatever W holds
    B = oracle.uniform((N,), 303 + M)
    import ctypes as C

    Y = np.empty((M, N), np.float32)
    f = built_lib.gemm_basic
    fp = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
    f.argtypes, f.restype = [fp, fp, fp, fp, C.c_int, C.c_int, C.c_int], None
    f(X.reshape(-1), np.ascontiguousarray(Wd).reshape(-1), B, Y.reshape(-1), M, N, K)
    np.testing.assert_array_equal(Y.view(np.uint32), ref.gemm_basic(X, Wd, B).view(np.uint32))


@pytest.mark.parametrize("binary", ["main_amd", "main_amd_rv"])
def test_main_amd_links_reference_dense(binary):
    """oracle/_ref/main_amd[_rv] (the reference's unmodified main.cpp) carries
    the reference's own dense/dense.c: gemm_basic, compare and the init_rand_*
    generators are defined in the executable, so only the tcsc_* entry points
    resolve to libtcsc_amd.so (VERDICT r3 "What's missing" #2).  main_amd_rv
    also carries oracle/harness_wrap.cpp's two --wrap hooks."""
    exe = os.path.join(ROOT, "oracle", "_ref", binary)
    if not os.path.exists(exe):
        pytest.skip(f"oracle/_ref/{binary} not built here (needs /root/reference: make -C oracle harness)")
    out = subprocess.run(["nm", "-C", exe], capture_output=True, text=True, check=True).stdout
    kind = {}
    for line in out.splitlines():
        parts = line.split(None, 2) if line[:1] != " " else ["", *line.split(None, 1)]
        if len(parts) == 3:
            kind[parts[2].split("(")[0]] = parts[1]
    for name in ("gemm_basic", "compare", "init_rand_dense", "init_rand_sparse"):
        if name == "gemm_basic" and binary == "main_amd_rv":
            continue  # nm -C folds dense.c's C++ gemm_basic and the library's C one (the timing calls)
        assert kind.get(name) == "T", (name, kind.get(name))
    for name in ("tcsc_from_dense", "tcsc_sgemm_basic", "tcsc_sgemm_optimized", "tcsc_sgemm_prelu_basic",
                 "tcsc_sgemm_prelu_optimized_separate", "tcsc_sgemm_prelu_optimized_onthego", "tcsc_free"):
        assert kind.get(name) == "U", (name, kind.get(name))
    if binary == "main_amd_rv":
        raw = subprocess.run(["nm", exe], capture_output=True, text=True, check=True).stdout
        for sym in ("_Z10gemm_basicPfS_S_S_iii", "__wrap__Z10gemm_basicPfS_S_S_iii", "__wrap__Z15tcsc_from_densePfii"):
            assert f" T {sym}" in raw, sym
