"""The SparseGEMM.h drop-in: include/SparseGEMM.h
and the raw-array C ABI behind it (include/sparse_gemm.h).

CPU: SparseFormat (tcsc_sparse_format) is bit-exact with the reference's
SparseFormat (golden fixture and the oracle, values beyond +-1 included); the
header compiles for T = float and refuses other T; a C++ program using the
header builds, links and runs its host part; the compute entry points abort
loudly without a GPU.

GPU: sparseGEMM / sparseGEMM_PReLU against every golden fixture's
Y_sparsegemm* (the reference's SparseGEMM.h compiled in place,
tests/golden/gen_golden.py): within the fp32 bound in the fast order, bit for
bit in the reference order and on integer inputs; GEMM / GEMM_PReLU against
the fixtures' Y_gemm*; the raw-array plan cache (in-place rebuild, eviction);
and the reference's own SparseGEMM.cpp harness compiled against this header
(oracle/Makefile `harness`).
"""
import os
import subprocess

import numpy as np
import pytest

import pyoracle
import tcsc_amd
from conftest import GOLDEN_NAMES, PKG, ROOT, load_golden, tcsc_of

INC = os.path.join(ROOT, "include")
LIBDIR = os.path.join(PKG, "lib")


@pytest.fixture(scope="module")
def built_lib():
    tcsc_amd.build()
    return tcsc_amd.lib()


# --- CPU -------------------------------------------------------------------

def test_sparse_format_matches_reference_fixture(built_lib):
    g = load_golden("sparseformat_48x40")
    got = tcsc_amd.sparse_format(g["mat"])
    for a, k in zip(got, ("csp", "csn", "rip", "rin")):
        np.testing.assert_array_equal(a, g[k], err_msg=k)


@pytest.mark.parametrize("shape,seed", [((1, 1), 0), ((37, 53), 1), ((256, 300), 2), ((0, 5), 3), ((7, 0), 4)])
def test_sparse_format_matches_oracle(built_lib, oracle, shape, seed):
    """Thresholds >= 1 / <= -1 (SparseGEMM.h:27-33): 2 and -7 count too."""
    mat = np.random.default_rng(seed).integers(-3, 4, size=shape).astype(np.int32)
    mat[np.random.default_rng(seed + 9).random(shape) < 0.6] = 0
    got = tcsc_amd.sparse_format(mat)
    ref = oracle.sparseformat(mat) if mat.size else None
    if ref is None:
        assert got[0].tolist() == [0] * (shape[1] + 1) and got[2].size == 0 and got[3].size == 0
        return
    for a, b in zip(got, ref.arrays()):
        np.testing.assert_array_equal(a, b)


def _compile(tmp_path, src, name, extra=()):
    p = tmp_path / (name + ".cpp")
    p.write_text(src)
    exe = tmp_path / name
    cmd = ["g++", "-std=c++17", "-Wall", "-Werror", "-I", INC, str(p), "-o", str(exe), "-L", LIBDIR, "-ltcsc_amd",
           "-Wl,-rpath," + LIBDIR, *extra]
    return subprocess.run(cmd, capture_output=True, text=True), exe


PROGRAM = r"""
#include "SparseGEMM.h"
// SparseGEMM.cpp:36-49 deduces these function-pointer types from the templates
template <typename... Args> void* take(void (*f)(Args...)) { return (void*)f; }
int main() {
    vector<int> W = generateSparseMatrix<int>(64, 48, 4, false);
    vector<int> U = generateSparseMatrix<int>(16, 48, 4, true);
    vector<float> X = initX<float>(3 * 64, 512);
    for (float x : X) if (x < -512 || x > 512 || x != (int)x) return 3;
    SparseFormat sf(W.data(), 64, 48);
    long nz = 0;
    for (int v : W) nz += (v != 0);
    if ((long)(sf.row_index_pos.size() + sf.row_index_neg.size()) != nz) return 4;
    long nu = 0;
    for (int v : U) nu += (v != 0);
    if (nu != 16 * 48 / 4) return 5;  // one +1 and one -1 per 8-wide window
    float Y[2] = {1.0f, 2.0f}, Z[2] = {1.0f, 2.0f + 5e-6f}, Q[2] = {1.0f, 2.1f};
    if (!compare_results(Y, Z, 1, 2) || compare_results(Y, Q, 1, 2)) return 6;
    void* fp[4] = {take<float*, int*, int*, int*, int*, float*, float*, int, int, int>(sparseGEMM),
                   take<float*, float*, float*, float*, int, int, int>(GEMM),
                   take<float*, float*, float*, float*, int, int, int, float>(GEMM_PReLU),
                   take<float*, int*, int*, int*, int*, float*, float*, int, int, int, float>(sparseGEMM_PReLU)};
    for (void* p : fp) if (!p) return 7;
    for (int n = 0; n < 48; ++n) cout << sf.col_start_pos[n + 1] - sf.col_start_pos[n] << ' ';
    cout << endl;
    return 0;
}
"""


def test_header_compiles_links_and_runs_host_part(tmp_path, built_lib):
    r, exe = _compile(tmp_path, PROGRAM, "prog")
    assert r.returncode == 0, r.stderr
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, (out.returncode, out.stdout, out.stderr)
    lines = out.stdout.splitlines()
    assert lines[0].startswith("Error at: H=0, W=1"), lines  # the failing compare_results prints first
    assert len(lines[-1].split()) == 48


def test_header_refuses_non_float(tmp_path, built_lib):
    src = r"""
#include "SparseGEMM.h"
int main() {
    double x[1] = {0}, b[1] = {0}, y[1];
    int cs[2] = {0, 0}, ri[1] = {0};
    sparseGEMM(x, cs, cs, ri, ri, b, y, 1, 1, 1);
}
"""
    r, _ = _compile(tmp_path, src, "dbl")
    assert r.returncode != 0
    assert "fp32" in r.stderr


def test_entry_points_fail_loudly_without_device(built_lib):
    if tcsc_amd.device_count() > 0:
        pytest.skip("GPU present")
    for call in ("tcsc_amd.sparse_gemm(np.ones((2,4),np.float32), [0,1,1], [0,0,1], [0], [3], np.zeros(2,np.float32))",
                 "tcsc_amd.dense_gemm(np.ones((2,4),np.float32), np.ones((4,3),np.float32), np.zeros(3,np.float32))"):
        code = "import sys, numpy as np; sys.path.insert(0, %r); import tcsc_amd; %s" % (PKG, call)
        r = subprocess.run(["python", "-c", code], capture_output=True, text=True, timeout=120)
        assert r.returncode != 0, call
        assert "no HIP device" in r.stderr, r.stderr


def test_python_wrapper_checks_shapes(built_lib):
    X = np.ones((2, 4), np.float32)
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.sparse_gemm(X, [0, 1, 1], [0, 0, 1], [0], [3], np.zeros(3, np.float32))  # b has N+1
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.sparse_gemm(X, [0, 1, 2], [0, 0, 1], [0], [3], np.zeros(2, np.float32))  # rip too short
    with pytest.raises(tcsc_amd.TcscError):
        tcsc_amd.dense_gemm(X, np.ones((3, 3), np.float32), np.zeros(3, np.float32))


# --- GPU -------------------------------------------------------------------

@pytest.fixture(scope="module")
def gpu(built_lib):
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return built_lib


def _bits(Y, ref, what):
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(Y), nan), what
    np.testing.assert_array_equal(Y[~nan].view(np.uint32), ref[~nan].view(np.uint32), err_msg=what)


def _arrays(g):
    return g["csp"], g["csn"], g["rip"], g["rin"]


@pytest.mark.gpu
@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_sparse_gemm_fast_order_within_bound(gpu, oracle, name):
    g = load_golden(name)
    a = float(g["a"])
    Y64, S64 = oracle.f64_rows(g["X"], tcsc_of(g), g["B"])
    fin = np.isfinite(Y64)
    for prelu in (False, True):
        Y = tcsc_amd.sparse_gemm(g["X"], *_arrays(g), g["B"], a if prelu else None)
        ref = g["Y_sparsegemm_prelu" if prelu else "Y_sparsegemm"]
        ok, worst = pyoracle.check_close(Y[fin], Y64[fin], S64[fin], a if prelu else None)
        assert ok, (name, prelu, worst)
        assert np.array_equal(np.isnan(Y[~fin]), np.isnan(ref[~fin])), (name, prelu)
        if g["meta"]["kind"] == "int":
            _bits(Y, ref, f"{name}/{prelu}")


@pytest.mark.gpu
@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_sparse_gemm_reference_order_bit_exact(gpu, name):
    """TCSC_ORDER_REFERENCE: y = 0 + sum(+1) - sum(-1) + b in SparseGEMM.h's
    loop order, so the float outputs equal the reference's bit for bit."""
    g = load_golden(name)
    tcsc_amd.set_order("reference")
    tcsc_amd.cache_clear()
    try:
        _bits(tcsc_amd.sparse_gemm(g["X"], *_arrays(g), g["B"]), g["Y_sparsegemm"], name)
        _bits(tcsc_amd.sparse_gemm(g["X"], *_arrays(g), g["B"], float(g["a"])), g["Y_sparsegemm_prelu"], name)
    finally:
        tcsc_amd.set_order("fast")
        tcsc_amd.cache_clear()


@pytest.mark.gpu
@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_dense_gemm_matches_reference_gemm(gpu, name):
    g = load_golden(name)
    X, Wd, B, a = g["X"], g["Wd"].astype(np.float32), g["B"], float(g["a"])
    S = np.abs(B.astype(np.float64)) + np.abs(X.astype(np.float64)) @ np.abs(Wd.astype(np.float64))
    for prelu in (False, True):
        Y = tcsc_amd.dense_gemm(X, Wd, B, a if prelu else None)
        ref = g["Y_gemm_prelu" if prelu else "Y_gemm"]
        fin = np.isfinite(ref) & np.isfinite(S)
        bound = max(1.0, a) * 2.0 ** -19 * S[fin] + 1e-30
        assert np.all(np.abs(Y[fin].astype(np.float64) - ref[fin]) <= bound), (name, prelu)


@pytest.mark.gpu
def test_raw_cache_sees_in_place_rebuild_and_evicts(gpu, oracle):
    rng = np.random.default_rng(7)
    K, N, M = 96, 80, 5
    X = rng.integers(-50, 50, size=(M, K)).astype(np.float32)
    B = rng.integers(-5, 5, size=N).astype(np.float32)

    def mat(seed):
        m = np.random.default_rng(seed).integers(-1, 2, size=(K, N)).astype(np.int32)
        m[np.random.default_rng(seed + 1).random((K, N)) < 0.7] = 0
        return m

    def expect(csp, csn, rip, rin):
        return oracle.sgemm("optimized", X, pyoracle.TCSC(K, N, csp, csn, rip, rin), B)

    arrs = [list(tcsc_amd.sparse_format(mat(s))) for s in range(11)]
    first = arrs[0]
    np.testing.assert_array_equal(tcsc_amd.sparse_gemm(X, *first, B), expect(*first))
    # rebuild the row indices in place (same nnz, same buffers): the next call must see it
    rip = first[2]
    if rip.size > 1:
        rip[[0, -1]] = (rip[0] + 1) % K, (rip[-1] + 3) % K
        c = first[0]
        for n in range(N):  # keep every column ascending
            rip[c[n]:c[n + 1]] = np.sort(rip[c[n]:c[n + 1]])
    np.testing.assert_array_equal(tcsc_amd.sparse_gemm(X, *first, B), expect(*first))
    # more distinct matrices than the cache keeps, then the first again
    for a in arrs[1:]:
        np.testing.assert_array_equal(tcsc_amd.sparse_gemm(X, *a, B), expect(*a))
    np.testing.assert_array_equal(tcsc_amd.sparse_gemm(X, *first, B), expect(*first))


@pytest.mark.gpu
def test_reference_sparsegemm_harness_passes(gpu):
    """The reference's SparseGEMM.cpp, unmodified, compiled against
    include/SparseGEMM.h (oracle/Makefile `harness`): all 27 cases validate
    sparseGEMM(_PReLU) against GEMM(_PReLU) with its own compare_results."""
    exe = os.path.join(ROOT, "oracle", "_ref", "sparsegemm_amd")
    if not os.path.exists(exe):
        pytest.skip("oracle/_ref/sparsegemm_amd not built (needs /root/reference at build time)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count("M=") == 27, r.stdout[-2000:]
    assert "not passed" not in r.stdout, r.stdout[-4000:]
    assert r.stdout.count("sGEMM_PReLU cycles=") == 27


@pytest.mark.gpu
@pytest.mark.config_parity
@pytest.mark.parametrize("seed", range(6))
def test_raw_api_matches_device_plan_and_oracle(gpu, oracle, seed, monkeypatch):
    """Seeded random shapes: the raw host API (SparseGEMM.h path) against the
    device API with TCSC_VARIANT_SPARSE_GEMM (bit for bit: the host API's
    exact mode is the device API's gather with K unsplit) and against the
    fp64 oracle (bound); integer inputs bit-exact with the oracle's a8
    restatement (SparseGEMM.h:104-119)."""
    import torch

    monkeypatch.delenv("TCSC_HOST_FAST", raising=False)
    monkeypatch.setenv("TCSC_PATH", "gather")
    monkeypatch.setenv("TCSC_SLICES", "1")

    rng = np.random.default_rng(1000 + seed)
    M = int(rng.choice([1, 3, 17, 64, 300, 1024]))
    K = int(rng.integers(1, 3000))
    N = int(rng.integers(1, 700))
    dens = float(rng.choice([0.01, 0.05, 0.3]))
    mat = rng.random((K, N))
    mat = np.where(mat < dens / 2, 1, np.where(mat < dens, -1, 0)).astype(np.int32)
    csp, csn, rip, rin = tcsc_amd.sparse_format(mat)
    W = pyoracle.TCSC(K, N, csp, csn, rip, rin)
    integer = seed % 2 == 1
    X = (rng.integers(-512, 513, size=(M, K)) if integer else rng.uniform(-1, 1, size=(M, K))).astype(np.float32)
    B = (rng.integers(-8, 9, size=N) if integer else rng.uniform(-1, 1, size=N)).astype(np.float32)
    Y = tcsc_amd.sparse_gemm(X, csp, csn, rip, rin, B)
    Yp = tcsc_amd.sparse_gemm(X, csp, csn, rip, rin, B, 0.2)
    Y64, S64 = oracle.f64_rows(X, W, B)
    assert pyoracle.check_close(Y, Y64, S64)[0]
    assert pyoracle.check_close(Yp, Y64, S64, 0.2)[0]
    if integer:
        _bits(Y, oracle.sparse_gemm_omp(X, W, B, False), "int")
        _bits(Yp, oracle.sparse_gemm_omp(X, W, B, True, 0.2), "int prelu")
    dev = torch.device("cuda:0")
    plan = tcsc_amd.Plan(tcsc_amd.TcscMatrix.from_arrays(K, N, csp, csn, rip, rin))
    plan.reserve(M)
    Xd, Bd = torch.from_numpy(X).to(dev), torch.from_numpy(B).to(dev)
    Yd = torch.empty((M, N), device=dev)
    for variant, ref in (("sparse_gemm", Y), ("prelu_basic", Yp)):
        plan.sgemm(Xd, Bd, Yd, M, N, variant, 0.2)
        torch.cuda.synchronize()
        _bits(Yd.cpu().numpy(), ref, variant)
    plan.destroy()
