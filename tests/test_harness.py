"""The native benchmark driver (harness/tcsc_bench) and the
out.txt -> CSV parser that replaces the stale parse-out2csv.sh.

CPU: the parser on a hand-written out.txt in main.cpp's layout
(main.cpp:190-196 header, :296 matrix info, :409-432 legacy lines), the
driver's CLI errors and its no-GPU exit.  GPU: a BASELINE config and the
reference's own cases through the driver, device and host API, checking
its validation, its records and that its stdout parses.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG

BIN = os.path.join(PKG, "bin", "tcsc_bench")
sys.path.insert(0, os.path.join(PKG, "harness"))
import out2csv  # noqa: E402

ALGOS = ("dense_gemm", "basic", "optimized", "prelu_basic", "prelu_separate", "prelu_onthego")
LEGACY = ("GEMM", "TCSC_basic", "TCSC_opt", "TCSC_PReLU_basic", "TCSC_PReLU_sep", "TCSC_PReLU_otg")

SAMPLE = """\
** banner **
[*] Overall Benchmark Progress [=====     ] 1/2
+----------------------------------------------------------------------+
|  [TEST 1/2] Matrix Size: 1x512x2048 (Sparsity: 50%)                 |
+----------------------------------------------------------------------+
[*] Matrix info: 524301 non-zeros out of 1048576 elements
[OK] All validation tests passed!
| TCSC Basic          |      123456 |     1050650 |     8.5100 |
GEMM         cycles=2000000, flops=2099200, performance=1.0496
TCSC_basic   cycles=123456, flops=1050650, performance=8.5100
TCSC_opt     cycles=223456, flops=1050650, performance=4.7018
TCSC_PReLU_basic cycles=130000, flops=1050650, performance=8.0819
TCSC_PReLU_sep   cycles=240000, flops=1050650, performance=4.3777
TCSC_PReLU_otg   cycles=230000, flops=1050650, performance=4.5680
|  [TEST 2/2] Matrix Size: 256x1024x4096 (Sparsity: 50%)               |
[*] Matrix info: 2097000 non-zeros out of 4194304 elements
GEMM         cycles=9e9, flops=2148532224, performance=0.2387
TCSC_basic   cycles=5000000, flops=1074741248, performance=214.9482
"""


def test_out2csv_parses_main_cpp_layout():
    algos, cases = out2csv.parse(SAMPLE.splitlines())
    assert algos == list(LEGACY)
    assert [(c["M"], c["K"], c["N"], c["nonZero"]) for c in cases] == [(1, 512, 2048, 524301),
                                                                        (256, 1024, 4096, 2097000)]
    csv = out2csv.to_csv(algos, cases).splitlines()
    head = csv[0].split(",")
    assert head[:4] == ["M", "K", "N", "nonZero"] and len(head) == 4 + 3 * len(LEGACY)
    row1 = dict(zip(head, csv[1].split(",")))
    assert row1["cycles_TCSC_PReLU_sep"] == "240000" and row1["performance_TCSC_basic"] == "8.5100"
    row2 = dict(zip(head, csv[2].split(",")))
    assert row2["cycles_GEMM"] == "9e9" and row2["flops_TCSC_opt"] == ""  # missing algorithm: empty cells


def test_out2csv_rejects_legacy_line_without_case():
    with pytest.raises(ValueError, match="before any test header"):
        out2csv.parse(["TCSC_basic   cycles=1, flops=2, performance=2.0000"])


def test_out2csv_cli(tmp_path):
    p = tmp_path / "out.txt"
    p.write_text(SAMPLE)
    r = subprocess.run([sys.executable, os.path.join(PKG, "harness", "out2csv.py"), str(p)], capture_output=True,
                       text=True, check=True)
    assert r.stdout.count("\n") == 3 and r.stdout.startswith("M,K,N,nonZero,cycles_GEMM")


def _bin():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-C", PKG, "harness"])
    return BIN


def test_driver_cli_errors_and_no_device_exit():
    b = _bin()
    r = subprocess.run([b, "--help"], capture_output=True, text=True)
    assert r.returncode == 0 and "--config 1..5" in r.stdout
    for bad in (["--shape", "1,2"], ["--config", "9"], ["--api", "cpu"], ["--bogus"], ["--no-dense"]):
        r = subprocess.run([b] + bad, capture_output=True, text=True)
        assert r.returncode == 2, bad
    import tcsc_amd

    if tcsc_amd.lib().tcsc_gpu_device_count() == 0:
        r = subprocess.run([b, "--config", "1"], capture_output=True, text=True)
        assert r.returncode == 2 and "no gfx950 device" in r.stderr


def _run(args, tmp_path, timeout=300):
    js, cs = tmp_path / "r.jsonl", tmp_path / "r.csv"
    r = subprocess.run([_bin()] + args + ["--json", str(js), "--csv", str(cs)], capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    recs = [json.loads(line) for line in js.read_text().splitlines()]
    rows = cs.read_text().splitlines()
    assert len(rows) == len(recs) + 1
    return r.stdout, recs


@pytest.mark.gpu
@pytest.mark.config_parity
def test_driver_baseline_config_device(tmp_path):
    out, recs = _run(["--config", "2", "--warmup", "2", "--reps", "5"], tmp_path)
    assert [r["algorithm"] for r in recs] == list(ALGOS)
    assert "[OK] All validation tests passed!" in out
    for r in recs:
        assert (r["M"], r["K"], r["N"]) == (1024, 4096, 4096)
        assert r["ms_median"] > 0 and r["ms_min"] <= r["ms_median"]
        if r["algorithm"] != "dense_gemm":
            assert r["worst_err_over_bound"] <= 1.0
            assert r["g_add_ops_per_s"] > 0 and 0 < r["hbm_frac"] < 1
            assert r["flops"] == 2 * 1024 * r["nnz"] + 1024 * 4096  # main.cpp:47-51
    algos, cases = out2csv.parse(out.splitlines())
    assert algos == list(LEGACY) and cases[0]["nonZero"] == recs[0]["nnz"]
    # the driver's W is the library generator's under the recorded seed
    # (X, then B, then W drawn from one stream): same nonzero count
    assert _library_nnz(recs[0]["seed"], 1024, 4096, 4096, 20) == recs[0]["nnz"]


def _library_nnz(seed, M, K, N, nz):
    import ctypes as C

    import tcsc_amd

    L = tcsc_amd.lib()
    libc = C.CDLL(None)
    for f in (L.init_rand_dense, L.init_rand_sparse):
        f.restype = C.c_void_p
    L.tcsc_set_seed(seed)
    ptrs = [L.init_rand_dense(M, K), L.init_rand_dense(N, 1), L.init_rand_sparse(K, N, nz)]
    W = np.ctypeslib.as_array(C.cast(ptrs[2], C.POINTER(C.c_float)), shape=(K * N,))
    nnz = int(np.count_nonzero(W))
    libc.free.argtypes = [C.c_void_p]
    for p in ptrs:
        libc.free(p)
    return nnz


@pytest.mark.gpu
@pytest.mark.config_parity
def test_driver_reference_cases_host_api(tmp_path):
    """main.cpp's five cases through the drop-in host-pointer API, timed with
    the reference protocol (shortened): what benchmark.sh would run."""
    out, recs = _run(["--api", "host", "--num-runs", "1", "--rep", "2", "--cycles-required", "0"], tmp_path)
    algos, cases = out2csv.parse(out.splitlines())
    assert [(c["M"], c["K"], c["N"]) for c in cases] == [(1, 512, 2048), (1, 1024, 4096), (1, 2048, 8192),
                                                         (256, 512, 2048), (256, 1024, 4096)]
    assert algos == list(LEGACY)
    assert len(recs) == 5 * len(ALGOS) and all(r["api"] == "host" for r in recs)
    nnz = np.array([c["nonZero"] for c in cases], dtype=np.float64)
    dens = nnz / np.array([c["K"] * c["N"] for c in cases])
    assert np.all(np.abs(dens - 0.5) < 0.01)  # init_rand_sparse(K, N, 2), main.cpp:278


@pytest.mark.gpu
def test_driver_reference_order(tmp_path):
    out, recs = _run(["--shape", "64,3000,700,20", "--order", "reference", "--warmup", "1", "--reps", "3"], tmp_path)
    assert all(r["order"] == "reference" for r in recs)
    assert all(r["worst_err_over_bound"] <= 1.0 for r in recs if r["algorithm"] != "dense_gemm")
