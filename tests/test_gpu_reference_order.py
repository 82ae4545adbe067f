"""TCSC_ORDER_REFERENCE: every variant summed in the reference's own order,
so float outputs equal the reference's bit for bit.

The golden fixtures hold the reference's outputs (sparse/tcsc.c compiled in
place with IEEE flags: oracle/Makefile, tests/golden/gen_golden.py).  In the
reference order the GPU must reproduce each of them exactly -- float inputs
included -- for all five variants (tcsc.c:84-93 basic, :113-137 optimized,
:149-161 prelu_basic, :184-226 prelu_optimized_separate, :244-273
prelu_optimized_onthego).  NaN payloads are the one exception (x86's default
NaN is negative, gfx950's positive), so the specials fixture compares NaN
positions and everything else bit for bit.  At the BASELINE sizes, sampled
rows are compared with the C oracle, which restates each variant's order.
"""
import numpy as np
import pytest

import pyoracle
import tcsc_amd
from conftest import GOLDEN_NAMES, load_golden, tcsc_of
from tcsc_amd import workloads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    tcsc_amd.set_num_shards(0)
    return tcsc_amd.lib()


@pytest.fixture
def reference_order(gpu):
    tcsc_amd.set_order("reference")
    tcsc_amd.cache_clear()
    yield
    tcsc_amd.set_order("fast")
    tcsc_amd.cache_clear()


def assert_bits(Y, ref, what):
    Y = np.asarray(Y, np.float32)
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(Y), nan), what
    np.testing.assert_array_equal(Y[~nan].view(np.uint32), ref[~nan].view(np.uint32), err_msg=what)


@pytest.mark.config_parity
@pytest.mark.parametrize("name", GOLDEN_NAMES)
def test_host_api_bit_exact_all_variants(reference_order, name):
    g = load_golden(name)
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    for variant in pyoracle.VARIANTS:
        Y = tcsc_amd.sgemm(variant, g["X"], W, g["B"], float(g["a"]))
        assert_bits(Y, g["Y_" + variant], f"{name}/{variant}")
    W.free()


@pytest.mark.parametrize("shards", [2, 3])
def test_column_blocks_bit_exact(reference_order, shards):
    g = load_golden("grid_m16_k512_n1024_nz8")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    tcsc_amd.set_num_shards(shards)
    try:
        for variant in ("basic", "prelu_separate"):
            assert_bits(tcsc_amd.sgemm(variant, g["X"], W, g["B"], 0.2), g["Y_" + variant], variant)
    finally:
        tcsc_amd.set_num_shards(0)
    W.free()


def test_plan_reports_its_order_and_switching_back(reference_order):
    g = load_golden("cfg1")
    W = tcsc_amd.TcscMatrix.from_dense(g["Wd"].astype(np.float32))
    assert tcsc_amd.Plan(W).info()["order"] == 1
    Yr = tcsc_amd.sgemm("optimized", g["X"], W, g["B"])
    assert_bits(Yr, g["Y_optimized"], "reference")
    tcsc_amd.set_order("fast")  # the cached plan is rebuilt in the fast order
    assert tcsc_amd.Plan(W).info()["order"] == 0
    Yf = tcsc_amd.sgemm("optimized", g["X"], W, g["B"])
    Y64, S64 = pyoracle.load_oracle().f64_rows(g["X"], tcsc_of(g), g["B"])
    assert pyoracle.check_close(Yf, Y64, S64)[0]
    W.free()


@pytest.mark.config_parity
@pytest.mark.parametrize("cfg_idx", [2, 3, 4])
def test_baseline_sizes_sampled_rows_bit_exact(reference_order, oracle, cfg_idx):
    """Full BASELINE shapes through the device API (plan from device arrays,
    the GPU builder): sampled rows equal the C oracle's reference-order sums."""
    import torch

    cfg = workloads.CONFIGS[cfg_idx]
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    K, N = cfg.K, cfg.N
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
    torch.cuda.synchronize()
    pyoracle.assert_builder_matches(oracle, inp.pop("Wd").cpu().numpy(), csp.cpu().numpy(), csn.cpu().numpy(),
                                    rip[:npos].cpu().numpy(), rin[:nneg].cpu().numpy())
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(cfg.M)
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    rows = np.unique(np.concatenate([[0, cfg.M - 1], np.random.default_rng(cfg_idx).integers(0, cfg.M, 6)]))
    idx = torch.from_numpy(rows).to(dev)
    Xs = inp["X"][idx].cpu().numpy()
    B = inp["B"].cpu().numpy()
    for variant in ("basic", "prelu_onthego"):
        Y = torch.empty((cfg.M, N), device=dev)
        plan.sgemm(inp["X"], inp["B"], Y, cfg.M, N, variant, 0.2)
        torch.cuda.synchronize()
        assert_bits(Y[idx].cpu().numpy(), oracle.sgemm(variant, Xs, W, B, 0.2), f"cfg{cfg_idx}/{variant}")
    plan.destroy()
