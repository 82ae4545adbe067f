"""The fused persistent gather (k_fused: X^T written by the gather's own
workgroups, DESIGN.md §4 "k_fused") against the two-kernel path
(k_transpose + k_stream, TCSC_FUSED=0): the same per-element summation order,
so the outputs must be bit-identical -- on the BASELINE shapes, on ragged
shapes (M not a multiple of 256, N not a multiple of 256, K not a multiple of
the 48-row chunk), with split-K, across repeated launches with new X on the
same plan (the piece counters carry a launch epoch and are never reset), and
for graph replays with new X."""
import numpy as np
import pytest

import pyoracle
import tcsc_amd
from tcsc_amd import workloads

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    return tcsc_amd.lib()


def _plan(torch, K, N, density, seed):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    r = torch.rand((K, N), generator=g, device=dev)
    Wd = torch.where(r < density / 2, 1.0, torch.where(r < density, -1.0, 0.0)).float()
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    return plan, W, (csp, csn, rip, rin)


def _run(torch, plan, X, B, M, N, variant, fused, monkeypatch):
    monkeypatch.setenv("TCSC_FUSED", "1" if fused else "0")
    Y = torch.full((M, N), float("nan"), device=X.device)
    plan.sgemm(X, B, Y, M, N, variant, 0.2)
    torch.cuda.synchronize()
    return Y


SHAPES = [  # M, K, N, density, variant, forced slices
    (1024, 4096, 4096, 0.05, "basic", None),          # cfg 2 (split-K by the cost model)
    (1024, 4096, 4096, 0.05, "prelu_basic", None),    # cfg 3
    (300, 1000, 200, 0.05, "prelu_onthego", None),    # ragged M, N; K not a multiple of 48
    (513, 2400, 700, 0.1, "basic", "3"),              # forced split-K, ragged everything
    (4096, 4096, 2048, 0.02, "prelu_basic", None),    # many row tiles, few column blocks
    (256, 96, 512, 0.3, "basic", None),               # two chunks
]


@pytest.mark.parametrize("M,K,N,density,variant,slices", SHAPES)
def test_fused_bit_identical_to_two_kernel_path(gpu, oracle, monkeypatch, M, K, N, density, variant, slices):
    import torch

    if slices:
        monkeypatch.setenv("TCSC_SLICES", slices)
    plan, W, _ = _plan(torch, K, N, density, 7 + M)
    plan.reserve(M)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(11 + K)
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    for it in range(3):  # new X on the same plan each time (epochs)
        X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
        Yf = _run(torch, plan, X, B, M, N, variant, True, monkeypatch)
        Y2 = _run(torch, plan, X, B, M, N, variant, False, monkeypatch)
        assert torch.equal(Yf.view(torch.int32), Y2.view(torch.int32)), f"iteration {it}"
    rows = np.unique(np.concatenate([[0, M - 1], np.random.default_rng(M).integers(0, M, 6)]))
    Y64, S64 = oracle.f64_rows(X[torch.from_numpy(rows).to(dev)].cpu().numpy(), W, B.cpu().numpy())
    a = 0.2 if variant in pyoracle.PRELU_VARIANTS else None
    ok, ratio = pyoracle.check_close(Yf[torch.from_numpy(rows).to(dev)].cpu().numpy(), Y64, S64, a)
    assert ok, ratio
    plan.destroy()


def test_fused_cfg4_full_size_and_integer_exact(gpu, oracle, monkeypatch):
    """BASELINE cfg 4 through the fused kernel: bit-identical to the two-kernel
    path, and integer X exact against the oracle on sampled rows."""
    import torch

    cfg = workloads.CONFIGS[4]
    dev = torch.device("cuda:0")
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    K, N, M = cfg.K, cfg.N, cfg.M
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
    del inp["Wd"]
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(M)
    Yf = _run(torch, plan, inp["X"], inp["B"], M, N, cfg.variant, True, monkeypatch)
    Y2 = _run(torch, plan, inp["X"], inp["B"], M, N, cfg.variant, False, monkeypatch)
    assert torch.equal(Yf.view(torch.int32), Y2.view(torch.int32))
    Xi = torch.randint(-512, 513, (M, K), device=dev, dtype=torch.int32).float()
    Bi = inp["B"].round()
    Yi = _run(torch, plan, Xi, Bi, M, N, "basic", True, monkeypatch)
    rows = np.unique(np.concatenate([[0, M - 1], np.random.default_rng(5).integers(0, M, 10)]))
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    ref = oracle.sgemm("basic", Xi[torch.from_numpy(rows).to(dev)].cpu().numpy(), W, Bi.cpu().numpy())
    np.testing.assert_array_equal(Yi[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
    plan.destroy()


def test_fused_graph_replay_with_new_x(gpu, monkeypatch):
    """A captured launch of the fused kernel, replayed with new X in place:
    the epoch comes from the plan's device-side block, so every replay waits
    for its own X^T rows (a frozen epoch would let a replay read the previous
    replay's rows)."""
    import torch

    monkeypatch.setenv("TCSC_FUSED", "1")
    M, K, N = 1024, 4096, 2048
    plan, W, _ = _plan(torch, K, N, 0.05, 3)
    plan.reserve(M)
    dev = torch.device("cuda:0")
    X = torch.empty((M, K), device=dev)
    B = torch.rand((N,), device=dev) * 2 - 1
    Y = torch.empty((M, N), device=dev)
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    X.uniform_(-1, 1)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr, stream=side):
        plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2, torch.cuda.current_stream().cuda_stream)
    for it in range(4):
        X.uniform_(-1, 1)
        gr.replay()
        torch.cuda.synchronize()
        Yr = torch.empty_like(Y)
        monkeypatch.setenv("TCSC_FUSED", "0")
        plan.sgemm(X, B, Yr, M, N, "prelu_basic", 0.2)
        monkeypatch.setenv("TCSC_FUSED", "1")
        torch.cuda.synchronize()
        assert torch.equal(Y.view(torch.int32), Yr.view(torch.int32)), f"replay {it}"
    del gr
    plan.destroy()
