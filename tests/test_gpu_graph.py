"""tcsc_gpu_sgemm captured in a HIP graph (include/tcsc_gpu.h: once the
workspace covers M, a launch allocates nothing and never synchronises, so it
may be captured).  Replays must give the eager launch's bits on every path:
the gather (k_transpose + k_stream), split-K (+ k_reduce), the small-M path
and the MFMA path (k_split3 + k_gemm3 + k_fixup)."""
import numpy as np
import pytest

import tcsc_amd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_gpu():
    import torch

    tcsc_amd.build()
    tcsc_amd.require_gpu()
    return torch


@pytest.mark.parametrize("M,K,N,density,variant", [
    (300, 777, 333, 0.05, "prelu_basic"),    # gather
    (1024, 4096, 96, 0.05, "basic"),         # few column groups: split-K + k_reduce
    (2, 2048, 700, 0.05, "prelu_onthego"),   # small-M path
    (256, 1024, 512, 0.5, "optimized"),      # MFMA path (near-dense W)
])
def test_graph_replay_bit_identical(torch_gpu, oracle, M, K, N, density, variant):
    torch = torch_gpu
    dev = torch.device("cuda:0")
    Wd = oracle.ternary((K, N), density, 900 + M)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    X = torch.from_numpy(oracle.uniform((M, K), 901 + M)).to(dev)
    B = torch.from_numpy(oracle.uniform((N,), 902 + M)).to(dev)
    side = torch.cuda.Stream()
    plan = tcsc_amd.Plan(W, 0, N, 0, side.cuda_stream)
    plan.reserve(M)
    Ye = torch.empty((M, N), device=dev)
    with torch.cuda.stream(side):
        plan.sgemm(X, B, Ye, M, N, variant, 0.2, side.cuda_stream)  # eager (and the BLAS warm-up)
    side.synchronize()
    Yg = torch.full((M, N), float("nan"), device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        plan.sgemm(X, B, Yg, M, N, variant, 0.2, torch.cuda.current_stream().cuda_stream)
    for _ in range(3):
        Yg.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(Yg.cpu().numpy().view(np.uint32), Ye.cpu().numpy().view(np.uint32))
    del g
    plan.destroy()
    W.free()


def test_graph_replay_mfma_path_with_and_without_special_rows(torch_gpu, oracle, monkeypatch):
    """the MFMA path's row flags must not carry over between
    replays.  One captured launch, replayed on X holding inf / NaN / tiny
    values (flagged rows, recomputed exactly), then on X without them, then
    with them again: every replay equals the eager launch on the same X, bit
    for bit.  The path is forced (at this size the cost model picks the
    gather); its grid splits K, so the capture holds k_reduce4 too."""
    monkeypatch.setenv("TCSC_PATH", "mfma")
    torch = torch_gpu
    dev = torch.device("cuda:0")
    M, K, N = 256, 1024, 512
    Wd = oracle.ternary((K, N), 0.5, 950)
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    plain = oracle.uniform((M, K), 951)
    special = plain.copy()
    special[3, 5] = np.inf
    special[100, 7] = np.nan
    special[200, 9] = 1e-35
    B = torch.from_numpy(oracle.uniform((N,), 952)).to(dev)
    side = torch.cuda.Stream()
    plan = tcsc_amd.Plan(W, 0, N, 0, side.cuda_stream)
    plan.reserve(M)
    assert plan.info()["mfma_min_M"] and M >= plan.info()["mfma_min_M"]
    assert plan.launch_info(M) == ("mfma", 2)
    X = torch.empty((M, K), device=dev)
    eager = {}
    for name, x in (("plain", plain), ("special", special)):
        X.copy_(torch.from_numpy(x))
        Ye = torch.empty((M, N), device=dev)
        with torch.cuda.stream(side):
            plan.sgemm(X, B, Ye, M, N, "prelu_basic", 0.2, side.cuda_stream)
        side.synchronize()
        eager[name] = Ye.cpu().numpy().view(np.uint32).copy()
    assert not np.array_equal(eager["plain"], eager["special"])
    Yg = torch.empty((M, N), device=dev)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        plan.sgemm(X, B, Yg, M, N, "prelu_basic", 0.2, torch.cuda.current_stream().cuda_stream)
    for name in ("special", "plain", "special", "plain"):
        X.copy_(torch.from_numpy(special if name == "special" else plain))
        Yg.fill_(float("nan"))
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(Yg.cpu().numpy().view(np.uint32), eager[name], err_msg=name)
    del g
    plan.destroy()
    W.free()
