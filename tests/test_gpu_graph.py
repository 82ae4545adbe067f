"""tcsc_gpu_sgemm captured in a HIP graph (include/tcsc_gpu.h: once the
workspace covers M, a launch allocates nothing and never synchronises, so it
may be captured).  Replays must give the eager launch's bits on every path:
the gather (k_transpose + k_stream), split-K (+ k_reduce), the small-M path
and the MFMA path (one eager launch first: the BLAS library may allocate on
its first call)."""
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
