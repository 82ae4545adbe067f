"""The in-launch split-K combines (k_stream OUT 2, `combine_tile`, by row
bands; OUT 3, pairwise at 2 slices -- split halves on resident grids, the
classic form on larger ones; DESIGN.md §4 k_reduce; TCSC_COMBINE=1)
against the k_stream + k_reduce4 pair
(TCSC_COMBINE=0): the same adds in the same order per element, so the outputs
must be bit-identical -- on cfg 2/3, on ragged shapes (M not a multiple of
256, the last column block partial), for forced slice counts 2, 3 (uneven row
bands) and 16, for every variant's bias order, across repeated launches on
one plan (the tile words are reset by each launch's last workgroup) and for
graph replays with new X.  Grids larger than the chip (the combine does not
apply) must give the same bits too."""
import numpy as np
import pytest

import pyoracle
import tcsc_amd

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    tcsc_amd.build()
    tcsc_amd.require_gpu()
    return tcsc_amd.lib()


@pytest.fixture(autouse=True)
def gather_plans(monkeypatch):
    """These are the gather's combines: plans of the denser shapes (0.1)
    would otherwise hold the MFMA image and the cost model may take it."""
    monkeypatch.setenv("TCSC_PATH", "gather")


def _plan(torch, K, N, density, seed):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    r = torch.rand((K, N), generator=g, device=dev)
    Wd = torch.where(r < density / 2, 1.0, torch.where(r < density, -1.0, 0.0)).float()
    del r
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    W = pyoracle.TCSC(K, N, csp.cpu().numpy(), csn.cpu().numpy(), rip[:npos].cpu().numpy(),
                      rin[:nneg].cpu().numpy())
    return plan, W


def _run(torch, plan, X, B, M, N, variant, combine, monkeypatch):
    monkeypatch.setenv("TCSC_COMBINE", "1" if combine else "0")
    Y = torch.full((M, N), float("nan"), device=X.device)
    plan.sgemm(X, B, Y, M, N, variant, 0.2)
    torch.cuda.synchronize()
    return Y


SHAPES = [  # M, K, N, density, variant, forced slices
    (1024, 4096, 4096, 0.05, "basic", None),            # cfg 2 (4 slices by the cost model, 256 workgroups)
    (1024, 4096, 4096, 0.05, "prelu_basic", None),      # cfg 3
    (1024, 4096, 4096, 0.05, "prelu_separate", "2"),    # bias last, two row bands
    (300, 1000, 200, 0.05, "prelu_onthego", None),      # ragged M, one partial column block
    (513, 2400, 700, 0.1, "basic", "3"),                # forced 3 slices: bands of 85/85/86 rows
    (517, 2400, 700, 0.1, "prelu_basic", "4"),          # 4 slices (own band kept in the LDS), ragged M and N
    (1024, 16384, 1024, 0.02, "prelu_basic", "16"),     # 16 slices x 16 tiles = 256 workgroups
    (4096, 16384, 2048, 0.02, "prelu_basic", None),     # the 8-way column block of cfg 4
    (2048, 4096, 8192, 0.05, "basic", "2"),             # 1024 workgroups: no combine, same bits
]


@pytest.mark.parametrize("M,K,N,density,variant,slices", SHAPES)
def test_combine_bit_identical_to_reduce_launch(gpu, oracle, monkeypatch, M, K, N, density, variant, slices):
    import torch

    if slices:
        monkeypatch.setenv("TCSC_SLICES", slices)
    plan, W = _plan(torch, K, N, density, 5 + M)
    plan.reserve(M)
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(13 + K)
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    for it in range(3):  # new X on the same plan: the tile words must be back at zero each time
        X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
        Yc = _run(torch, plan, X, B, M, N, variant, True, monkeypatch)
        Yr = _run(torch, plan, X, B, M, N, variant, False, monkeypatch)
        assert not torch.isnan(Yc).any(), f"iteration {it}: rows left unwritten"
        assert torch.equal(Yc.view(torch.int32), Yr.view(torch.int32)), f"iteration {it}"
    rows = np.unique(np.concatenate([[0, M - 1], np.random.default_rng(M).integers(0, M, 6)]))
    Y64, S64 = oracle.f64_rows(X[torch.from_numpy(rows).to(dev)].cpu().numpy(), W, B.cpu().numpy())
    a = 0.2 if variant in pyoracle.PRELU_VARIANTS else None
    ok, ratio = pyoracle.check_close(Yc[torch.from_numpy(rows).to(dev)].cpu().numpy(), Y64, S64, a)
    assert ok, ratio
    plan.destroy()


def test_combine_integer_exact(gpu, oracle, monkeypatch):
    """Integer X and bias: every partial sum is exact, so the combined output
    equals the oracle bit for bit on sampled rows."""
    import torch

    monkeypatch.setenv("TCSC_COMBINE", "1")
    M, K, N = 1024, 4096, 4096
    plan, W = _plan(torch, K, N, 0.05, 21)
    plan.reserve(M)
    dev = torch.device("cuda:0")
    X = torch.randint(-512, 513, (M, K), device=dev, dtype=torch.int32).float()
    B = torch.randint(-64, 65, (N,), device=dev, dtype=torch.int32).float()
    Y = torch.empty((M, N), device=dev)
    plan.sgemm(X, B, Y, M, N, "basic", 0.2)
    torch.cuda.synchronize()
    rows = np.unique(np.concatenate([[0, M - 1], np.random.default_rng(3).integers(0, M, 10)]))
    ref = oracle.sgemm("basic", X[torch.from_numpy(rows).to(dev)].cpu().numpy(), W, B.cpu().numpy())
    np.testing.assert_array_equal(Y[torch.from_numpy(rows).to(dev)].cpu().numpy(), ref)
    plan.destroy()


@pytest.mark.parametrize("M,K,N,slices,split,expect", [
    (1024, 4096, 4096, None, None, "bands"),     # cfg 2: row bands, own band in the LDS
    (1024, 8192, 2048, "2", None, "pairwise-split"),  # 64 workgroups, resident: split halves
    (1024, 8192, 2048, "2", "0", "pairwise"),         # the same in the classic form
])
def test_combine_graph_replay_with_new_x(gpu, monkeypatch, M, K, N, slices, split, expect):
    """A captured split-K launch with the in-launch combine, replayed with new
    X in place: each replay must find the tile words at zero."""
    import torch

    monkeypatch.setenv("TCSC_COMBINE", "1")
    if slices:
        monkeypatch.setenv("TCSC_SLICES", slices)
    if split:
        monkeypatch.setenv("TCSC_PAIR_SPLIT", split)
    plan, _ = _plan(torch, K, N, 0.05, 9)
    plan.reserve(M)
    assert plan.combine_mode(M) == expect
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
        monkeypatch.setenv("TCSC_COMBINE", "0")
        plan.sgemm(X, B, Yr, M, N, "prelu_basic", 0.2)
        monkeypatch.setenv("TCSC_COMBINE", "1")
        torch.cuda.synchronize()
        assert torch.equal(Y.view(torch.int32), Yr.view(torch.int32)), f"replay {it}"
    del gr
    plan.destroy()


@pytest.mark.parametrize("M,K,N,density,env,expect", [
    (1024, 4096, 4096, 0.05, None, "bands"),      # cfg 2: 4 slices, 256 workgroups
    (1024, 4096, 4096, 0.05, "0", None),          # switched off
    (128, 256, 256, 0.1, None, None),             # cfg 1: 6 workgroups, k_reduce4 is cheaper
    (128, 256, 256, 0.1, "1", "bands"),           # forced
    (4096, 16384, 2048, 0.02, None, "pairwise-split"),  # the 8-way column block: 256 workgroups, resident
    (2048, 4096, 8192, 0.05, None, "pairwise"),   # 2 slices x 256 tiles: the grid exceeds the chip, pairs need no residency
    (2048, 4096, 8192, 0.05, "0", None),
])
def test_launch_combine_reports_the_path(gpu, monkeypatch, M, K, N, density, env, expect):
    import torch

    if env is None:
        monkeypatch.delenv("TCSC_COMBINE", raising=False)
    else:
        monkeypatch.setenv("TCSC_COMBINE", env)
    if M == 2048:
        monkeypatch.setenv("TCSC_SLICES", "2")
    else:
        monkeypatch.delenv("TCSC_SLICES", raising=False)
    plan, _ = _plan(torch, K, N, density, 1)
    plan.reserve(M)
    path, slices = plan.launch_info(M)
    assert path == "gather" and slices > 1
    assert plan.combine_mode(M) == expect
    assert plan.launch_combine(M) == (expect is not None)
    plan.destroy()


@pytest.mark.parametrize("M,K,N,density,variant,slices", [
    (1024, 4096, 4096, 0.05, "prelu_basic", None),      # cfg 3: 4 slices
    (513, 2400, 700, 0.1, "basic", "3"),                # uneven bands
    (517, 2400, 700, 0.1, "prelu_basic", "4"),          # own bands written out on giving up, ragged M
    (1024, 16384, 1024, 0.02, "prelu_separate", "16"),  # 16 slices: one workgroup reduces all 16 bands
    (4096, 16384, 2048, 0.02, "prelu_basic", "2"),      # the 8-way column block
])
def test_combine_give_up_path_bit_identical(gpu, monkeypatch, M, K, N, density, variant, slices):
    """the path a slice takes when its partners are not resident
    (its bounded wait runs out) never ran in a test.  TCSC_COMBINE_GIVEUP=1
    makes every slice but each tile's last arrival give up at once, so the
    last arrival claims and reduces every band: the output must still equal
    the k_reduce4 launch bit for bit, launch after launch on one plan."""
    import torch

    if slices:
        monkeypatch.setenv("TCSC_SLICES", slices)
    plan, _ = _plan(torch, K, N, density, 31 + M)
    plan.reserve(M)
    monkeypatch.setenv("TCSC_COMBINE", "1")
    assert plan.combine_mode(M) == ("pairwise-split" if slices == "2" else "bands")
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(77 + K)
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    for it in range(3):
        X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
        monkeypatch.setenv("TCSC_COMBINE_GIVEUP", "1")
        Yg = _run(torch, plan, X, B, M, N, variant, True, monkeypatch)
        monkeypatch.delenv("TCSC_COMBINE_GIVEUP")
        Yc = _run(torch, plan, X, B, M, N, variant, True, monkeypatch)  # the words are back at zero
        Yr = _run(torch, plan, X, B, M, N, variant, False, monkeypatch)
        assert not torch.isnan(Yg).any(), f"iteration {it}: bands left unreduced"
        assert torch.equal(Yg.view(torch.int32), Yr.view(torch.int32)), f"iteration {it}: give-up path"
        assert torch.equal(Yc.view(torch.int32), Yr.view(torch.int32)), f"iteration {it}: after the give-up path"
    plan.destroy()
