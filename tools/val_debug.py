import sys, os, time
sys.path.insert(0, "sparse-matrix-multiplication-benchmark_amd")
import torch, tcsc_amd
from tcsc_amd import workloads
dev = torch.device("cuda:0")
cfg = workloads.CONFIGS[2]
inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
K, N, M = cfg.K, cfg.N, cfg.M
csp = torch.empty(N + 1, dtype=torch.int32, device=dev); csn = torch.empty_like(csp)
p, q = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn)
rip = torch.empty(p, dtype=torch.int32, device=dev); rin = torch.empty(q, dtype=torch.int32, device=dev)
tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin)
plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
plan.reserve(M)
X, B, Wd = inp["X"], inp["B"], inp["Wd"]
Y = torch.empty((M, N), device=dev)
sh = torch.cuda.current_stream().cuda_stream
plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2, sh)
Yd = torch.empty_like(Y)
tcsc_amd.dense_sgemm(X, Wd, B, Yd, M, N, K, N, "prelu_basic", 0.2, sh)
S = torch.empty_like(Y)
tcsc_amd.dense_sgemm(X.abs(), Wd.abs(), B.abs(), S, M, N, K, N, "basic", 0.0, sh)
torch.cuda.synchronize()
print("Y", Y[0, :4].tolist(), "Yd", Yd[0, :4].tolist(), "S", S[0, :4].tolist())
err = (Y - Yd).abs()
print("max err", err.max().item(), "n nonzero err", int((err > 0).sum().item()), "S min/max", S.min().item(), S.max().item())
t = time.perf_counter()
for _ in range(3):
    tcsc_amd.dense_sgemm(X, Wd, B, Yd, M, N, K, N, "prelu_basic", 0.2, sh)
torch.cuda.synchronize(); print("dense ms", (time.perf_counter() - t) / 3 * 1e3)
sys.path.insert(0, ".")
import bench
step = lambda: plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2, sh)
print(bench.validate_against_dense(tcsc_amd, cfg, N, "prelu_basic", X, Wd, B, Y, step, sh))
