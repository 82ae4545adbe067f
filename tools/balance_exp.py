#!/usr/bin/env python3
"""How much does per-chunk load imbalance cost the lock-step gather kernel?

Times cfg4 (M=4096, K=N=16384, 2 % density) with three W patterns of the
same density:
  random    iid ternary (the benchmark's W)
  balanced  W[k, n] != 0 iff (k + 13 n) % 50 == 0: every column has one
            nonzero per 50 rows, so every wave's per-chunk stream has nearly
            the same length
  lumpy     the same count per column, but a wave's 16 columns all share one
            phase: per-chunk counts swing between 0 and 16
Usage (GPU box): python tools/balance_exp.py
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))

import torch  # noqa: E402

import tcsc_amd  # noqa: E402


def run(name, Wd, X, B, M, K, N, dev, steps=10):
    sh = torch.cuda.current_stream(dev).cuda_stream
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, stream=sh)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin, stream=sh)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin, 0, N, dev.index or 0, sh)
    plan.reserve(M)
    Y = torch.empty((M, N), device=dev, dtype=torch.float32)
    for _ in range(3):
        plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2, sh)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2, sh)
    e1.record()
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / steps
    nnz = npos + nneg
    print(f"{name:9s} nnz={nnz:9d}  {ms:.3f} ms  {(M * nnz + M * N) / ms / 1e6:.0f} G-add-ops/s", flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tcsc_amd.require_gpu()
    M, K, N = 4096, 16384, 16384
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    k = torch.arange(K, device=dev).view(K, 1)
    n = torch.arange(N, device=dev).view(1, N)
    sign = torch.where((n % 2) == 0, 1.0, -1.0).to(torch.float32)
    # balanced: phases spread across each wave's columns
    Wd = torch.where((k + 13 * n) % 50 == 0, sign, torch.zeros((), device=dev))
    run("balanced", Wd, X, B, M, K, N, dev)
    # lumpy: all 16 columns of a wave share one phase
    Wd = torch.where((k + 13 * (n // 16)) % 50 == 0, sign, torch.zeros((), device=dev))
    run("lumpy", Wd, X, B, M, K, N, dev)
    del Wd
    u = torch.rand((K, N), generator=g, device=dev)
    Wd = torch.zeros((K, N), device=dev)
    Wd[u < 0.01] = 1.0
    Wd[(u >= 0.01) & (u < 0.02)] = -1.0
    del u
    run("random", Wd, X, B, M, K, N, dev)


if __name__ == "__main__":
    main()
