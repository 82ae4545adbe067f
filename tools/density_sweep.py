#!/usr/bin/env python3
"""k_stream time at the cfg 4 shape (M=4096, K=N=16384) against W density:
separates the per-nonzero gather cost (slope) from the staging and per-chunk
overhead that does not depend on nnz (intercept).
Usage (GPU box): python tools/density_sweep.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))

import torch  # noqa: E402

import tcsc_amd  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tcsc_amd.require_gpu()
    M, K, N = 4096, 16384, 16384
    g = torch.Generator(device=dev)
    g.manual_seed(11)
    X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    Y = torch.empty((M, N), device=dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    XT = None
    rows = []
    for dens in (0.0, 0.0025, 0.005, 0.01, 0.02, 0.03, 0.04):
        u = torch.rand((K, N), generator=g, device=dev)
        Wd = torch.zeros((K, N), device=dev)
        Wd[u < dens / 2] = 1.0
        Wd[(u >= dens / 2) & (u < dens)] = -1.0
        del u
        csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
        csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
        npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, stream=sh)
        rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
        rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
        tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin, stream=sh)
        del Wd
        plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin, 0, N, 0, sh)
        plan.reserve(M)
        plan.prepare_x(X, M, sh)
        for _ in range(3):
            plan.sgemm_prepared(B, Y, M, N, "prelu_basic", 0.2, sh)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            plan.sgemm_prepared(B, Y, M, N, "prelu_basic", 0.2, sh)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        nnz = npos + nneg
        rows.append((dens, nnz, ms))
        print(f"density {dens:.4f} nnz {nnz:9d} k_stream {ms:.4f} ms", flush=True)
        del plan
    import numpy as np

    a = np.array([(r[1], r[2]) for r in rows if r[1] > 0])
    slope, icpt = np.polyfit(a[:, 0], a[:, 1], 1)
    print(f"fit: {icpt:.4f} ms + {slope * 1e6:.4f} ms per M nonzeros")


if __name__ == "__main__":
    main()
