#!/usr/bin/env python3
"""Does giving the older wave slots more work shorten the chunk interval?

cfg4 shape (M=4096, K=N=16384, mean density 2 %), W iid ternary but the
density of a column depends on the wave slot that owns it (column n ->
wave (n % 256) // 16 of its workgroup -> slot wave // 4, the SIMD
arbiter's age order: tools/trace.py).  Multipliers per slot keep the mean
at 2 %, so nnz (and add-ops) stay the same; only who does the work changes.
Usage (GPU box): python tools/slot_skew_exp.py
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import tcsc_amd  # noqa: E402
from balance_exp import run  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tcsc_amd.require_gpu()
    M, K, N = 4096, 16384, 16384
    g = torch.Generator(device=dev)
    g.manual_seed(7)
    X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
    B = torch.rand((N,), generator=g, device=dev) * 2 - 1
    slot = ((torch.arange(N, device=dev) % 256) // 16) // 4
    for mult in ([1, 1, 1, 1], [1.3, 1.1, 0.9, 0.7], [1.5, 1.2, 0.8, 0.5], [1.8, 1.2, 0.6, 0.4],
                 [0.7, 0.9, 1.1, 1.3]):
        d = 0.02 * torch.tensor(mult, device=dev, dtype=torch.float32)[slot].view(1, N)
        u = torch.rand((K, N), generator=g, device=dev)
        Wd = torch.zeros((K, N), device=dev)
        Wd[u < d / 2] = 1.0
        Wd[(u >= d / 2) & (u < d)] = -1.0
        del u
        run("x".join(str(m) for m in mult), Wd, X, B, M, K, N, dev)
        del Wd


if __name__ == "__main__":
    main()
