#!/usr/bin/env python3
"""PCIe-inclusive rate of the drop-in host API at cfg 4.

The reference's entry point `tcsc_sgemm_prelu_basic(X, W, B, a, Y, M, N, K)`
(sparse/tcsc.h:30) takes host pointers, so every call through it copies X
(268 MB) to the GPU and Y (268 MB) back.  This times that path as a user of
the reference would call it: the first call (which also uploads W and builds
the device plan) and the steady state.  It is reported beside the bench line,
never as `value`, which is the on-device rate with inputs already in HBM.

    python tools/host_api_rate.py [--calls 5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=4096)
    ap.add_argument("--K", type=int, default=16384)
    ap.add_argument("--N", type=int, default=16384)
    ap.add_argument("--sparsity", type=float, default=0.98)
    ap.add_argument("--calls", type=int, default=5)
    args = ap.parse_args()
    tcsc_amd.require_gpu()
    M, K, N = args.M, args.K, args.N
    rng = np.random.default_rng(4)
    r = rng.random((K, N), dtype=np.float32)
    half = (1.0 - args.sparsity) / 2
    Wd = np.where(r < half, np.float32(1), np.where(r < 2 * half, np.float32(-1), np.float32(0)))
    del r
    t0 = time.perf_counter()
    W = tcsc_amd.TcscMatrix.from_dense(Wd)
    t_build = time.perf_counter() - t0
    del Wd
    X = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, N).astype(np.float32)
    Y = np.empty((M, N), np.float32)
    nnz = W.nnz
    t0 = time.perf_counter()
    tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
    t_first = time.perf_counter() - t0
    ts = []
    for _ in range(args.calls):
        t0 = time.perf_counter()
        tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
        ts.append(time.perf_counter() - t0)
    ms = 1e3 * float(np.median(ts))
    rec = {
        "path": "host API tcsc_sgemm_prelu_basic (host X, Y; H2D + kernels + D2H per call)",
        "M": M, "K": K, "N": N, "sparsity": args.sparsity, "gpus": tcsc_amd.num_shards(),
        "tcsc_from_dense_s": t_build,
        "first_call_ms": 1e3 * t_first,
        "steady_ms_median": ms,
        "steady_ms_all": [1e3 * t for t in ts],
        "pcie_bytes_per_call": 4 * (M * K + M * N),
        "pcie_inclusive_gb_s": 4 * (M * K + M * N) / (ms * 1e-3) / 1e9,
    }
    rec["nnz"] = nnz
    rec["effective_g_add_ops_per_s"] = M * nnz / (ms * 1e-3) / 1e9
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
