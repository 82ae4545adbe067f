#!/usr/bin/env python3
"""Per-call split of a small drop-in host call (TCSC_HOST_TRACE=1): plan
lookup + content fingerprint against the whole call, for main.cpp's M = 1
shapes (main.cpp:258-261).  Development tool."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402

for M, K, N in ((1, 512, 2048), (1, 2048, 8192), (256, 1024, 4096)):
    rng = np.random.default_rng(1)
    r = rng.random((K, N), dtype=np.float32)
    W = tcsc_amd.TcscMatrix.from_dense(np.where(r < 0.25, 1.0, np.where(r < 0.5, -1.0, 0.0)).astype(np.float32))
    X = rng.uniform(-1, 1, (M, K)).astype(np.float32)
    B = rng.uniform(-1, 1, N).astype(np.float32)
    Y = np.empty((M, N), np.float32)
    for _ in range(5):
        tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
    t = time.perf_counter()
    for _ in range(50):
        tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
    print(f"M={M} K={K} N={N} nnz={W.nnz}: {1e6 * (time.perf_counter() - t) / 50:.1f} us per call", flush=True)
    W.free()
