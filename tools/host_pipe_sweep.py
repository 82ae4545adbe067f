#!/usr/bin/env python3
"""Host API (drop-in, PCIe included) at cfg 4 over band counts, for the
copy-worker count in $TCSC_HOST_THREADS (read once per process): median of
--calls calls per band count.  Development tool for DESIGN.md §8."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 6
M, K, N, dens = 4096, 16384, 16384, 0.02
if len(sys.argv) > 2:  # M,K,N,density
    a = sys.argv[2].split(",")
    M, K, N, dens = int(a[0]), int(a[1]), int(a[2]), float(a[3])
rng = np.random.default_rng(4)
r = rng.random((K, N), dtype=np.float32)
Wd = np.where(r < dens / 2, np.float32(1), np.where(r < dens, np.float32(-1), np.float32(0)))
del r
W = tcsc_amd.TcscMatrix.from_dense(Wd)
del Wd
X = rng.uniform(-1, 1, (M, K)).astype(np.float32)
B = rng.uniform(-1, 1, N).astype(np.float32)
Y = np.empty((M, N), np.float32)
tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
out = {"threads": os.environ.get("TCSC_HOST_THREADS", "8"), "shape": [M, K, N, dens]}
for bands in (1, 2, 4, 8, 16):
    os.environ["TCSC_HOST_BANDS"] = str(bands)
    tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        tcsc_amd.sgemm("prelu_basic", X, W, B, 0.2, Y)
        ts.append(time.perf_counter() - t0)
    out[f"bands{bands}_ms"] = round(1e3 * float(np.median(ts)), 3)
    out[f"bands{bands}_min_ms"] = round(1e3 * float(np.min(ts)), 3)
print(json.dumps(out), flush=True)
