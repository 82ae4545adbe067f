#!/usr/bin/env python3
"""Device tcsc_from_dense at BASELINE cfg 4 (K = N = 16384, 98 % sparse):
both calls (counts, then fill), 5 times; run under rocprofv3 --kernel-trace
--stats to see k_dense_tile_counts / _scan / _fill."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import torch  # noqa: E402

import tcsc_amd  # noqa: E402
from tcsc_amd import workloads  # noqa: E402

cfg = workloads.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 4]
dev = torch.device("cuda:0")
inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
d = inp["Wd"]
csp = torch.empty(cfg.N + 1, dtype=torch.int32, device=dev)
csn = torch.empty(cfg.N + 1, dtype=torch.int32, device=dev)
for it in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    npos, nneg = tcsc_amd.gpu_from_dense(d, cfg.K, cfg.N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(d, cfg.K, cfg.N, csp, csn, rip, rin)
    torch.cuda.synchronize()
    print(f"build {it}: {(time.perf_counter() - t0) * 1e3:.3f} ms wall, nnz {npos + nneg}", flush=True)
