#!/usr/bin/env python3
"""Run the TCSC_STAMPS diagnostic build on cfg4 and summarise where each
wave's chunk-loop cycles go (shader clock): DMA wait + barrier, waiting for
the scalar stream load, the gather itself, the rest."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TCSC_AMD_LIB"] = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd", "lib", "abl",
                                          "libtcsc_amd_stamps.so")
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tcsc_amd  # noqa: E402
from tcsc_amd import workloads  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = workloads.CONFIGS[int(sys.argv[1]) if len(sys.argv) > 1 else 4]
    inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
    sh = torch.cuda.current_stream(dev).cuda_stream
    K, N, M = cfg.K, cfg.N, cfg.M
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, stream=sh)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], K, N, csp, csn, rip, rin, stream=sh)
    del inp["Wd"]
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin, 0, N, 0, sh)
    plan.reserve(M)
    Y = torch.zeros((M, N), device=dev)
    for _ in range(3):
        plan.sgemm(inp["X"], inp["B"], Y, M, N, cfg.variant, 0.2, sh)
    torch.cuda.synchronize()
    ngroups = (N + 15) // 16
    nwg = ((ngroups + 15) // 16) * ((M + 255) // 256)
    st = Y.view(torch.int32).flatten()[: nwg * 16 * 5].cpu().numpy().astype(np.uint32).reshape(nwg * 16, 5)
    st = st.astype(np.float64)
    tot, bar, smem, gat, dma = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4]
    other = tot - bar - smem - gat - dma
    print(f"waves={len(tot)} mean cycles per wave: total {tot.mean():.0f}")
    for n, v in (("dma vmcnt wait", dma), ("barrier wait", bar), ("stream s_load wait", smem), ("gather asm", gat),
                 ("rest", other)):
        print(f"  {n:20s} {v.mean():12.0f}  {100 * v.mean() / tot.mean():5.1f} %")


if __name__ == "__main__":
    main()
