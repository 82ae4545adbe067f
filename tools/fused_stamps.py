#!/usr/bin/env python3
"""Timing diagnostic for k_fused (GPU, the TCSC_FUSED_STAMPS=1 build:
`make -C sparse-matrix-multiplication-benchmark_amd -f ../tools/ab.mk lib/abl/libtcsc_amd_fst.so`,
loaded through TCSC_AMD_LIB).  Runs cfg 4 (M=4096, K=N=16384, 2 % ternary)
a few times and prints, per workgroup and launch, the s_memtime cycles of
each item phase, of the producer steps that acted, of the poll wave's checks
and of wave 0's chunk-barrier waits."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402
import torch  # noqa: E402

SLOTS = ["prologue", "chunk loop", "epilogue", "producer steps", "blocking polls", "blocking poll count", "wave0 barrier waits",
         "producer step count", "step: record read", "step: vmcnt wait", "step: slot read+stores", "step: DMA issue",
         "step: signal"]


def main(M=4096, K=16384, N=16384, density=0.02, reps=5):
    os.environ["TCSC_FUSED"] = "1"
    lib = C.CDLL(tcsc_amd.LIB_PATH)
    lib.tcsc_diag_fused_stamps.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    r = torch.rand((K, N), generator=g, device=dev)
    Wd = torch.where(r < density / 2, 1.0, torch.where(r < density, -1.0, 0.0)).float()
    del r
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
    del Wd
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(M)
    X = torch.randn((M, K), generator=g, device=dev)
    B = torch.zeros(N, device=dev)
    Y = torch.empty((M, N), device=dev)
    buf = (C.c_ulonglong * (4096 * 16))()
    for _ in range(2):
        plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2)
    torch.cuda.synchronize()
    lib.tcsc_diag_fused_stamps(buf, 4096 * 16)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        plan.sgemm(X, B, Y, M, N, "prelu_basic", 0.2)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / reps
    lib.tcsc_diag_fused_stamps(buf, 4096 * 16)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 16)
    used = a[:, 1] > 0
    a = a[used].astype(np.float64) / reps
    print(f"{ms:.3f} ms per launch, {used.sum()} workgroups, {plan.launch_info(M)}")
    tot = a[:, 0] + a[:, 1] + a[:, 2]
    print(f"  per-WG item total: mean {tot.mean():.0f} cycles, min {tot.min():.0f}, max {tot.max():.0f}")
    for i, name in enumerate(SLOTS):
        if name == "-":
            continue
        col = a[:, i]
        frac = col.mean() / tot.mean()
        print(f"  {name:22s} mean {col.mean():12.0f}  max {col.max():12.0f}  ({100 * frac:5.1f} % of item time)"
              if i not in (5, 7) else f"  {name:22s} mean {col.mean():12.1f}")
    plan.destroy()


if __name__ == "__main__":
    main()
