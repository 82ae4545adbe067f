#!/usr/bin/env python3
"""Diagnostic for k_fused's X^T staging (GPU): W = one +1 per column at row
n (so Y[m, n] - b[n] is exactly the X^T element (n, m) the gather read), X
holds unique codes; prints where the fused launch read something other than
X[m, n], grouped by row tile, chunk and unit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402
import torch  # noqa: E402


def run(M, K, fused, slices=None):
    os.environ["TCSC_FUSED"] = "1" if fused else "0"
    if slices:
        os.environ["TCSC_SLICES"] = str(slices)
    else:
        os.environ.pop("TCSC_SLICES", None)
    N = K
    dev = torch.device("cuda:0")
    csp = torch.arange(N + 1, dtype=torch.int32, device=dev)
    csn = torch.zeros(N + 1, dtype=torch.int32, device=dev)
    rip = torch.arange(N, dtype=torch.int32, device=dev)
    rin = torch.zeros(1, dtype=torch.int32, device=dev)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(M)
    X = (torch.arange(M, device=dev, dtype=torch.float32)[:, None] * 4096
         + torch.arange(K, device=dev, dtype=torch.float32)[None, :] % 4096)
    B = torch.zeros(N, device=dev)
    Y = torch.full((M, N), -1.0, device=dev)
    plan.sgemm(X, B, Y, M, N, "basic", 0.0)
    torch.cuda.synchronize()
    info = plan.launch_info(M)
    plan.destroy()
    return X.cpu().numpy(), Y.cpu().numpy(), info


def main():
    for (M, K, s) in [(512, 1536, None), (1024, 4096, None), (256, 960, 2)]:
        X, Y, info = run(M, K, True, s)
        bad = np.argwhere(Y != X[:, :K])
        print(f"M={M} K={K} slices={s} path={info}: {len(bad)} wrong of {Y.size}")
        if len(bad):
            m, k = bad[:, 0], bad[:, 1]
            print("  row tiles:", np.unique(m // 256)[:20], " chunks:", np.unique(k // 48)[:40])
            print("  k mod 4:", np.bincount(k % 4), " m mod 4:", np.bincount(m % 4))
            for mm, kk in bad[:12]:
                got = Y[mm, kk]
                print(f"   (m={mm}, k={kk}) expected {X[mm, kk]:.0f} = ({mm},{kk}) got {got:.0f}"
                      f" = ({int(got) // 4096},{int(got) % 4096})")


if __name__ == "__main__" and len(sys.argv) == 1:
    main()


def compare(M, K, N, density, variant, slices=None, seed=3):
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    r = torch.rand((K, N), generator=g, device=dev)
    Wd = torch.where(r < density / 2, 1.0, torch.where(r < density, -1.0, 0.0)).float()
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(M)
    X = torch.randint(-8, 9, (M, K), generator=g, device=dev).float()
    B = torch.zeros(N, device=dev)
    out = {}
    for fused in (0, 1):
        os.environ["TCSC_FUSED"] = str(fused)
        if slices:
            os.environ["TCSC_SLICES"] = str(slices)
        Y = torch.full((M, N), -777.0, device=dev)
        plan.sgemm(X, B, Y, M, N, variant, 0.2)
        torch.cuda.synchronize()
        out[fused] = Y.cpu().numpy()
    os.environ.pop("TCSC_SLICES", None)
    ref = (X @ Wd).cpu().numpy()
    info = plan.launch_info(M)
    plan.destroy()
    for f in (0, 1):
        bad = np.argwhere(out[f] != ref)
        print(f"M={M} K={K} N={N} d={density} {variant} slices={slices} fused={f} {info}: {len(bad)} wrong")
        if len(bad):
            m, n = bad[:, 0], bad[:, 1]
            print("  row tiles:", np.unique(m // 256)[:16], " col blocks:", np.unique(n // 256)[:16],
                  " waves:", np.unique((n % 256) // 16)[:16], " cols in wave:", np.bincount(n % 16, minlength=16))
            print("  rows mod 256 (first):", np.unique(m % 256)[:20])
            for mm, nn in bad[:6]:
                print(f"   (m={mm}, n={nn}) expected {ref[mm, nn]:.0f} got {out[f][mm, nn]:.0f}")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "cmp":
    compare(1024, 4096, 4096, 0.05, "basic")
    compare(512, 960, 512, 0.05, "basic")
    compare(256, 96, 256, 0.3, "basic")
    compare(512, 1536, 512, 0.02, "basic")


def probe(M, K, extra, density, slices=None, seed=5, reps=3):
    """W = [I_K | R] (R: K x extra, random ternary): Y[:, :K] - b is the X^T
    the gather read, under the load of the random columns."""
    dev = torch.device("cuda:0")
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    N = K + extra
    r = torch.rand((K, extra), generator=g, device=dev)
    R = torch.where(r < density / 2, 1.0, torch.where(r < density, -1.0, 0.0)).float()
    Wd = torch.cat([torch.eye(K, device=dev), R], dim=1).contiguous()
    csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
    plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
    plan.reserve(M)
    os.environ["TCSC_FUSED"] = "1"
    if slices:
        os.environ["TCSC_SLICES"] = str(slices)
    X = (torch.arange(M, device=dev, dtype=torch.float32)[:, None] * 4096
         + torch.arange(K, device=dev, dtype=torch.float32)[None, :] % 4096)
    B = torch.zeros(N, device=dev)
    info = plan.launch_info(M)
    for rep in range(reps):
        Y = torch.full((M, N), -1.0, device=dev)
        plan.sgemm(X, B, Y, M, N, "basic", 0.0)
        torch.cuda.synchronize()
        Yh = Y[:, :K].cpu().numpy()
        Xh = X.cpu().numpy()
        bad = np.argwhere(Yh != Xh)
        print(f"probe M={M} K={K} extra={extra} d={density} {info} rep {rep}: {len(bad)} wrong X^T reads")
        if len(bad):
            m, k = bad[:, 0], bad[:, 1]
            print("  row tiles:", np.unique(m // 256), " chunks:", np.unique(k // 48)[:30], " units(k//4):",
                  np.unique(k // 4)[:20])
            print("  lanes (m%256//4):", np.unique((m % 256) // 4)[:40])
            for mm, kk in bad[:8]:
                got = int(Yh[mm, kk])
                print(f"   X^T(k={kk}, m={mm}) read as X[{got // 4096}][{got % 4096}]")
    os.environ.pop("TCSC_SLICES", None)
    plan.destroy()


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "probe":
    probe(1024, 4096, 4096, 0.05)
    probe(2048, 4096, 4096, 0.05)
