#!/usr/bin/env python3
"""Would overlapping the Xᵀ staging with the gather pay?  (round 5 probe)

Times, on cfg 4's column block 0 of an S-way split (S = 1: the whole matrix):
  full     plan.sgemm over all M rows (k_transpose, then k_stream)
  halves   the rows in two halves, one after the other, on one stream
  overlap  the second half's k_transpose on a second stream, concurrent with
           the first half's gather (two plans: two Xᵀ workspaces)
HIP events on the launch stream, median over rounds of 20 steps.

    python tools/overlap_probe.py [--shard-of 8] [--rounds 5]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import tcsc_amd  # noqa: E402
from tcsc_amd import workloads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shard-of", type=int, default=1)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    tcsc_amd.require_gpu()
    cfg = workloads.CONFIGS[4]
    c0, c1 = 0, cfg.N // args.shard_of
    ncols = c1 - c0
    s1 = torch.cuda.current_stream(dev)
    s2 = torch.cuda.Stream(dev)
    sh1, sh2 = s1.cuda_stream, s2.cuda_stream
    inp = workloads.make_device_inputs(cfg, c0, c1, dev)
    csp = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, stream=sh1)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, rip, rin, stream=sh1)
    del inp["Wd"]
    M = cfg.M
    h = (M // 2 + 255) // 256 * 256
    pa = tcsc_amd.Plan.from_device(cfg.K, ncols, csp, csn, rip, rin, 0, ncols, 0, sh1)
    pb = tcsc_amd.Plan.from_device(cfg.K, ncols, csp, csn, rip, rin, 0, ncols, 0, sh1)
    pa.reserve(M)
    pb.reserve(M - h)
    X, B = inp["X"], inp["B"]
    Y = torch.empty((M, ncols), device=dev)
    Y2 = torch.empty((M, ncols), device=dev)
    v = cfg.variant

    def full():
        pa.sgemm(X, B, Y, M, ncols, v, 0.2, sh1)

    def halves():
        pa.sgemm(X[:h], B, Y2[:h], h, ncols, v, 0.2, sh1)
        pa.sgemm(X[h:], B, Y2[h:], M - h, ncols, v, 0.2, sh1)

    def overlap():
        e0 = torch.cuda.Event()
        e0.record(s1)
        s2.wait_event(e0)
        pa.prepare_x(X[:h], h, sh1)
        pb.prepare_x(X[h:], M - h, sh2)
        pa.sgemm_prepared(B, Y2[:h], h, ncols, v, 0.2, sh1)
        e1 = torch.cuda.Event()
        e1.record(s2)
        s1.wait_event(e1)
        pb.sgemm_prepared(B, Y2[h:], M - h, ncols, v, 0.2, sh1)

    def timed(fn):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record(s1)
        for _ in range(args.steps):
            fn()
        b.record(s1)
        torch.cuda.synchronize()
        return a.elapsed_time(b) / args.steps

    out = {k: [] for k in ("full", "halves", "overlap")}
    for _ in range(args.rounds):
        for k, fn in (("full", full), ("halves", halves), ("overlap", overlap)):
            out[k].append(timed(fn))
    full()
    overlap()
    torch.cuda.synchronize()
    diff = (Y - Y2).abs().max().item()
    scale = Y.abs().max().item()
    med = {k: sorted(x)[len(x) // 2] for k, x in out.items()}
    print(json.dumps({"shard_of": args.shard_of, "M": M, "ncols": ncols, "half": h,
                      "slices_full": pa.launch_info(M)[1], "slices_half": pa.launch_info(h)[1],
                      "ms_median": med, "ms_rounds": out, "max_abs_diff_full_vs_overlap": diff,
                      "max_abs_y": scale}))


if __name__ == "__main__":
    main()
