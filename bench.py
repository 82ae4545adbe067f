#!/usr/bin/env python3
"""TCSC sparse-ternary GEMM benchmark (BASELINE.json metric) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 4]
    torchrun --nproc-per-node N bench.py --gpus N ...

A "step" is one pass of the hot path over one batch: one launch of the gfx950
gather kernel computing Y = PReLU(X*W + b) for this rank's output columns,
inputs already resident in HBM.  N=1 runs BASELINE configs[3] (cfg4: M=4096,
K=N=16384, 98 % sparse, PReLU) -- the configuration the north star's target
is quoted on.  With N ranks (the north star's "output-column
shard across 8 x MI355X"):
  --scaling strong (default) the cfg4 matrix itself is split over the N ranks:
                   into column blocks (--shard cols, the default: X replicated,
                   rank g owns columns [g*N/G, (g+1)*N/G)) or row blocks
                   (--shard rows: each rank stages only its rows of X; W is
                   replicated).  At N>1 the line also carries `alt_shard`, the
                   other axis timed with the same protocol;
  --scaling weak   every rank owns a full 16384-column block of a
                   N*16384-column W (per-GPU work fixed as N grows).
There is no collective on the data path; the only collectives are the
timing barrier and the max-over-ranks of the elapsed time.

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` for the gather kernel (algorithmic bytes per launch / average
launch time measured with HIP events on the launch stream) and
`cpu_baseline` (the reference's own sparse/tcsc.c, compiled in place into
oracle/_ref, timed on this host's cores on a bounded sample of the same
workload; its OpenMP form on every usable core beside it).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd")
sys.path.insert(0, PKG)

METRIC = "TCSC SpMM: effective G-add-ops/s + achieved HBM GB/s vs roofline, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
# LDS gather roof: ds_read_b64/b128 move 256 B/clk/CU = 64 fp32 per clk per CU
LDS_GATHER_PEAK = 64 * 256 * 2.4e9  # gathered fp32 values / s
VALU_ADD_PEAK = 128 * 256 * 2.4e9  # fp32 adds / s (4 SIMD32 per CU)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--config", type=int, default=4)
    p.add_argument("--scaling", choices=("weak", "strong"), default="strong",
                   help="strong (default): cfg's matrix split over the N ranks (--shard); weak: every rank a full copy")
    p.add_argument("--variant", default=None, help="override the config's variant")
    p.add_argument("--shard", choices=("cols", "rows"), default="cols",
                   help="strong scaling / --shard-of: split N (X replicated) or M (X split, W replicated)")
    p.add_argument("--no-alt-shard", action="store_true",
                   help="N>1 strong: skip the extra timing of the other split axis (rows when --shard cols)")
    p.add_argument("--shard-of", type=int, default=0,
                   help="time only rank 0's block of an S-way strong split (per-GPU view of S GPUs)")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-dense-baseline", action="store_true", help="skip the rocBLAS dense comparison (N=1 only)")
    p.add_argument("--no-bcsr", action="store_true", help="skip the BCSR (1x8 blocks) line (N=1 only)")
    p.add_argument("--no-reference-order", action="store_true",
                   help="skip the reference-summation-order line (N=1 only)")
    p.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                   help="nccl (= RCCL, one GPU per rank); gloo lets ranks share a GPU (rehearsal only)")
    p.add_argument("--no-other-configs", action="store_true",
                   help="skip the other BASELINE configs' timings (N=1 only)")
    p.add_argument("--no-validate", action="store_true", help="skip the pre-timing check against the dense product")
    p.add_argument("--no-graph", action="store_true",
                   help="skip the HIP-graph line (the same steps captured once and replayed; N=1 only)")
    p.add_argument("--no-host-api", action="store_true",
                   help="skip the drop-in host-pointer call line (PCIe included; N=1 only)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"))
    p.add_argument("--override", default="", help="experiments only: e.g. 'K=16448,N=4096' (marks the line)")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import tcsc_amd
    from tcsc_amd import workloads
    from tcsc_amd.shard import column_range, rank_env

    rank, local_rank, world = rank_env()
    if world != args.gpus:
        if world == 1 and args.gpus > 1:
            raise SystemExit("--gpus N>1 needs one process per GPU: launch with torchrun --nproc-per-node N")
    distributed = world > 1
    # one GPU per rank; with --dist-backend gloo several ranks may share a GPU
    # (a rehearsal of the multi-rank path on a one-GPU box: RCCL refuses that)
    ndev = torch.cuda.device_count()  # does not initialise the GPU
    gpu = local_rank if args.dist_backend == "nccl" or ndev == 0 else local_rank % ndev
    if distributed:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(gpu)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    local_rank = gpu
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    tcsc_amd.require_gpu()

    cfg = workloads.CONFIGS[args.config]
    if args.override:
        import dataclasses

        kv = dict(x.split("=") for x in args.override.split(","))
        cfg = dataclasses.replace(cfg, **{k: (float(v) if k == "sparsity" else int(v)) for k, v in kv.items()})
    variant = args.variant or cfg.variant
    # this rank's block: all rows x a column block (--shard cols), or a row
    # block x all columns (--shard rows: X split instead of replicated)
    cfg_full = cfg
    r0, r1 = 0, cfg.M
    if args.scaling == "weak":
        c0, c1, seed_off = 0, cfg.N, rank
    else:
        c0, c1, seed_off = 0, cfg.N, 0
        if args.shard == "cols":
            c0, c1 = column_range(cfg.N, world, rank)
        else:
            r0, r1 = column_range(cfg.M, world, rank)
    if args.shard_of > 1:
        if args.shard == "cols":
            c0, c1 = column_range(cfg.N, args.shard_of, 0)
        else:
            r0, r1 = column_range(cfg.M, args.shard_of, 0)
    ncols = c1 - c0
    stream = torch.cuda.current_stream(dev)
    sh = stream.cuda_stream

    # ---- setup (not timed): synthetic inputs + device TCSC + plan --------
    inp = workloads.make_device_inputs(cfg, c0, c1, dev, seed_offset=seed_off)
    csp = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, stream=sh)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, rip, rin, stream=sh)
    Wd = inp.pop("Wd")  # validation, then the dense baseline and the BCSR line
    if (r0, r1) != (0, cfg.M):  # a row block: the same X on every rank, this rank's rows
        import dataclasses

        inp["X"] = inp["X"][r0:r1].contiguous()
        cfg = dataclasses.replace(cfg, M=r1 - r0)
    plan = tcsc_amd.Plan.from_device(cfg.K, ncols, csp, csn, rip, rin, 0, ncols, local_rank, sh)
    plan.reserve(cfg.M)
    nnz = npos + nneg
    X, B = inp["X"], inp["B"]
    Y = torch.empty((cfg.M, ncols), device=dev, dtype=torch.float32)
    torch.cuda.synchronize(dev)

    def step():
        plan.sgemm(X, B, Y, cfg.M, ncols, variant, 0.2, sh)

    # ---- validation (not timed): as the reference harness validates before it
    # measures (main.cpp:299-368), every rank checks one step's full output
    validation = None
    if not args.no_validate:
        validation = validate_against_dense(tcsc_amd, cfg, ncols, variant, X, Wd, B, Y, step, sh)
        validation["determinism"] = check_determinism(step, Y, 24)
    if world > 1 or (args.no_dense_baseline and args.no_bcsr):
        Wd = None
    torch.cuda.synchronize(dev)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    step_events_s = ev0.elapsed_time(ev1) / 1e3 / max(args.steps, 1)

    # Per-kernel split on the same stream (not part of `value`): the X^T
    # staging (k_transpose) and the gather (k_stream) back to back, each
    # averaged over `steps` launches with HIP events, so roofline.kernel_ms is
    # the average duration of the kernel the rocprofv3 summary lists.
    def timed(fn, n):
        a_ev = torch.cuda.Event(enable_timing=True)
        b_ev = torch.cuda.Event(enable_timing=True)
        a_ev.record(stream)
        for _ in range(n):
            fn()
        b_ev.record(stream)
        b_ev.synchronize()
        return a_ev.elapsed_time(b_ev) / 1e3 / n

    nsplit = max(args.steps, 5)
    # the step's kernels (k_transpose, then k_stream, + k_reduce4 when K is
    # split and not combined in the launch), timed with HIP events on the
    # launch stream: the whole step, then the X^T staging and the gather apart
    path, slices = plan.launch_info(cfg.M)
    step_kernels_s = timed(step, nsplit)
    transpose_s = timed(lambda: plan.prepare_x(X, cfg.M, sh), nsplit)
    plan.prepare_x(X, cfg.M, sh)
    gather_s = timed(lambda: plan.sgemm_prepared(B, Y, cfg.M, ncols, variant, 0.2, sh), nsplit)
    kernel_s = gather_s
    combine = plan.combine_mode(cfg.M) if slices > 1 else None
    # the two halves per path: prepare_x / sgemm_prepared run k_transpose / k_stream
    # on the gather path, k_split3 / k_gemm3 + k_fixup on the MFMA path
    if path == "mfma":
        kernel_name, stage_names = "k_gemm3 + k_fixup", ("k_split3", "k_gemm3 + k_fixup")
    else:
        kernel_name = "k_stream" + ((f" (+ in-launch {combine} combine)" if combine else " + k_reduce4") +
                                    f", {slices} K slices" if slices > 1 else "")
        stage_names = ("k_transpose", "gather")

    alt = None
    if distributed and args.scaling == "strong" and not args.no_alt_shard and args.shard_of <= 1:
        # the other collective-free split of the same config, timed with the same
        # protocol (SURVEY.md §8e "Alternative"): row blocks when the line is column
        # blocks.  Every rank takes part; rank 0 reports it beside the main line.
        alt = alt_shard_line(args, tcsc_amd, workloads, cfg_full, variant, rank, world, dev, sh, stream)

    ops_rank = workloads.add_ops(cfg.M, nnz, ncols) * args.steps
    stats = torch.tensor([elapsed, float(ops_rank)], dtype=torch.float64,
                         device=dev if args.dist_backend == "nccl" else "cpu")
    if distributed:
        t_max = stats[:1].clone()
        dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        ops_tot = stats[1:].clone()
        dist.all_reduce(ops_tot, op=dist.ReduceOp.SUM)
        elapsed_max, ops_total = float(t_max.item()), float(ops_tot.item())
    else:
        elapsed_max, ops_total = elapsed, float(ops_rank)

    if rank == 0:
        algo_bytes = workloads.algorithmic_bytes(cfg.M, cfg.K, ncols, nnz)
        achieved = algo_bytes / kernel_s / 1e9
        adds_per_launch = workloads.add_ops(cfg.M, nnz, ncols)
        traffic = None
        try:
            with open(args.traffic) as f:
                t = json.load(f)
            # a row block (--shard rows) is its own launch shape: keyed by its rows too
            key = f"cfg{cfg.idx}:{variant}:{ncols}"
            if cfg.M != workloads.CONFIGS[cfg.idx].M:
                key += f":M{cfg.M}"
            if key in t:
                traffic = t[key]["hbm_bytes_per_launch"]
        except (OSError, ValueError, KeyError):
            traffic = None
        out = {
            "metric": METRIC,
            "value": ops_total / elapsed_max / 1e9,
            "unit": "G-add-ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (X,B ~ U[-1,1), W iid ternary; seeded torch generators)",
            "config": {
                "workload": f"{cfg_full.name}: {cfg_full.describe()}"
                            + (f" [override {args.override}]" if args.override else ""),
                "M": cfg_full.M, "K": cfg.K, "N": cfg.N, "sparsity": cfg.sparsity, "variant": variant,
                "columns_per_gpu": ncols, "nnz_per_gpu": nnz,
                "parallelism": (f"per-GPU view: rank 0's block of a {args.shard_of}-way {args.shard} split"
                                if args.shard_of > 1 else
                                f"{'row' if args.shard == 'rows' and args.scaling == 'strong' else 'column'}"
                                f"-shard x{world} ({args.scaling}), no collective"),
                "rows_per_gpu": cfg.M,
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "kernel": kernel_name,
                "path": path,
                "k_slices": slices,
                "combine_in_launch": combine,
                "algorithmic_bytes_per_launch": algo_bytes,
                "kernel_ms": kernel_s * 1e3,
                "step_ms_events": step_events_s * 1e3,
                # the same algorithmic bytes over the whole step (k_transpose
                # included): the HBM fraction that matches `value`
                "step_achieved": algo_bytes / (elapsed_max / args.steps) / 1e9,
                "step_frac": algo_bytes / (elapsed_max / args.steps) / 1e9 / HBM_PEAK_GBS,
                "step_parts_ms": {stage_names[0]: transpose_s * 1e3, stage_names[1]: gather_s * 1e3,
                                  "step_kernels": step_kernels_s * 1e3,
                                  "note": "HIP events on the launch stream, each averaged over the same launches"},
                "lds_gather_frac": (cfg.M * nnz / kernel_s) / LDS_GATHER_PEAK,
                "valu_add_frac": (adds_per_launch / kernel_s) / VALU_ADD_PEAK,
            },
        }
        if validation is not None:
            out["validation"] = validation
        if alt is not None:
            out["alt_shard"] = alt
        if Wd is not None and not args.no_dense_baseline:
            # the reference's "TCSC vs Dense" line (main.cpp:379-391) on the
            # device -- gemm_basic's dense product with the same ternary W as an fp32 rocBLAS
            # SGEMM + the bias/PReLU epilogue, same X, B and Y, timed with HIP events
            Yd = torch.empty_like(Y)

            def dense_step():
                tcsc_amd.dense_sgemm(X, Wd, B, Yd, cfg.M, ncols, cfg.K, ncols, variant, 0.2, sh)

            dense_step()
            dense_s = timed(dense_step, 3)
            out["dense_baseline"] = {
                "kernel": "rocblas_sgemm fp32 (dense ternary W) + k_bias_act",
                "ms": dense_s * 1e3,
                "dense_tflops": 2.0 * cfg.M * cfg.K * ncols / dense_s / 1e12,
                "tcsc_speedup": dense_s / (elapsed_max / args.steps),
            }
            del Yd
        if Wd is not None and not args.no_bcsr:
            out["bcsr"] = bcsr_line(cfg, Wd, X, B, Y, nnz, kernel_s, timed, sh, nsplit)
        if world == 1 and not args.no_host_api:
            # end to end through the drop-in symbol, H2D of X/B and D2H of Y
            # included (pageable numpy buffers, as main.cpp passes them); Y still holds the
            # device API's output of the same X, so the two are compared bit for bit
            out["host_api"] = host_api_line(tcsc_amd, cfg, ncols, variant, X, B, Y, csp, csn, rip[:npos],
                                            rin[:nneg], adds_per_launch)
        if world == 1 and not args.no_reference_order:
            # include/tcsc_gpu.h TCSC_ORDER_REFERENCE: each variant in the reference's own
            # summation order (float outputs bit-identical to sparse/tcsc.c); K is walked once
            # per sign, so the gather is slower than the merged (fast) order the value uses
            tcsc_amd.set_order("reference")
            try:
                rplan = tcsc_amd.Plan.from_device(cfg.K, ncols, csp, csn, rip, rin, 0, ncols, local_rank, sh)
            finally:
                tcsc_amd.set_order("fast")
            rplan.reserve(cfg.M)
            rplan.prepare_x(X, cfg.M, sh)
            ref = {"kernel": "k_stream ORDER 1 / 2 (two sign chains)"}
            for v in ("prelu_basic", "prelu_separate"):
                rplan.sgemm_prepared(B, Y, cfg.M, ncols, v, 0.2, sh)
                t = timed(lambda: rplan.sgemm_prepared(B, Y, cfg.M, ncols, v, 0.2, sh), nsplit)
                ref[v] = {"ms": t * 1e3, "g_add_ops_per_s": adds_per_launch / t / 1e9, "vs_fast_order": t / kernel_s}
            rplan.destroy()
            out["reference_order"] = ref
        if world == 1 and not args.no_graph:
            # the same K steps captured in one HIP graph and replayed (not `value`): what the
            # launch gaps between k_transpose and k_stream cost on the eager stream
            out["graph"] = graph_line(plan, X, B, Y, cfg.M, ncols, variant, args.steps, stream, elapsed_max)
        if world == 1 and not args.no_other_configs and not args.override:
            out["other_configs"] = other_configs(args, tcsc_amd, workloads, dev, sh, timed, cfg.idx)
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args, cfg, variant, X, B, csp, csn, rip[:npos], rin[:nneg])
        print(json.dumps(out), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def alt_shard_line(args, tcsc_amd, workloads, cfg, variant, rank, world, dev, sh, stream):
    """The strong-scaling split along the other axis (rows if the line splits
    columns): warm-up, barrier + sync, `steps` steps, barrier + sync, max over
    ranks; whole-job add-ops / that time.  Each rank holds the plan of the
    whole W and its M/N rows of X (no collective on the data path)."""
    import dataclasses

    import torch
    import torch.distributed as dist
    from tcsc_amd.shard import column_range

    shard = "rows" if args.shard == "cols" else "cols"
    r0, r1, c0, c1 = 0, cfg.M, 0, cfg.N
    if shard == "rows":
        r0, r1 = column_range(cfg.M, world, rank)
    else:
        c0, c1 = column_range(cfg.N, world, rank)
    ncols = c1 - c0
    inp = workloads.make_device_inputs(cfg, c0, c1, dev)
    csp = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    csn = torch.empty(ncols + 1, dtype=torch.int32, device=dev)
    npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, stream=sh)
    rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
    rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
    tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, ncols, csp, csn, rip, rin, stream=sh)
    del inp["Wd"]
    c = dataclasses.replace(cfg, M=r1 - r0)
    X = inp["X"][r0:r1].contiguous()
    B = inp["B"]
    plan = tcsc_amd.Plan.from_device(c.K, ncols, csp, csn, rip, rin, 0, ncols, dev.index or 0, sh)
    plan.reserve(c.M)
    Y = torch.empty((c.M, ncols), device=dev)
    for _ in range(max(args.warmup, 5)):
        plan.sgemm(X, B, Y, c.M, ncols, variant, 0.2, sh)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        plan.sgemm(X, B, Y, c.M, ncols, variant, 0.2, sh)
    torch.cuda.synchronize(dev)
    dist.barrier()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    ops = workloads.add_ops(c.M, npos + nneg, ncols) * args.steps
    st = torch.tensor([el, float(ops)], dtype=torch.float64, device=dev if args.dist_backend == "nccl" else "cpu")
    t_max, o_tot = st[:1].clone(), st[1:].clone()
    dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
    dist.all_reduce(o_tot, op=dist.ReduceOp.SUM)
    plan.destroy()
    del X, Y, csp, csn, rip, rin, inp
    torch.cuda.empty_cache()
    return {"shard": shard, "value": float(o_tot.item()) / float(t_max.item()) / 1e9, "unit": "G-add-ops/s",
            "ms_per_step": float(t_max.item()) / args.steps * 1e3, "rows_per_gpu": c.M, "columns_per_gpu": ncols,
            "note": "same protocol as the line; X rows split (W replicated)" if shard == "rows" else
                    "same protocol as the line; W columns split (X replicated)"}


def host_api_line(tcsc_amd, cfg, ncols, variant, X, B, Y, csp, csn, rip, rin, adds, calls=6):
    """tcsc_sgemm_<variant> (sparse/tcsc.h:21-46) on host copies of the same
    inputs: the first call (plan build + W upload) and the median of `calls`
    steady-state calls, each synchronous with its PCIe copies (not `value`)."""
    import numpy as np

    Xh, Bh, Yd = X.cpu().numpy(), B.cpu().numpy(), Y.cpu().numpy()
    W = tcsc_amd.TcscMatrix.from_arrays(cfg.K, ncols, csp.cpu().numpy(), csn.cpu().numpy(), rip.cpu().numpy(),
                                        rin.cpu().numpy())
    Yh = np.zeros((cfg.M, ncols), np.float32)
    t0 = time.perf_counter()
    tcsc_amd.sgemm(variant, Xh, W, Bh, 0.2, Yh)
    first = time.perf_counter() - t0
    same = bool(np.array_equal(Yh.view(np.uint32), Yd.view(np.uint32)))
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        tcsc_amd.sgemm(variant, Xh, W, Bh, 0.2, Yh)
        ts.append(time.perf_counter() - t0)
    tcsc_amd.cache_clear()
    W.free()
    ms = float(np.median(ts)) * 1e3
    return {"symbol": f"tcsc_sgemm_{variant}", "ms": ms, "g_add_ops_per_s": adds / (ms * 1e-3) / 1e9,
            "min_ms": min(ts) * 1e3, "first_call_ms": first * 1e3, "calls": calls,
            "pcie_bytes": 4 * (cfg.M * cfg.K + cfg.M * ncols + ncols),
            "bit_identical_to_device_api": same,
            "note": "pageable host X/B/Y; H2D + kernels + D2H, row bands through pinned slots over 3 streams; "
                    "the host API's exact mode (K unsplit, no MFMA: dense.c gemm_basic's order), so its bits equal "
                    "the device API's only where the device launch does not split K"}


MFMA_BF16_PEAK = 2.5e15  # dense bf16 MFMA FLOP/s (MI355X_MICROARCH.md chip table, spec)


def other_configs(args, tcsc_amd, workloads, dev, sh, timed, skip):
    """The other BASELINE configs on this GPU (not part of `value`): one full
    tcsc_gpu_sgemm per step (X staging + gather, or split + GEMM on the MFMA
    path for near-dense W), inputs resident, HIP events over 30 launches
    after 10 warm-up launches; each with the roof that binds it (LDS gather
    for the gather path, bf16 MFMA for the MFMA path) and, unless
    --no-cpu-baseline, the reference's CPU path timed beside it (SURVEY.md
    §8d: main.cpp's own loop for cfg 1-3, 1 warm-up + median of 3 for cfg 5)."""
    import torch

    res = {}
    for idx in (1, 2, 3, 5):
        if idx == skip:
            continue
        c = workloads.CONFIGS[idx]
        inp = workloads.make_device_inputs(c, 0, c.N, dev)
        csp = torch.empty(c.N + 1, dtype=torch.int32, device=dev)
        csn = torch.empty(c.N + 1, dtype=torch.int32, device=dev)
        npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], c.K, c.N, csp, csn, stream=sh)
        rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
        rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
        tcsc_amd.gpu_from_dense(inp["Wd"], c.K, c.N, csp, csn, rip, rin, stream=sh)
        del inp["Wd"]
        plan = tcsc_amd.Plan.from_device(c.K, c.N, csp, csn, rip, rin, 0, c.N, dev.index or 0, sh)
        plan.reserve(c.M)
        Yc = torch.empty((c.M, c.N), device=dev)

        def one():
            plan.sgemm(inp["X"], inp["B"], Yc, c.M, c.N, c.variant, 0.2, sh)

        for _ in range(10):
            one()
        t = timed(one, 30)
        nnz = npos + nneg
        lpath, lslices = plan.launch_info(c.M)
        mfma = lpath == "mfma"
        path = {"mfma": "mfma (bf16 x3 split GEMM: k_split3 + k_gemm3)", "small": "small-M (one wave per column)",
                "gather": "gather (k_transpose + k_stream)"}[lpath] + \
            ((f", K split {lslices} ways, combined in the k_stream launch ({plan.combine_mode(c.M)})"
              if plan.launch_combine(c.M) else
              f", K split {lslices} ways + k_reduce4") if lslices > 1 else "")
        r = {
            "workload": c.describe(), "variant": c.variant, "nnz": nnz, "ms": t * 1e3,
            "g_add_ops_per_s": workloads.add_ops(c.M, nnz, c.N) / t / 1e9,
            "hbm_frac": workloads.algorithmic_bytes(c.M, c.K, c.N, nnz) / t / (HBM_PEAK_GBS * 1e9),
            "path": path,
        }
        if mfma:
            # the split GEMM's depth: 3 parts of each 64-k block (tcsc_internal.h
            # mfma_ldk = 3 * kMfmaBlk * ceil(K / kMfmaBlk), kMfmaBlk = 64)
            ldk = 3 * 64 * ((c.K + 63) // 64)
            flops = 2.0 * c.M * c.N * ldk
            r["mfma_flops_per_step"] = flops
            r["mfma_frac"] = flops / t / MFMA_BF16_PEAK
            # the north star's add/sub-only contract on the same W (tcsc.c:86-93): the
            # gather path timed beside the MFMA one (a plan made with TCSC_PATH=gather)
            r["gather_path"] = gather_leg(tcsc_amd, workloads, c, inp, csp, csn, rip, rin, nnz, dev, sh, timed)
        else:
            r["lds_gather_frac"] = (c.M * nnz / t) / LDS_GATHER_PEAK
        if not args.no_cpu_baseline:
            cb = cpu_baseline(args, c, c.variant, inp["X"], inp["B"], csp, csn, rip[:npos], rin[:nneg],
                              protocol="harness" if idx <= 3 else "median3", seconds=8.0, legs=False)
            r["cpu_baseline"] = cb
            r["gpu_vs_cpu_1core"] = r["g_add_ops_per_s"] / cb["value"]
        res[c.name] = r
        plan.destroy()
        del inp, csp, csn, rip, rin, Yc
    torch.cuda.empty_cache()
    return res


def gather_leg(tcsc_amd, workloads, c, inp, csp, csn, rip, rin, nnz, dev, sh, timed):
    """The add/sub-only gather path (k_transpose + k_stream) on a config the
    cost model sends to the MFMA path: the same W in a plan built with
    TCSC_PATH=gather, the same protocol (10 warm-up + 30 timed launches)."""
    import torch

    old = os.environ.get("TCSC_PATH")
    os.environ["TCSC_PATH"] = "gather"
    try:
        gp = tcsc_amd.Plan.from_device(c.K, c.N, csp, csn, rip, rin, 0, c.N, dev.index or 0, sh)
    finally:
        if old is None:
            del os.environ["TCSC_PATH"]
        else:
            os.environ["TCSC_PATH"] = old
    gp.reserve(c.M)
    Yg = torch.empty((c.M, c.N), device=dev)

    def one():
        gp.sgemm(inp["X"], inp["B"], Yg, c.M, c.N, c.variant, 0.2, sh)

    for _ in range(10):
        one()
    t = timed(one, 30)
    lpath, lslices = gp.launch_info(c.M)
    gp.destroy()
    del Yg
    return {"path": f"{lpath} (k_transpose + k_stream{f', K split {lslices} ways' if lslices > 1 else ''}), "
                    "add/sub only, no MFMA", "ms": t * 1e3,
            "g_add_ops_per_s": workloads.add_ops(c.M, nnz, c.N) / t / 1e9,
            "hbm_frac": workloads.algorithmic_bytes(c.M, c.K, c.N, nnz) / t / (HBM_PEAK_GBS * 1e9),
            "lds_gather_frac": (c.M * nnz / t) / LDS_GATHER_PEAK}


def validate_against_dense(tcsc_amd, cfg, ncols, variant, X, Wd, B, Y, step, sh):
    """One step's full M x ncols output against the dense product of the same
    ternary W (tcsc_gpu_dense_sgemm: fp32 rocBLAS SGEMM + the same bias/PReLU
    epilogue), per element |y - y_dense| <= max(1, a) * 2^-19 * S with
    S = |B| + |X| . |W| from the same dense path on magnitudes: the oracle's
    2^-20 bound once for each of the two results.  Runs on the
    GPU; raises (the run fails, as main.cpp exit(1)s) on a violation."""
    import torch

    a = 0.2
    step()
    Yd = torch.empty_like(Y)
    tcsc_amd.dense_sgemm(X, Wd, B, Yd, cfg.M, ncols, cfg.K, ncols, variant, a, sh)
    S = torch.empty_like(Y)
    Xa, Wa, Ba = X.abs(), Wd.abs(), B.abs()
    tcsc_amd.dense_sgemm(Xa, Wa, Ba, S, cfg.M, ncols, cfg.K, ncols, "basic", 0.0, sh)
    del Xa, Wa, Ba
    bound = S.mul_(max(1.0, a) * 2.0 ** -19)
    err = (Y - Yd).abs_()
    nan_mismatch = int((Y.isnan() != Yd.isnan()).sum().item())
    ratio = torch.where(err == 0, torch.zeros_like(err), err / bound)
    ratio = torch.nan_to_num(ratio, nan=0.0, posinf=float("inf"))
    worst = float(ratio.max().item())
    if nan_mismatch or not worst <= 1.0:
        raise SystemExit(f"validation failed: worst |y - y_dense| / bound = {worst:.3g}, "
                         f"NaN mismatches {nan_mismatch}")
    return {"against": "dense fp32 rocBLAS SGEMM of the same ternary W (+ same epilogue)",
            "bound": "max(1,a) * 2^-19 * (|B| + |X|.|W|) per element", "elements": Y.numel(),
            "worst_err_over_bound": worst}


def check_determinism(step, Y, n):
    """The gather reduces in a fixed order (no atomics; split-K partials are
    combined in slice order), so repeated launches must give bit-identical
    outputs: n back-to-back launches, the last output compared bit for bit
    with the first.  (Also lets the GPU clocks settle before the warm-up,
    DESIGN.md §7 "clock ramp".)"""
    import torch

    step()
    first = Y.view(torch.int32).clone()
    for _ in range(n - 1):
        step()
    same = bool(torch.equal(Y.view(torch.int32), first))
    if not same:
        raise SystemExit(f"validation failed: output changed over {n} identical launches")
    return {"launches": n, "bit_identical": same}


def graph_line(plan, X, B, Y, M, ncols, variant, steps, stream, eager_s):
    """`steps` launches of the step captured in one HIP graph (include/tcsc_gpu.h:
    a launch whose workspace is reserved allocates nothing and never synchronises),
    replayed after one warm-up replay; HIP events around the replay."""
    import torch

    side = torch.cuda.Stream(device=X.device)
    side.wait_stream(stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side):
        h = torch.cuda.current_stream().cuda_stream
        for _ in range(steps):
            plan.sgemm(X, B, Y, M, ncols, variant, 0.2, h)
    g.replay()  # on torch's current stream
    torch.cuda.synchronize()
    cur = torch.cuda.current_stream(X.device)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(cur)
    g.replay()
    b.record(cur)
    b.synchronize()
    ms = a.elapsed_time(b) / steps
    del g
    return {"steps_per_graph": steps, "ms_per_step": ms, "vs_eager": ms / (eager_s / steps * 1e3)}


def bcsr_line(cfg, Wd, X, B, Y, nnz, tcsc_s, timed, sh, n):
    """the same W as 1x8 BCSR (the block shape of the
    reference's test/test_bcsr.cpp and of its AVX kernels), k_bcsr timed on
    the staged X^T like k_stream.  Work: every stored value (zeros inside
    stored blocks included) is one update per row, M*k*8; its roof is the
    VALU (one FMA per update for basic; PReLU after every update, bcsr.c:209,
    adds a multiply, a compare and a select)."""
    import torch
    from tcsc_amd import bcsr

    t0 = time.perf_counter()
    W = bcsr.BcsrMatrix.from_dense(Wd.cpu().numpy(), 1, 8)
    build_s = time.perf_counter() - t0
    plan = bcsr.BcsrPlan(W, X.device.index or 0, sh)
    plan.reserve(cfg.M, cfg.K)
    plan.prepare_x(X, cfg.M, cfg.K, sh)
    res = {"kernel": "k_bcsr", "block": "1x8", "blocks": W.k, "stored_values": W.k * 8,
           "host_bcsr_from_dense_s": build_s}
    updates = cfg.M * W.k * 8
    N = Wd.shape[1]
    Yb = torch.empty_like(Y)  # Y keeps the TCSC output (host_api_line compares against it)
    for v in ("basic", "prelu_basic"):
        plan.sgemm_prepared(B, Yb, cfg.M, N, cfg.K, N, v, 0.2, sh)
        t = timed(lambda: plan.sgemm_prepared(B, Yb, cfg.M, N, cfg.K, N, v, 0.2, sh), n)
        res[v] = {"ms": t * 1e3, "g_updates_per_s": updates / t / 1e9, "valu_fma_frac": updates / t / VALU_ADD_PEAK,
                  "effective_g_add_ops_per_s": (cfg.M * nnz + cfg.M * N) / t / 1e9,
                  "ms_vs_tcsc_k_stream": t / tcsc_s}
    plan.destroy()
    W.free()
    del Yb
    return res


def usable_cpus():
    """(cores this process may use, what the host reports): the affinity
    mask, capped by the cgroup CPU quota when one is set (a GPU box's share
    of a larger host), and os.cpu_count() / nproc for the record."""
    n_host = os.cpu_count() or 1
    try:
        n_aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        n_aff = n_host
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(period)))
    except (OSError, ValueError):
        quota = None
    return (min(n_aff, quota) if quota else n_aff), {"nproc": n_host, "affinity": n_aff, "cgroup_quota_cpus": quota}


# main.cpp:9-17: NUM_RUNS 20, CYCLES_REQUIRED 1e8 (TSC cycles), REP 50.  The
# harness's cycle counter ticks at the TSC rate (~2 GHz on these hosts), so
# 1e8 cycles is taken as 0.05 s of wall time.
NUM_RUNS, REP, CYCLES_REQUIRED_S = 20, 50, 0.05


def harness_protocol(call):
    """measure_tcsc_cycles (main.cpp:54-113) around a zero-argument call:
    warm-up passes of num_runs calls, num_runs scaled by CYCLES_REQUIRED /
    cycles until the multiplier is <= 2, then REP passes of num_runs calls;
    returns (mean seconds per call over the REP passes, num_runs)."""
    num_runs, multiplier = NUM_RUNS, 1.0
    while True:
        num_runs = max(1, int(num_runs * multiplier))
        t0 = time.perf_counter()
        for _ in range(num_runs):
            call()
        multiplier = CYCLES_REQUIRED_S / max(time.perf_counter() - t0, 1e-9)
        if multiplier <= 2:
            break
    total = 0.0
    for _ in range(REP):
        t0 = time.perf_counter()
        for _ in range(num_runs):
            call()
        total += (time.perf_counter() - t0) / num_runs
    return total / REP, num_runs


def cpu_baseline(args, cfg, variant, X, B, csp, csn, rip, rin, protocol="median3", seconds=None, legs=True):
    """SURVEY.md §8d, on this GPU box's host, rank 0 at N=1, on row samples
    of the same workload (all columns):
      * value: the reference's own tcsc_sgemm_<variant> (sparse/tcsc.c
        compiled in place with its authors' flags, -O3 -ffast-math, AVX2+FMA:
        oracle/_ref/libtcsc_ref_fast.so) on 1 core, as benchmark.sh pins it
        (benchmark.sh:36), timed with
          protocol "harness": the harness's own loop (main.cpp:54-113: warm-up
            until a pass covers CYCLES_REQUIRED, then REP passes of num_runs
            calls, the mean per call) on a row sample sized so one call takes
            a few ms (cfg 1-3);
          protocol "median3": 1 warm-up pass over the sample, then the median
            of 3 passes (cfg 4-5, where one harness run would take hours);
      * (legs=True) the same sources built IEEE (-O2, no fast-math: the parity
        build) and the oracle's C restatement, each 1 core, median of 3;
      * the reference's own OpenMP sparseGEMM_PReLU / sparseGEMM
        (SparseGEMM.h:104-168, the multi-core form it ships) on every usable
        core, median of 3 (all M rows, or a row sample of about 1 s per pass).
    Falls back to the oracle restatement ("port") where oracle/_ref is absent."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import numpy as np

    import pyoracle

    o = pyoracle.load_oracle()
    ref_fast = pyoracle.load_reference(fast=True)
    ref_ieee = pyoracle.load_reference() if legs else None
    ncols = csp.numel() - 1
    W = pyoracle.TCSC(cfg.K, ncols, csp.cpu().numpy(), csn.cpu().numpy(), rip.cpu().numpy(), rin.cpu().numpy())
    Bh = B.cpu().numpy()
    Xh = X.cpu().numpy()
    nnz = W.nnz
    var = variant if variant in pyoracle.VARIANTS else "prelu_basic"
    seconds = args.cpu_seconds if seconds is None else seconds

    def rate(rows, t):
        return (rows * nnz + rows * ncols) / t / 1e9

    def probe(fn):
        """seconds per row of one call, from an 8-row probe call (sizes the sample only)"""
        n = min(8, cfg.M)
        fn(var, Xh[:n], W, Bh, 0.2)  # first touch of W and the code
        t0 = time.perf_counter()
        fn(var, Xh[:n], W, Bh, 0.2)
        return (time.perf_counter() - t0) / n

    def median3(fn, secs):
        """1 warm-up pass over the sample, then the median of 3 timed passes
        over it; the sample is sized so that one pass takes about `secs`."""
        rows = int(min(cfg.M, max(8, secs / max(probe(fn), 1e-9))))
        fn(var, Xh[:rows], W, Bh, 0.2)  # warm-up pass
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            fn(var, Xh[:rows], W, Bh, 0.2)
            ts.append(time.perf_counter() - t0)
        t = float(np.median(ts))
        return {"rows": rows, "median_s": t, "value": rate(rows, t), "protocol": "1 warm-up pass + median of 3"}

    def harness(lib):
        """main.cpp's loop on a row sample of ~2.5 ms per call"""
        rows = int(min(cfg.M, max(1, 2.5e-3 / max(probe(lib.sgemm), 1e-9))))
        call = lib.sgemm_call(var, Xh[:rows], W, Bh, 0.2)
        t, runs = harness_protocol(call)
        return {"rows": rows, "mean_call_s": t, "num_runs": runs, "rep": REP, "value": rate(rows, t),
                "protocol": f"main.cpp:54-113 loop (NUM_RUNS {NUM_RUNS} scaled to >= {CYCLES_REQUIRED_S} s "
                            f"per pass -> {runs}, REP {REP}, mean per call)"}

    out_legs = {}
    if ref_fast:
        out_legs["reference_fast"] = harness(ref_fast) if protocol == "harness" else median3(ref_fast.sgemm,
                                                                                            seconds * 0.12)
    if ref_ieee:
        out_legs["reference_ieee"] = median3(ref_ieee.sgemm, seconds * 0.05)
    if legs or not ref_fast:
        out_legs["port"] = median3(o.sgemm, seconds * 0.05)
    threads, cpu_info = usable_cpus()
    omp_env = os.environ.get("OMP_NUM_THREADS")
    if omp_env:
        threads = min(threads, int(omp_env)) if omp_env.isdigit() else threads
    omp_lib = ref_fast or ref_ieee
    prelu = var in pyoracle.PRELU_VARIANTS
    # all rows unless a pass would take much longer than ~1 s (cfg 5)
    omp_rows = cfg.M
    per_row_1core = 1.0 / (out_legs.get("reference_fast") or out_legs["port"])["value"] * (nnz + ncols) / 1e9
    if per_row_1core * cfg.M / max(threads, 1) > 1.0:
        omp_rows = int(max(threads, min(cfg.M, 1.0 * threads / per_row_1core)))
    ts = []
    for i in range(4):  # the first pass starts the thread team (not timed)
        t0 = time.perf_counter()
        if omp_lib:
            o.set_omp_threads(threads)
            omp_lib.sparse_gemm(Xh[:omp_rows], W, Bh, prelu=prelu, a=0.2)
        else:
            o.sparse_gemm_omp(Xh[:omp_rows], W, Bh, prelu=prelu, a=0.2, threads=threads)
        if i:
            ts.append(time.perf_counter() - t0)
    t_omp = float(np.median(ts))
    main = out_legs.get("reference_fast") or out_legs.get("reference_ieee") or out_legs["port"]
    kind = "reference" if (ref_fast or ref_ieee) else "port"
    flags = ("g++ -O3 -ffast-math -mavx2 -mfma (the reference's build_and_run_m1.sh:77 flags, "
             "-march=native pinned to AVX2+FMA)" if ref_fast else
             "g++ -O2 -fno-fast-math -ffp-contract=off (IEEE parity build)" if ref_ieee else "gcc -O2")
    how = (f"{main['protocol']} ({main['mean_call_s'] * 1e3:.2f} ms per call)" if "mean_call_s" in main else
           f"{main['protocol']} passes ({main['median_s']:.2f} s each)")
    out = {
        "value": main["value"],
        "unit": "G-add-ops/s",
        "cores": 1,
        "kind": kind,
        "sample": (f"{cfg.name}: first {main['rows']} of {cfg.M} rows x all {ncols} columns, tcsc_sgemm_{var}, "
                   f"{'sparse/tcsc.c compiled in place' if kind == 'reference' else 'oracle/tcsc_oracle.c'} "
                   f"({flags}), 1 core, {how}"),
        "flags": flags,
        "legs": out_legs,
        "omp_value": rate(omp_rows, t_omp),
        "omp_cores": threads,
        "omp_cores_of_host": f"{threads} of {cpu_info['nproc']} host CPUs (affinity/cgroup share)",
        "omp_kind": (f"reference sparseGEMM{'_PReLU' if prelu else ''} (SparseGEMM.h:"
                     f"{'151-168' if prelu else '104-119'}, OpenMP)") if omp_lib else
                    "oracle_sparse_gemm_omp restatement",
        "omp_sample": f"first {omp_rows} of {cfg.M} rows x {ncols} columns, 1 warm-up + median of 3 ({t_omp:.3g} s each)",
        "host_cpus": cpu_info,
    }
    return out


if __name__ == "__main__":
    main()
