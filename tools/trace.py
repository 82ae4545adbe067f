#!/usr/bin/env python3
"""Per-interval timeline of the gather kernel (TCSC_TRACE diagnostic build).

Each wave records, for every K-chunk interval c: the shader clock at the top
of the interval, after the barrier, after its gather; its batch count; its
HW_ID (SIMD, wave slot).  This script runs cfg 4 once on that build, pulls
the records out of Y and reports where an interval's time goes:

  * interval length   = next barrier release - this barrier release
  * slowest gather    = max over the workgroup's waves of (gather end - release)
  * tail              = interval length - slowest gather (DMA issue, stream
                        load, loop overhead of the last wave, barrier latency)
  * how well the batch count predicts a wave's gather time, and whether the
    SIMD or wave slot does.

Usage (GPU box): python tools/trace.py [cfg] [--save gpurun_out/trace.npz]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["TCSC_AMD_LIB"] = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd", "lib", "abl",
                                          "libtcsc_amd_trace.so")
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))
import numpy as np  # noqa: E402


def analyse(tr, nb_waves=16):
    """tr: [n_wg, waves, intervals, 6] uint32 records."""
    t0 = tr[..., 0].astype(np.int64)
    t1 = tr[..., 1].astype(np.int64)
    ts = tr[..., 2].astype(np.int64)
    t2 = tr[..., 3].astype(np.int64)
    nb = tr[..., 4].astype(np.int64)
    hw = tr[:, :, 0, 5].astype(np.int64)
    # unwrap 32-bit clocks relative to the wave's first stamp
    base = t0[:, :, :1].min(axis=1, keepdims=True)  # one clock per CU
    t0 = (t0 - base) % (1 << 32)
    t1 = (t1 - base) % (1 << 32)
    ts = (ts - base) % (1 << 32)
    t2 = (t2 - base) % (1 << 32)
    rel = t1.min(axis=1)  # barrier release per (wg, c)
    length = np.diff(rel, axis=1)  # interval c: release(c+1) - release(c)
    g = t2 - t1  # per-wave gather (+trace store) duration
    gmax = g.max(axis=1)[:, :-1]
    gmean = g.mean(axis=1)[:, :-1]
    nbmax = nb.max(axis=1)[:, :-1]
    nbmean = nb.mean(axis=1)[:, :-1]
    out = {}
    out["interval_cycles_mean"] = float(length.mean())
    out["slowest_gather_mean"] = float(gmax.mean())
    out["mean_gather_mean"] = float(gmean.mean())
    out["tail_mean"] = float((length - gmax).mean())
    sw = ts - t1  # barrier release -> entry stream in SGPRs
    out["stream_wait_by_slot"] = [float(sw[:, 4 * k:4 * k + 4].mean()) for k in range(4)]
    out["gather_by_slot"] = [float((t2 - ts)[:, 4 * k:4 * k + 4].mean()) for k in range(4)]
    post = t0[:, :, 1:] - t2[:, :, :-1]
    out["post_gather_by_slot"] = [float(post[:, 4 * k:4 * k + 4].mean()) for k in range(4)]
    bw = t1[:, :, 1:] - t0[:, :, 1:]
    out["vmcnt_barrier_by_slot"] = [float(bw[:, 4 * k:4 * k + 4].mean()) for k in range(4)]
    r0 = t1.min(axis=1, keepdims=True)
    out["gather_end_after_release_by_slot"] = [float((t2 - r0)[:, 4 * k:4 * k + 4].mean()) for k in range(4)]
    out["next_top_after_release_by_slot"] = [float((t0[:, :, 1:] - r0[:, :, :-1])[:, 4 * k:4 * k + 4].mean())
                                             for k in range(4)]
    out["last_gather_end_after_release"] = float((t2 - r0).max(axis=1).mean())
    out["release_skew_by_slot"] = [float((t1 - t1.min(axis=1, keepdims=True))[:, 4 * k:4 * k + 4].mean())
                                   for k in range(4)]
    out["batches_max_mean"] = float(nbmax.mean())
    out["batches_mean"] = float(nbmean.mean())
    # linear fit gather ~ a + b*nb over all waves/intervals
    x = nb.reshape(-1).astype(np.float64)
    y = g.reshape(-1).astype(np.float64)
    A = np.vstack([np.ones_like(x), x]).T
    coef, *_ = np.linalg.lstsq(A, y, rcond=None)
    resid = y - A @ coef
    out["fit_cycles_fixed"] = float(coef[0])
    out["fit_cycles_per_batch"] = float(coef[1])
    out["fit_r2"] = float(1 - resid.var() / y.var())
    # which wave is slowest: is it the one with the most batches?
    arg_slow = g.argmax(axis=1)[:, :-1]
    arg_most = nb.argmax(axis=1)[:, :-1]
    out["slowest_is_most_batches"] = float((arg_slow == arg_most).mean())
    # per SIMD / wave slot residual
    simd = (hw >> 4) & 3
    slot = hw & 15
    r = resid.reshape(g.shape)
    per_simd = {int(s): float(r.transpose(0, 2, 1)[(simd == s)[:, None, :].repeat(g.shape[2], 1)].mean())
                for s in range(4)}
    out["resid_by_simd"] = per_simd
    slots = {}
    for s in np.unique(slot):
        m = (slot == s)[:, None, :].repeat(g.shape[2], 1)
        slots[int(s)] = float(r.transpose(0, 2, 1)[m].mean())
    out["resid_by_wave_slot"] = slots
    # order of gather end inside an interval vs wave index (arbitration)
    rank = g.argsort(axis=1).argsort(axis=1)  # 0 = fastest
    out["mean_rank_by_wave_index"] = [float(v) for v in rank.mean(axis=(0, 2))]
    return out


def main():
    import torch

    import tcsc_amd
    from tcsc_amd import workloads

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    cfg = workloads.CONFIGS[int(args[0]) if args else 4]
    save = None
    if "--save" in sys.argv:
        save = sys.argv[sys.argv.index("--save") + 1]
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
    nch = 32  # the kernel's trace window (kTraceN intervals from chunk 100)
    ngroups = (N + 15) // 16
    nwg = ((ngroups + 15) // 16) * ((M + 255) // 256)
    n = nwg * 16 * nch * 6
    assert n <= M * N
    tr = Y.view(torch.int32).flatten()[:n].cpu().numpy().view(np.uint32).reshape(nwg, 16, nch, 6)
    res = analyse(tr)
    for k, v in res.items():
        print(f"{k:28s} {v}")
    if save:
        np.savez_compressed(save, tr=tr[:256])


if __name__ == "__main__":
    main()
