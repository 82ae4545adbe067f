#!/usr/bin/env python3
"""Where a k_stream launch goes (TCSC_STAMPS diagnostic build,
lib/abl/libtcsc_amd_stamps.so; read shares, never the run time).

Per wave the kernel sums, over its chunk loop, the s_memtime cycles of
  gather : barrier release -> end of its gather
  post   : end of gather -> next stream landed + DMA issued
  wait   : that -> next barrier release (vmcnt wait + barrier)
and per workgroup it records s_memrealtime (100 MHz, one clock for the chip)
at entry, chunk-loop start, chunk-loop end, epilogue end (the Y or slab
stores issued) and kernel end (after the in-launch combine, if any).  This
runs a BASELINE config (rank 0's block of an S-way column split with
--shard-of S) through the device API and reports per-chunk means -- over
all waves, for the wave that waited least at the barrier in its workgroup
(the critical one) -- and the launch timeline: prologue, chunk loop,
epilogue and combine per workgroup, and the spread of workgroup starts and
ends.

    python tools/stamps.py [--cfg 4] [--shard-of S] [--lib path/to/libtcsc_amd_stamps.so]
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd")
ap = argparse.ArgumentParser()
ap.add_argument("cfg_pos", nargs="?", type=int, default=None)
ap.add_argument("--cfg", type=int, default=4)
ap.add_argument("--shard-of", type=int, default=1)
ap.add_argument("--lib", default=os.path.join(PKG, "lib", "abl", "libtcsc_amd_stamps.so"))
args = ap.parse_args()
cfg_idx = args.cfg_pos if args.cfg_pos is not None else args.cfg
os.environ["TCSC_AMD_LIB"] = args.lib
os.environ["TCSC_ALLOW_DIAG"] = "1"  # the stamps build is diagnostic
sys.path.insert(0, PKG)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tcsc_amd  # noqa: E402
from tcsc_amd import workloads  # noqa: E402
from tcsc_amd.shard import column_range  # noqa: E402

cfg = workloads.CONFIGS[cfg_idx]
c0, c1 = column_range(cfg.N, args.shard_of, 0) if args.shard_of > 1 else (0, cfg.N)
N = c1 - c0
dev = torch.device("cuda:0")
inp = workloads.make_device_inputs(cfg, c0, c1, dev)
csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, N, csp, csn)
rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, N, csp, csn, rip, rin)
del inp["Wd"]
plan = tcsc_amd.Plan.from_device(cfg.K, N, csp, csn, rip, rin)
plan.reserve(cfg.M)
Y = torch.empty((cfg.M, N), device=dev)
plan.prepare_x(inp["X"], cfg.M)
for _ in range(30):
    plan.sgemm_prepared(inp["B"], Y, cfg.M, N, cfg.variant, 0.2)
torch.cuda.synchronize()
path, slices = plan.launch_info(cfg.M)
combine = plan.launch_combine(cfg.M) if slices > 1 else False
L = tcsc_amd.lib()
waves, n_wg = 16, 4096
buf = np.zeros(n_wg * waves * 4, np.uint64)
L.tcsc_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert L.tcsc_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.reshape(n_wg, waves, 4).astype(np.float64)
used = s[:, :, 3].max(axis=1) > 0
s = s[used]
nch = (cfg.K + 47) // 48
cps = (nch + slices - 1) // slices
print(f"cfg{cfg_idx} cols [{c0}, {c1}) M {cfg.M}: {s.shape[0]} workgroups, {nch} chunks, {slices} K slice(s) "
      f"({cps} chunks each), combine in launch: {combine}")
g, p, w, tot = (s[:, :, i] / cps for i in range(4))
crit = np.argmin(w, axis=1)
rows = np.arange(s.shape[0])
print(f"chunk period (total / chunks): {tot.mean():8.1f} cycles")
print(f"all waves   : gather {g.mean():7.1f}  post {p.mean():7.1f}  wait {w.mean():7.1f}")
print(f"critical    : gather {g[rows, crit].mean():7.1f}  post {p[rows, crit].mean():7.1f}  "
      f"wait {w[rows, crit].mean():7.1f}")
for k in range(waves):
    print(f"  wave {k:2d}: gather {g[:, k].mean():7.1f} post {p[:, k].mean():7.1f} wait {w[:, k].mean():7.1f}")
try:
    L.tcsc_debug_wgtimes.argtypes = [C.c_void_p, C.c_size_t]
    tb = np.zeros(n_wg * 8, np.uint64)
    assert L.tcsc_debug_wgtimes(tb.ctypes.data, tb.nbytes) == 0
    t = tb.reshape(n_wg, 8)[:, :7].astype(np.float64)
    t = t[t[:, 0] > 0]
    t0 = t[:, 0].min()
    us = (t - t0) / 100.0  # 100 MHz ticks -> us
    pro, loop, epi, comb = (us[:, 1] - us[:, 0]), (us[:, 2] - us[:, 1]), (us[:, 3] - us[:, 2]), (us[:, 4] - us[:, 3])
    print(f"timeline of the last launch ({t.shape[0]} workgroups, us from the first workgroup's entry):")
    print(f"  entry      : first 0.0, last {us[:, 0].max():7.2f}, median {np.median(us[:, 0]):7.2f}")
    print(f"  prologue   : mean {pro.mean():7.2f}  max {pro.max():7.2f}   (entry -> chunk loop)")
    print(f"  chunk loop : mean {loop.mean():7.2f}  min {loop.min():7.2f}  max {loop.max():7.2f}")
    print(f"  epilogue   : mean {epi.mean():7.2f}  max {epi.max():7.2f}   (LDS transpose + Y/slab stores issued)")
    if (t[:, 5] > 0).all() and (t[:, 6] > 0).all():
        drain, bar = (us[:, 5] - us[:, 2]), (us[:, 6] - us[:, 5])
        print(f"    of which : loads drained {drain.mean():6.2f} (max {drain.max():6.2f}), "
              f"first barrier {bar.mean():6.2f} (max {bar.max():6.2f}), passes {(epi - drain - bar).mean():6.2f}")
    print(f"  combine    : mean {comb.mean():7.2f}  max {comb.max():7.2f}")
    print(f"  end        : first {us[:, 4].min():7.2f}, last {us[:, 4].max():7.2f}, median {np.median(us[:, 4]):7.2f}")
except (AttributeError, AssertionError) as e:
    print("no workgroup timeline in this build:", e)
