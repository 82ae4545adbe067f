#!/usr/bin/env python3
"""Where a chunk of k_stream goes (TCSC_STAMPS diagnostic build,
lib/abl/libtcsc_amd_stamps.so; read shares, never the run time).

Per wave the kernel sums, over its chunk loop, the s_memtime cycles of
  gather : barrier release -> end of its gather
  post   : end of gather -> next stream landed + DMA issued
  wait   : that -> next barrier release (vmcnt wait + barrier)
This runs BASELINE cfg 4 (or argv[1]) through the device API and reports
per-chunk means: over all waves, for the wave that waited least at the
barrier in its workgroup (the critical one), and the chunk period.

    python tools/stamps.py [cfg] [path/to/libtcsc_amd_stamps.so]
"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd")
cfg_idx = int(sys.argv[1]) if len(sys.argv) > 1 else 4
os.environ["TCSC_AMD_LIB"] = sys.argv[2] if len(sys.argv) > 2 else os.path.join(PKG, "lib", "abl",
                                                                                 "libtcsc_amd_stamps.so")
sys.path.insert(0, PKG)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tcsc_amd  # noqa: E402
from tcsc_amd import workloads  # noqa: E402

cfg = workloads.CONFIGS[cfg_idx]
dev = torch.device("cuda:0")
inp = workloads.make_device_inputs(cfg, 0, cfg.N, dev)
csp = torch.empty(cfg.N + 1, dtype=torch.int32, device=dev)
csn = torch.empty(cfg.N + 1, dtype=torch.int32, device=dev)
npos, nneg = tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, cfg.N, csp, csn)
rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
tcsc_amd.gpu_from_dense(inp["Wd"], cfg.K, cfg.N, csp, csn, rip, rin)
del inp["Wd"]
plan = tcsc_amd.Plan.from_device(cfg.K, cfg.N, csp, csn, rip, rin)
plan.reserve(cfg.M)
Y = torch.empty((cfg.M, cfg.N), device=dev)
plan.prepare_x(inp["X"], cfg.M)
for _ in range(30):
    plan.sgemm_prepared(inp["B"], Y, cfg.M, cfg.N, cfg.variant, 0.2)
torch.cuda.synchronize()
L = tcsc_amd.lib()
waves, n_wg = 16, 4096
buf = np.zeros(n_wg * waves * 4, np.uint64)
L.tcsc_debug_stamps.argtypes = [C.c_void_p, C.c_size_t]
assert L.tcsc_debug_stamps(buf.ctypes.data, buf.nbytes) == 0
s = buf.reshape(n_wg, waves, 4).astype(np.float64)
used = s[:, :, 3].max(axis=1) > 0
s = s[used]
nch = (cfg.K + 47) // 48
info = plan.info()
print(f"cfg{cfg_idx}: {s.shape[0]} workgroups, {nch} chunks (assumes one K slice; n_groups {info.get('n_groups')})")
g, p, w, tot = (s[:, :, i] / nch for i in range(4))
crit = np.argmin(w, axis=1)
rows = np.arange(s.shape[0])
print(f"chunk period (total / chunks): {tot.mean():8.1f} cycles")
print(f"all waves   : gather {g.mean():7.1f}  post {p.mean():7.1f}  wait {w.mean():7.1f}")
print(f"critical    : gather {g[rows, crit].mean():7.1f}  post {p[rows, crit].mean():7.1f}  "
      f"wait {w[rows, crit].mean():7.1f}")
for k in range(waves):
    print(f"  wave {k:2d}: gather {g[:, k].mean():7.1f} post {p[:, k].mean():7.1f} wait {w[:, k].mean():7.1f}")
