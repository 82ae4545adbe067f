"""Gather vs MFMA crossover on the device API.

For each shape (M, K, N) and W density, builds two device plans of the same
W -- TCSC_PATH=gather (k_transpose + k_stream, the cost model's split-K) and
TCSC_PATH=mfma (k_split3 + k_gemm3 + k_fixup), and the default plan (auto:
the per-launch cost model's choice) -- and times one full
tcsc_gpu_sgemm step of each with HIP events on the launch stream (median of
`reps` after `warm` warm-up steps).  Prints one JSON line per (shape,
density) with both times and the winner, so the default plan's density and
M thresholds (csrc/tcsc_api.cpp kMfmaDensity, kMfmaMinM) can be set from
measurement.

  python tools/crossover.py [--shapes 2048x8192x8192,...] [--densities 0.05,0.1,...]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "sparse-matrix-multiplication-benchmark_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="2048x8192x8192,4096x4096x4096,256x8192x8192,128x8192x8192,64x8192x8192")
    ap.add_argument("--densities", default="0.04,0.06,0.08,0.1,0.12,0.15,0.2,0.3,0.5")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--warm", type=int, default=3)
    ap.add_argument("--modes", default="gather,mfma,auto", help="plans to time (a subset of gather,mfma,auto)")
    args = ap.parse_args()
    import torch

    import tcsc_amd

    tcsc_amd.require_gpu()
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    sh = st.cuda_stream

    def time_plan(plan, X, B, Y, M, N):
        plan.reserve(M)
        for _ in range(args.warm):
            plan.sgemm(X, B, Y, M, N, "basic", 0.0, sh)
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            plan.sgemm(X, B, Y, M, N, "basic", 0.0, sh)
            e1.record(st)
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    for shape in args.shapes.split(","):
        M, K, N = (int(v) for v in shape.split("x"))
        g = torch.Generator(device=dev)
        g.manual_seed(M * 7 + K)
        X = torch.rand((M, K), generator=g, device=dev) * 2 - 1
        B = torch.rand((N,), generator=g, device=dev) * 2 - 1
        Y = torch.empty((M, N), device=dev)
        for d in (float(v) for v in args.densities.split(",")):
            u = torch.rand((K, N), generator=g, device=dev)
            Wd = torch.zeros((K, N), device=dev)
            Wd[u < d / 2] = 1.0
            Wd[(u >= d / 2) & (u < d)] = -1.0
            del u
            csp = torch.empty(N + 1, dtype=torch.int32, device=dev)
            csn = torch.empty(N + 1, dtype=torch.int32, device=dev)
            npos, nneg = tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn)
            rip = torch.empty(max(npos, 1), dtype=torch.int32, device=dev)
            rin = torch.empty(max(nneg, 1), dtype=torch.int32, device=dev)
            tcsc_amd.gpu_from_dense(Wd, K, N, csp, csn, rip, rin)
            del Wd
            out = {"M": M, "K": K, "N": N, "density": d, "nnz": npos + nneg}
            for mode in args.modes.split(","):
                if mode == "auto":
                    os.environ.pop("TCSC_PATH", None)
                else:
                    os.environ["TCSC_PATH"] = mode
                plan = tcsc_amd.Plan.from_device(K, N, csp, csn, rip, rin)
                plan.reserve(M)  # the gather's K split depends on the workspace
                path, slices = plan.launch_info(M)
                out[mode + "_path"] = f"{path}/s{slices}"
                out[mode + "_ms"] = time_plan(plan, X, B, Y, M, N)
                plan.destroy()
            os.environ.pop("TCSC_PATH", None)
            if "gather_ms" in out and "mfma_ms" in out:
                out["winner"] = "mfma" if out["mfma_ms"] < out["gather_ms"] else "gather"
                out["mfma_over_gather"] = out["mfma_ms"] / out["gather_ms"]
                if "auto_ms" in out:
                    out["auto_over_best"] = out["auto_ms"] / min(out["mfma_ms"], out["gather_ms"])
            print(json.dumps(out), flush=True)
            del csp, csn, rip, rin
            torch.cuda.empty_cache()
            time.sleep(0.01)


if __name__ == "__main__":
    main()
