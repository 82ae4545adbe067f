"""CPU model of the reference harness's validation margin.

main.cpp validates tcsc_sgemm_basic against dense.c's gemm_basic with
compare()'s absolute 1e-4 (main.cpp:307-320, dense.c:42-59) on fresh
random_device data: X ~ U[-1, 1), W ternary with P(+-1) = 1/4 each
(init_rand_sparse(K, N, 2)), B ~ U[-1, 1).  This models, in numpy, what
|y_path - y_gemm_basic| looks like on its two M = 256 shapes for:

  * gemm_basic itself: y = 0; y = fl(y + x*w) over ascending k; fl(y + b)
    (sequential fp32, exactly dense.c:64-77 under IEEE flags);
  * the MFMA path (k_gemm3): x split exactly into bf16 parts h + m + l
    (truncations, tcsc_mfma.hip k_split3), the accumulator updated once per
    (64-k block, part, 32-k half) with the exactly-summed 32 products
    (one rounding per MFMA, the model DESIGN.md §4 uses), bias last;
  * the host API's exact mode (round 6): the fast order with K unsplit,
    i.e. gemm_basic's own sequence -- difference 0 by construction.

It prints, per shape, the largest difference over all draws, how many
elements passed 1e-4, and the empirical tail P(max over one case > t) for a
few thresholds, so DESIGN.md can state the failure probability per harness
run of the round-5 default (MFMA) path.  Usage:
  python tools/margin_model.py --draws 20
"""
import argparse
import json
import time

import numpy as np


def bf16_trunc(x):
    u = x.view(np.uint32) & np.uint32(0xFFFF0000)
    return u.view(np.float32)


def split3(x):
    h = bf16_trunc(x)
    r = (x - h).astype(np.float32)
    m = bf16_trunc(r)
    l = (r - m).astype(np.float32)
    return h, m, l


def gemm_basic_f32(X, W, B):
    M, K = X.shape
    y = np.zeros((M, W.shape[1]), np.float32)
    for k in range(K):
        w = W[k]
        nz = np.flatnonzero(w)
        if nz.size:  # zero products add +-0: an exact no-op on y
            y[:, nz] += X[:, k:k + 1] * w[nz]
    return (y + B).astype(np.float32)


def mfma_model(X, W, B, blk=64, half=32):
    M, K = X.shape
    parts = split3(X)
    W64 = W.astype(np.float64)
    acc = np.zeros((M, W.shape[1]), np.float32)
    for b0 in range(0, K, blk):
        for p in parts:
            for h0 in range(b0, min(b0 + blk, K), half):
                h1 = min(h0 + half, K)
                s = p[:, h0:h1].astype(np.float64) @ W64[h0:h1]  # exact: <= 32 products of <= 16 bits
                acc = (acc.astype(np.float64) + s).astype(np.float32)
    return (acc + B).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--draws", type=int, default=10)
    ap.add_argument("--seed", type=int, default=2026)
    args = ap.parse_args()
    rng = np.random.default_rng(args.seed)
    out = {}
    for (M, K, N) in [(256, 512, 2048), (256, 1024, 4096)]:
        maxes, over = [], 0
        t0 = time.time()
        for d in range(args.draws):
            X = rng.uniform(-1, 1, (M, K)).astype(np.float32)
            W = rng.choice(np.array([-1, 0, 1], np.float32), size=(K, N), p=[0.25, 0.5, 0.25])
            B = rng.uniform(-1, 1, N).astype(np.float32)
            yg = gemm_basic_f32(X, W, B)
            ym = mfma_model(X, W, B)
            diff = np.abs(ym.astype(np.float64) - yg)
            maxes.append(float(diff.max()))
            over += int((diff > 1e-4).sum())
            print(f"{M}x{K}x{N} draw {d}: max |mfma - gemm_basic| = {maxes[-1]:.3e}, "
                  f"> 1e-4: {int((diff > 1e-4).sum())}  ({time.time() - t0:.0f} s)", flush=True)
        mx = np.array(maxes)
        out[f"{M}x{K}x{N}"] = {
            "draws": args.draws, "elements_per_draw": M * N, "max_diff": float(mx.max()),
            "mean_case_max": float(mx.mean()), "elements_over_1e-4": over,
            "P_case_max_over": {str(t): float((mx > t).mean()) for t in (5e-5, 7e-5, 8e-5, 9e-5, 1e-4)},
        }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
