#!/usr/bin/env python3
"""Generate tests/golden/bcsr/*.npz from the REFERENCE ITSELF (BCSR path).

Runs only in the build container: it needs oracle/_ref/libtcsc_ref.so, which
oracle/Makefile compiles from /root/reference/sparse/bcsr.c (+ tcsc.c,
dense.c) with IEEE flags (-O2 -fno-fast-math -ffp-contract=off; -mavx2 -mfma
for bcsr.c's intrinsics).  Inputs come from the seeded generators of
oracle/tcsc_oracle.c.

Each fixture holds
  X, B, a          inputs (X float32 M x K, B float32 N)
  Wd               dense K x N W handed to bcsr_from_dense (int8 when ternary, else float32)
  r, c             block shape
  rs, ci, vals     reference bcsr_from_dense output (bcsr.c:19-139); rs has
                   br+1 entries, those past `written` (uninitialised in the
                   reference) set to k
  written          entries of rs the reference writes (non-empty block rows + 1)
  Y_<variant>      reference bcsr_sgemm_<variant> output, for the variants the
                   shape allows (pyoracle.bcsr_variant_allowed)
  meta             JSON: shape, block, density, seed, flags, kind

Usage: python tests/golden/gen_golden_bcsr.py   (writes tests/golden/bcsr/)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
OUT = os.path.join(HERE, "bcsr")
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402

SEED0 = 0x7C5C0000 + 0x8000
A = 0.2  # main.cpp:268

# name, M, K, N, r, c, density, kind
CASES = [
    # test/test_bcsr.cpp:13-21: M=1, K=512, N=2048, 1x8 blocks, init_rand_sparse(.., 2)
    ("test_bcsr_1x8", 1, 512, 2048, 1, 8, 0.5, "float"),
    # the commented-out case of test/test_bcsr.cpp:8-12 (4x4 blocks)
    ("m16_k512_n1024_4x4", 16, 512, 1024, 4, 4, 0.05, "float"),
    # 8x8 blocks: the only shape bcsr_sgemm_avx2 is defined for (bcsr.c:347-377)
    ("m16_k256_n256_8x8", 16, 256, 256, 8, 8, 0.02, "float"),
    # cfg-like sparsity with the 1x8 shape, integer X (exact sums)
    ("m64_k256_n512_1x8_int", 64, 256, 512, 1, 8, 0.05, "int"),
    ("m300_k300_n160_1x8", 300, 300, 160, 1, 8, 0.05, "float"),
    # ragged: rows % r and cols % c != 0 (trailing rows / columns ignored,
    # bcsr.c:23-24; the columns past bc*c keep the bias)
    ("ragged_m5_k67_n70_3x8", 5, 67, 70, 3, 8, 0.1, "float"),
    # c > 8 (two 8-column strips per block column) and c < 8
    ("m20_k64_n64_16x16", 20, 64, 64, 16, 16, 0.01, "float"),
    ("m7_k5_n9_1x1", 7, 5, 9, 1, 1, 0.5, "float"),
    ("m9_k40_n42_2x3", 9, 40, 42, 2, 3, 0.1, "float"),
    # all-zero W (k = 0) and fully dense W
    ("allzero_m3_k16_n16_2x8", 3, 16, 16, 2, 8, 0.0, "float"),
    ("dense_m4_k32_n32_2x8", 4, 32, 32, 2, 8, 1.0, "int"),
]


def make_inputs(o, M, K, N, density, seed, kind):
    if kind == "int":
        X = o.integers((M, K), seed, 512)
        B = o.integers((N,), seed + 1, 512)
    else:
        X = o.uniform((M, K), seed)
        B = o.uniform((N,), seed + 1)
    Wd = o.ternary((K, N), density, seed + 2)
    return X, B, Wd


def run(ref, name, X, B, Wd, r, c, meta):
    W, written = ref.bcsr_from_dense(Wd, r, c)
    N = B.size
    tern = bool(np.all(np.isin(Wd, (-1.0, 0.0, 1.0))) and not np.any(np.signbit(Wd[Wd == 0])))
    arrays = dict(X=X, B=B, a=np.float32(A), Wd=Wd.astype(np.int8 if tern else np.float32), r=np.int32(r), c=np.int32(c),
                  rs=W.b_row_start, ci=W.b_col_idx, vals=W.b_values, written=np.int32(written))
    for v in pyoracle.BCSR_VARIANTS:
        if pyoracle.bcsr_variant_allowed(v, r, c, N):
            arrays["Y_" + v] = ref.bcsr_sgemm(v, X, W, B, A)
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)
    print(path, "k", W.k, "written", written, "variants", [k[2:] for k in arrays if k.startswith("Y_")])


def main():
    ref = pyoracle.load_reference()
    if ref is None:
        sys.exit("oracle/_ref/libtcsc_ref.so missing: run `make -C oracle ref` (needs /root/reference)")
    o = pyoracle.load_oracle()
    os.makedirs(OUT, exist_ok=True)
    flags = "g++ -O2 -fno-fast-math -ffp-contract=off -mavx2 -mfma (oracle/Makefile)"
    src = "reference sparse/bcsr.c via oracle/_ref"
    for i, (name, M, K, N, r, c, d, kind) in enumerate(CASES):
        seed = SEED0 + 10 * i
        X, B, Wd = make_inputs(o, M, K, N, d, seed, kind)
        run(ref, name, X, B, Wd, r, c, dict(name=name, M=M, K=K, N=N, r=r, c=c, density=d, seed=seed, kind=kind,
                                            flags=flags, source=src))

    # empty block rows: b_row_start is compacted by the reference
    # (bcsr.c:114-117) -- rows 2 and 5 of 10 hold no +-1
    seed = SEED0 + 500
    X, B, Wd = make_inputs(o, 3, 40, 32, 0.08, seed, "float")
    Wd[8:12] = 0.0
    Wd[20:24] = 0.0
    run(ref, "empty_block_rows_4x8", X, B, Wd, 4, 8,
        dict(name="empty_block_rows_4x8", M=3, K=40, N=32, r=4, c=8, density=0.08, seed=seed, kind="float",
             flags=flags, source=src + "; block rows 2 and 5 zeroed"))

    # non-ternary values inside stored blocks (bcsr.c:132 keeps them):
    # non-power-of-two values make the basic (mul + add) and avx (fma)
    # variants round differently
    seed = SEED0 + 600
    vals = np.array([1.0, -1.0, 0.0, -0.0, 0.5, 2.0, -1.0000001, 0.99999994, 0.3, -7.25, 1.1, -0.7],
                    dtype=np.float32)
    U = o.uniform((38, 32), seed)
    Wd = vals[(np.abs(U) * 1e6).astype(np.int64) % len(vals)]
    X = o.uniform((6, 38), seed + 1)
    B = o.uniform((32,), seed + 2)
    run(ref, "nonternary_2x8", X, B, Wd, 2, 8,
        dict(name="nonternary_2x8", M=6, K=38, N=32, r=2, c=8, density=None, seed=seed, kind="float",
             flags=flags, source=src + "; non-ternary W values"))

    # NaN / inf values stored in W propagate through every later update
    seed = SEED0 + 650
    vals = np.array([1.0, -1.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, np.nan, np.inf, -np.inf],
                    dtype=np.float32)
    U = o.uniform((12, 24), seed)
    Wd = vals[(np.abs(U) * 1e6).astype(np.int64) % len(vals)]
    X = o.uniform((3, 12), seed + 1)
    B = o.uniform((24,), seed + 2)
    run(ref, "nonfinite_values_1x8", X, B, Wd, 1, 8,
        dict(name="nonfinite_values_1x8", M=3, K=12, N=24, r=1, c=8, density=None, seed=seed, kind="special",
             flags=flags, source=src + "; NaN/inf W values"))

    # special X / B values: inf * 0 inside a stored block is NaN; -0.0 bias
    seed = SEED0 + 700
    X = o.uniform((4, 16), seed)
    X[0, 3] = np.inf
    X[1, 5] = np.nan
    X[2, :] = -0.0
    B = o.uniform((16,), seed + 1)
    B[2] = -0.0
    Wd = o.ternary((16, 16), 0.3, seed + 2)
    run(ref, "specials_1x8", X, B, Wd, 1, 8,
        dict(name="specials_1x8", M=4, K=16, N=16, r=1, c=8, density=0.3, seed=seed, kind="special",
             flags=flags, source=src + "; X with inf/nan/-0.0"))


if __name__ == "__main__":
    main()
