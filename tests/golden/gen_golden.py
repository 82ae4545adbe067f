#!/usr/bin/env python3
"""Generate tests/golden/*.npz from the REFERENCE ITSELF.

Runs only in the build container (it needs oracle/_ref/libtcsc_ref.so, which
is compiled from /root/reference/sparse/tcsc.c + dense/dense.c by
oracle/Makefile).  The reference pins nothing itself (unseeded RNG, no unit
tests: SURVEY.md §4), so these fixtures are the pin: inputs from the seeded
SplitMix64 generators of oracle/tcsc_oracle.c, outputs from the reference's
functions compiled with IEEE flags (-O2 -fno-fast-math -ffp-contract=off).

Each fixture holds
  X, B, a                        inputs (X float32 M x K, B float32 N)
  Wd (int8 or float32)           dense K x N W handed to tcsc_from_dense
  csp, csn, rip, rin             reference tcsc_from_dense output (tcsc.c:6-66)
  Y_<variant>                    reference tcsc_sgemm_* output, 5 variants
  Y_gemm                         reference gemm_basic (dense.c:64-77)
  Y_sparsegemm[_prelu]           reference sparseGEMM[_PReLU] (SparseGEMM.h:104,151)
  Y_gemm_prelu                   reference GEMM_PReLU (SparseGEMM.h:135-149)
  meta                           JSON: shape, density, seed, flags, kind

Usage: python tests/golden/gen_golden.py   (writes next to this file)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402

SEED0 = 0x7C5C0000
A = 0.2  # main.cpp:268

# name, M, K, N, density, seed, kind
CASES = [
    # build_and_run_m1.sh:137-186 quick test (M=2, K=4, N=4, nz=2)
    ("smoke_2x4x4", 2, 4, 4, 0.5, SEED0 + 100, "float"),
    # BASELINE.json configs[0]: M=128 K=N=256 at 90 % sparsity
    ("cfg1", 128, 256, 256, 0.10, SEED0 + 1, "float"),
    ("cfg1_int", 128, 256, 256, 0.10, SEED0 + 11, "int"),
    # SparseGEMM.cpp:73-80 grid subset (M, K, N, nonZero -> density 1/nz)
    ("grid_m1_k256_n512_nz2", 1, 256, 512, 0.5, SEED0 + 201, "float"),
    ("grid_m16_k512_n1024_nz8", 16, 512, 1024, 0.125, SEED0 + 202, "float"),
    ("grid_m64_k256_n512_nz16", 64, 256, 512, 1.0 / 16, SEED0 + 203, "int"),
    # main.cpp:258-264 first case shape (M=1, K=512, N=2048, nz=2)
    ("main_case1", 1, 512, 2048, 0.5, SEED0 + 301, "float"),
    # edge cases
    ("edge_allzero_w", 3, 64, 70, 0.0, SEED0 + 401, "float"),
    ("edge_ragged_n65", 5, 96, 65, 0.05, SEED0 + 402, "float"),
    ("edge_m1", 1, 300, 130, 0.03, SEED0 + 403, "int"),
    ("edge_k1", 7, 1, 5, 0.9, SEED0 + 404, "float"),
    ("edge_k_not_mult4", 9, 131, 67, 0.2, SEED0 + 405, "float"),
    ("edge_dense_w", 4, 50, 40, 1.0, SEED0 + 406, "int"),
    ("edge_long_k", 3, 2100, 33, 0.3, SEED0 + 407, "float"),
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


def run_reference(ref, X, Wd, B, a):
    out = {}
    W = ref.tcsc_from_dense(Wd)
    out["csp"], out["csn"] = W.col_start_pos, W.col_start_neg
    out["rip"], out["rin"] = W.row_index_pos, W.row_index_neg
    for v in pyoracle.VARIANTS:
        out["Y_" + v] = ref.sgemm(v, X, W, B, a)
    out["Y_gemm"] = ref.gemm_basic(X, Wd, B)
    out["Y_gemm_prelu"] = ref.gemm_prelu(X, Wd, B, a)
    out["Y_sparsegemm"] = ref.sparse_gemm(X, W, B, False, a)
    out["Y_sparsegemm_prelu"] = ref.sparse_gemm(X, W, B, True, a)
    return out


def save(name, arrays, meta):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, meta=np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8), **arrays)
    return path


def main():
    ref = pyoracle.load_reference()
    if ref is None:
        sys.exit("oracle/_ref/libtcsc_ref.so missing: run `make -C oracle ref` (needs /root/reference)")
    o = pyoracle.load_oracle()
    flags = "g++ -O2 -fno-fast-math -ffp-contract=off (oracle/Makefile)"
    for name, M, K, N, d, seed, kind in CASES:
        X, B, Wd = make_inputs(o, M, K, N, d, seed, kind)
        out = run_reference(ref, X, Wd, B, A)
        arrays = dict(X=X, B=B, a=np.float32(A), Wd=Wd.astype(np.int8), **out)
        meta = dict(name=name, M=M, K=K, N=N, density=d, seed=seed, kind=kind, flags=flags,
                    source="reference sparse/tcsc.c + dense/dense.c + SparseGEMM.h via oracle/_ref")
        print(save(name, arrays, meta), "nnz", int(out["csp"][-1] + out["csn"][-1]))

    # tcsc_from_dense on non-ternary input: only == +1.0f / == -1.0f count
    # (tcsc.c:14-17,54-58); 0.999, 2, -0.0, NaN, inf are all "zero".
    rng_vals = np.array([1.0, -1.0, 0.0, -0.0, 0.5, 2.0, -1.0000001, 0.99999994, np.nan, np.inf, -np.inf, -2.0],
                        dtype=np.float32)
    Wd = o.uniform((37, 29), SEED0 + 500)
    idx = (np.abs(Wd) * 1e6).astype(np.int64) % len(rng_vals)
    Wd = rng_vals[idx]
    X = o.uniform((6, 37), SEED0 + 501)
    B = o.uniform((29,), SEED0 + 502)
    out = run_reference(ref, X, Wd, B, A)
    arrays = dict(X=X, B=B, a=np.float32(A), Wd=Wd, **out)
    meta = dict(name="edge_nonternary", M=6, K=37, N=29, density=None, seed=SEED0 + 500, kind="float",
                flags=flags, source="reference tcsc_from_dense on non-ternary values")
    print(save("edge_nonternary", arrays, meta))

    # special X values: inf/nan/-0.0 (PReLU keeps NaN and -0.0: (v<0)?a*v:v)
    X = o.uniform((4, 16), SEED0 + 600)
    X[0, 3] = np.inf
    X[1, 5] = np.nan
    X[2, :] = -0.0
    B = o.uniform((8,), SEED0 + 601)
    B[2] = -0.0
    Wd = o.ternary((16, 8), 0.4, SEED0 + 602)
    Wd[:, 6] = 0.0  # an empty column: output is the bias alone
    out = run_reference(ref, X, Wd, B, A)
    arrays = dict(X=X, B=B, a=np.float32(A), Wd=Wd.astype(np.int8), **out)
    meta = dict(name="edge_specials", M=4, K=16, N=8, density=0.4, seed=SEED0 + 600, kind="special",
                flags=flags, source="reference, X with inf/nan/-0.0")
    print(save("edge_specials", arrays, meta))

    # SparseFormat (SparseGEMM.h:13-40) on an integer matrix vs tcsc_from_dense
    mat = (o.ternary((48, 40), 0.3, SEED0 + 700)).astype(np.int32)
    W = ref.sparseformat(mat)
    print(save("sparseformat_48x40", dict(mat=mat, csp=W.col_start_pos, csn=W.col_start_neg,
                                          rip=W.row_index_pos, rin=W.row_index_neg),
               dict(name="sparseformat_48x40", source="reference SparseFormat", flags=flags)))


if __name__ == "__main__":
    main()
