"""BASELINE.json configurations and synthetic device-side inputs.

cfg index follows BASELINE.json "configs" (1-based):
  1: M=128  K=256   N=256   90 % sparse  (reference's own CPU case)
  2: M=1024 K=4096  N=4096  95 %         plain tcsc_gemm
  3: M=1024 K=4096  N=4096  95 %         tcsc_gemm_prelu (fused epilogue)
  4: M=4096 K=16384 N=16384 98 %         headline; column shard over 8 GPUs
  5: M=2048 K=8192  N=8192  50 %         near-dense stress
Inputs: X, B ~ U[-1,1) fp32, W iid ternary with P(+1)=P(-1)=(1-s)/2
(dense/utils.h:9-16,36-68), a = 0.2 (main.cpp:268).  Seed 0x7C5C0000+cfg.
"""
from __future__ import annotations

from dataclasses import dataclass

SEED0 = 0x7C5C0000


@dataclass(frozen=True)
class Config:
    idx: int
    M: int
    K: int
    N: int
    sparsity: float
    variant: str

    @property
    def density(self) -> float:
        return 1.0 - self.sparsity

    @property
    def seed(self) -> int:
        return SEED0 + self.idx

    @property
    def name(self) -> str:
        return f"cfg{self.idx}"

    def describe(self) -> str:
        return (f"M={self.M} K={self.K} N={self.N}, {round(self.sparsity * 100)}% ternary sparsity, fp32, "
                f"{'tcsc_gemm_prelu' if 'prelu' in self.variant else 'tcsc_gemm'}")


CONFIGS = {
    1: Config(1, 128, 256, 256, 0.90, "basic"),
    2: Config(2, 1024, 4096, 4096, 0.95, "basic"),
    3: Config(3, 1024, 4096, 4096, 0.95, "prelu_basic"),
    4: Config(4, 4096, 16384, 16384, 0.98, "prelu_basic"),
    5: Config(5, 2048, 8192, 8192, 0.50, "basic"),
}


def add_ops(M: int, nnz: int, n_cols: int) -> int:
    """Work unit: one add/sub per nonzero per row + the bias add."""
    return M * nnz + M * n_cols


def algorithmic_bytes(M: int, K: int, n_cols: int, nnz: int) -> int:
    """Compulsory HBM bytes of one launch: X read once, Y
    written once, the TCSC index arrays (row indices + 2 x (cols+1) column
    starts) and B read once -- all 4-byte words."""
    return 4 * (M * K + M * n_cols + nnz + 2 * (n_cols + 1) + n_cols)


def make_device_inputs(cfg: Config, col_begin: int, col_end: int, device, seed_offset: int = 0,
                       x_seed: int | None = None):
    """Synthetic inputs for columns [col_begin, col_end) of cfg, generated on
    the GPU with torch (X is the full M x K matrix, identical on every rank):
    returns dict(X, B, Wd_cols) with Wd_cols the dense K x (c1-c0) ternary
    slice.  Column blocks are generated independently per block seed so a
    rank never materialises the full K x N matrix."""
    import torch

    g = torch.Generator(device=device)
    g.manual_seed(cfg.seed if x_seed is None else x_seed)
    X = torch.rand((cfg.M, cfg.K), generator=g, device=device, dtype=torch.float32) * 2 - 1
    nc = col_end - col_begin
    g.manual_seed(cfg.seed + 1 + seed_offset)
    B = torch.rand((cfg.N,), generator=g, device=device, dtype=torch.float32)[col_begin:col_end] * 2 - 1
    g.manual_seed(cfg.seed + 1000 * (seed_offset + 1) + col_begin)
    u = torch.rand((cfg.K, nc), generator=g, device=device, dtype=torch.float32)
    d = cfg.density
    Wd = torch.zeros((cfg.K, nc), device=device, dtype=torch.float32)
    Wd[u < d / 2] = 1.0
    Wd[(u >= d / 2) & (u < d)] = -1.0
    del u
    return {"X": X.contiguous(), "B": B.contiguous(), "Wd": Wd}
