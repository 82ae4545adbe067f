#!/usr/bin/env python3
"""What the vendor bf16 GEMM (torch.matmul -> hipBLASLt) reaches at cfg 5's
split-GEMM shape: [M x 3K] bf16 times [3K x N] bf16 (M=2048, K=8192, N=8192),
bf16 and fp32 outputs, against k_gemm3's 824.6 GFLOP per step."""
import torch

M, K3, N = 2048, 3 * 8192, 8192
dev = torch.device("cuda:0")
A = torch.randn(M, K3, device=dev).to(torch.bfloat16)
B = torch.randn(K3, N, device=dev).to(torch.bfloat16)
Bt = B.t().contiguous().t()  # column-major view of the same values
flop = 2.0 * M * N * K3
for name, fn in (("bf16 out, B row-major", lambda: A @ B), ("bf16 out, B col-major", lambda: A @ Bt),
                 ("fp32 out (out_dtype)", lambda: torch.matmul(A, Bt, out_dtype=torch.float32))):
    try:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{name}: {ms:.3f} ms, {flop / ms / 1e9:.1f} TFLOP/s = {flop / ms / 1e9 / 2500:.3f} of 2.5 PF")
    except Exception as ex:  # noqa: BLE001
        print(f"{name}: {type(ex).__name__}: {ex}")
