import sys, os, numpy as np
sys.path.insert(0, "sparse-matrix-multiplication-benchmark_amd")
mode = sys.argv[1]
import tcsc_amd
from tcsc_amd import bcsr
tcsc_amd.require_gpu()
if mode == "bcsr":
    W = bcsr.BcsrMatrix.from_dense(np.eye(16, dtype=np.float32), 1, 8)
    print(bcsr.sgemm("basic", np.ones((3, 16), np.float32), W, np.zeros(16, np.float32))[0, :4])
elif mode == "tcsc":
    W = tcsc_amd.TcscMatrix.from_dense(np.eye(16, dtype=np.float32))
    print(tcsc_amd.sgemm("basic", np.ones((3, 16), np.float32), W, np.zeros(16, np.float32))[0, :4])
import torch
print(mode, "torch available:", torch.cuda.is_available(), torch.cuda.device_count())
