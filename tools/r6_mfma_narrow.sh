#!/bin/bash
# Round 6: the MFMA GEMM's 64 x 256 tiles for M <= 64 and k_split3's batched
# loads.  The MFMA tests, then gather vs MFMA at small M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/narrow_pytest.log 2>&1 || { tail -30 gpurun_out/narrow_pytest.log; exit 1; }
tail -2 gpurun_out/narrow_pytest.log
SH="8x8192x8192,16x8192x8192,32x8192x8192,64x8192x8192,128x8192x8192,16x4096x4096,32x2048x2048,64x4096x4096,256x4096x4096"
timeout -k 10 600 python -u tools/crossover.py --shapes $SH --densities 0.06,0.1,0.3 --reps 20 \
    > gpurun_out/xnarrow.jsonl 2> gpurun_out/xnarrow.err || { tail -20 gpurun_out/xnarrow.err; exit 1; }
echo ALL_DONE
