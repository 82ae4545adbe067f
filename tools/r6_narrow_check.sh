#!/bin/bash
# Round 6: the full GPU suite with the MFMA path from M = 5 (64 x 256 tiles),
# then gather vs MFMA vs the default plan at small M and on small shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
tail -2 gpurun_out/suite.log
SH="5x8192x8192,8x8192x8192,16x8192x8192,32x8192x8192,64x8192x8192,128x8192x8192,16x4096x4096,32x2048x2048,64x4096x4096,8x1024x1024,48x512x512"
timeout -k 10 600 python -u tools/crossover.py --shapes $SH --densities 0.06,0.1,0.3 --reps 20 \
    > gpurun_out/xnarrow2.jsonl 2> gpurun_out/xnarrow2.err || { tail -20 gpurun_out/xnarrow2.err; exit 1; }
SH="128x256x256,64x512x512,128x1024x1024,256x1024x1024,256x2048x2048,512x2048x2048,1024x4096x4096,64x2048x8192,100x8192x2048,2048x2048x2048"
timeout -k 10 300 python -u tools/crossover.py --shapes $SH --densities 0.06,0.1,0.2,0.5 --reps 20 \
    > gpurun_out/xcheck_small2.jsonl 2> gpurun_out/xcheck_small2.err || { tail -20 gpurun_out/xcheck_small2.err; exit 1; }
echo ALL_DONE
