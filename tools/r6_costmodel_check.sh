#!/bin/bash
# Round 6: the full GPU suite on the refit cost model, then the crossover
# sweeps again (big and small shapes) to check the default plan's choices.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/suite.log 2>&1 || { tail -40 gpurun_out/suite.log; exit 1; }
tail -3 gpurun_out/suite.log
SH="64x8192x8192,128x8192x8192,256x8192x8192,256x4096x4096,512x8192x8192,1024x8192x8192,2048x8192x8192,4096x4096x4096"
timeout -k 10 600 python -u tools/crossover.py --shapes $SH --densities 0.02,0.04,0.06,0.08,0.1,0.12,0.15,0.2,0.3,0.5 \
    > gpurun_out/xcheck_big.jsonl 2> gpurun_out/xcheck_big.err || { tail -20 gpurun_out/xcheck_big.err; exit 1; }
SH="128x256x256,64x512x512,128x1024x1024,256x1024x1024,256x2048x2048,512x2048x2048,1024x4096x4096,64x2048x8192,100x8192x2048,2048x2048x2048"
timeout -k 10 300 python -u tools/crossover.py --shapes $SH --densities 0.06,0.1,0.2,0.5 --reps 20 \
    > gpurun_out/xcheck_small.jsonl 2> gpurun_out/xcheck_small.err || { tail -20 gpurun_out/xcheck_small.err; exit 1; }
echo ALL_DONE
