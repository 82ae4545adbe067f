#!/bin/bash
# Round 6: gather vs (split) MFMA on small shapes, for the cost model's fit.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SH="128x256x256,64x512x512,128x1024x1024,256x1024x1024,256x2048x2048,512x2048x2048,1024x4096x4096,64x2048x8192,100x8192x2048,2048x2048x2048"
timeout -k 10 600 python -u tools/crossover.py --shapes $SH --densities 0.06,0.1,0.2,0.5 --reps 20 \
    > gpurun_out/xsmall.jsonl 2> gpurun_out/xsmall.err || { tail -20 gpurun_out/xsmall.err; exit 1; }
echo ALL_DONE
