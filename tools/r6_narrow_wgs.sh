#!/bin/bash
# Round 6: the split target for the 64 x 256 tiles (M <= 64), MFMA plans only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 256 384 512 1024; do
    TCSC_MFMA_WGS=$w timeout -k 10 200 python -u tools/crossover.py --shapes 8x8192x8192,32x8192x8192,64x8192x8192,64x4096x4096,16x16384x16384 \
        --densities 0.1 --modes mfma --reps 20 > gpurun_out/xnw_$w.jsonl 2> gpurun_out/xnw_$w.err || { tail -20 gpurun_out/xnw_$w.err; exit 1; }
    echo "wgs=$w done"
done
