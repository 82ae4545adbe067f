#!/bin/bash
# Round 6: the 128 x 128 tiles' split target at K = N = 16384, MFMA plans only.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for w in 512 1024; do
    TCSC_MFMA_WGS=$w timeout -k 10 300 python -u tools/crossover.py --shapes 128x16384x16384,256x16384x16384,512x16384x16384,128x4096x16384,256x16384x4096 \
        --densities 0.1 --modes mfma --reps 10 > gpurun_out/xs16_$w.jsonl 2> gpurun_out/xs16_$w.err || { tail -20 gpurun_out/xs16_$w.err; exit 1; }
    echo "wgs=$w done"
done
