#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SH="64x8192x8192,128x8192x8192,256x8192x8192,256x4096x4096,512x8192x8192,100x4096x4096"
for w in 512 768 1024; do
    TCSC_MFMA_WGS=$w timeout -k 10 300 python -u tools/crossover.py --shapes $SH --densities 0.1 --modes mfma --reps 20 \
        > gpurun_out/xsplit2_w$w.jsonl 2> gpurun_out/xsplit2_w$w.err || { tail -20 gpurun_out/xsplit2_w$w.err; exit 1; }
    echo "wgs=$w done"
done
