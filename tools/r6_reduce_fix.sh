#!/bin/bash
# Round 6: k_fixup folded into the MFMA split's reduce.  MFMA + graph tests,
# then MFMA step times at small M.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_graph.py tests/test_gpu_fuzz.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/rf_pytest.log 2>&1 || { tail -40 gpurun_out/rf_pytest.log; exit 1; }
tail -2 gpurun_out/rf_pytest.log
timeout -k 10 300 python -u tools/crossover.py --shapes 8x8192x8192,64x8192x8192,128x8192x8192,256x8192x8192,256x4096x4096,1024x8192x8192 \
    --densities 0.1 --modes mfma --reps 20 > gpurun_out/xrf.jsonl 2> gpurun_out/xrf.err || { tail -20 gpurun_out/xrf.err; exit 1; }
echo ALL_DONE
