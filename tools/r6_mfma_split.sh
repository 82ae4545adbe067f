#!/bin/bash
# Round 6: the MFMA GEMM's split-K for grids with fewer tiles than they can
# run at once.  GPU tests of the MFMA path (and the suites whose shapes it
# can take), then the crossover sweep with the default plan (auto) beside
# both forced paths.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SH="64x8192x8192,128x8192x8192,256x8192x8192,256x4096x4096,512x8192x8192,1024x8192x8192,2048x8192x8192,4096x4096x4096"
timeout -k 10 900 python -u -m pytest tests/test_gpu_mfma.py tests/test_gpu_graph.py tests/test_gpu_dense_order.py \
    tests/test_gpu_fuzz.py tests/test_host_exact.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/mfma_split_pytest.log 2>&1 || { tail -30 gpurun_out/mfma_split_pytest.log; exit 1; }
tail -3 gpurun_out/mfma_split_pytest.log
timeout -k 10 900 python -u tools/crossover.py --shapes $SH --densities 0.02,0.04,0.06,0.08,0.1,0.12,0.15,0.2,0.3,0.5 \
    > gpurun_out/xsplit_all.jsonl 2> gpurun_out/xsplit_all.err || { tail -20 gpurun_out/xsplit_all.err; exit 1; }
echo ALL_DONE
