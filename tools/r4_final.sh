#!/bin/bash
# Round-4 closing GPU session: the full check (tools/gpu_check.sh: pytest -m gpu,
# smoke, bench, rocprofv3 kernel trace), the HBM traffic passes (tools/traffic.sh,
# with the no-DMA ablation build staged in lib/diag), the 8-way column block's line.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYTEST_ARGS="-q --timeout 650 --timeout-method thread" bash tools/gpu_check.sh || exit $?
ABL_LIB=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag/libtcsc_amd_abl0_nd.so bash tools/traffic.sh || exit $?
timeout -k 10 200 python bench.py --shard-of 8 --no-host-api --no-other-configs --no-bcsr --no-reference-order > gpurun_out/shard8.json 2> gpurun_out/shard8.err || exit 1
echo FINAL_DONE
