#!/bin/bash
# Round-6 closing GPU session on the final tree: tools/gpu_check.sh (pytest -m gpu,
# smoke, bench, rocprofv3 kernel trace of the bench), the trace summary and cfg 4's
# HBM traffic passes (tools/traffic.sh; the no-DMA ablation build staged in
# lib/traffic, which is not gpurun-ignored, unlike lib/abl and lib/diag).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYTEST_ARGS="-x -v --timeout 120 --timeout-method thread" bash tools/gpu_check.sh || exit $?
python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv 10 > gpurun_out/prof_summary.json || exit 1
ABL_LIB=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/traffic/libtcsc_amd_abl0_nd.so bash tools/traffic.sh || exit $?
echo FINAL_DONE
