#!/bin/bash
# Round-5 closing GPU session on the final tree: tools/gpu_check.sh (pytest -m gpu,
# smoke, bench, rocprofv3 kernel trace of the bench), the trace summary, cfg 4's HBM
# traffic passes (tools/traffic.sh with the no-DMA ablation build in lib/diag) and
# its SQ pass (tools/sq_pass.sh).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYTEST_ARGS="-x -q --timeout 120 --timeout-method thread" bash tools/gpu_check.sh || exit $?
python tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv 10 > gpurun_out/prof_summary.json || exit 1
ABL_LIB=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag/libtcsc_amd_abl0_nd.so bash tools/traffic.sh || exit $?
bash tools/sq_pass.sh || exit $?
echo FINAL_DONE
