#!/bin/bash
# Round-3 closing GPU session: the full check (tools/gpu_check.sh: pytest -m gpu,
# smoke, bench, rocprofv3 kernel trace), the HBM traffic passes
# (tools/traffic.sh), one SQ counter pass (tools/sq_pass.sh), the native
# driver's host-API records (profiles/r03_*), then any A/B given as arguments
# (tools/ab.sh specs).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
PYTEST_ARGS="-x -q --timeout 120 --timeout-method thread" bash tools/gpu_check.sh || exit $?
bash tools/traffic.sh || exit $?
bash tools/sq_pass.sh || exit $?
timeout -k 10 300 ./sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench --config 4 --config 2 --api host --num-runs 1 --rep 5 --cycles-required 0 --csv gpurun_out/r03_host_api.csv > gpurun_out/r03_host_api_out.txt 2>&1 || exit 1
echo FINAL_DONE
[ $# -gt 0 ] && BENCH_ARGS='--no-reference-order' bash tools/ab.sh "$@"
exit 0
