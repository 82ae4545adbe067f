#!/bin/bash
# Round-2 closing GPU session: the full check (tools/gpu_check.sh), then the
# native driver's host-API records and the reference's SparseGEMM.cpp harness
# built against include/SparseGEMM.h (profiles/r02_*).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
bash tools/gpu_check.sh || exit $?
timeout -k 10 300 ./sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench --config 4 --config 2 --api host --num-runs 1 --rep 5 --cycles-required 0 --csv gpurun_out/r02_host_api.csv > gpurun_out/r02_host_api_out.txt 2>&1 || exit 1
timeout -k 10 300 ./oracle/_ref/sparsegemm_amd > gpurun_out/r02_sparsegemm_harness_out.txt 2>&1 || exit 1
echo FINAL_DONE
