cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_mfma.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/mfma_tests.log 2>&1; rc=$?
tail -25 gpurun_out/mfma_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench --config 5 --config 2 --warmup 3 --reps 20 --csv gpurun_out/h_mfma.csv > gpurun_out/h_mfma.txt 2>&1; rc=$?
cat gpurun_out/h_mfma.csv; exit $rc
