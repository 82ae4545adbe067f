cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/reduce_tests.log 2>&1; rc=$?
tail -3 gpurun_out/reduce_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench --config 2 --config 3 --no-dense --no-validate --warmup 10 --reps 50 --csv gpurun_out/red.csv > /dev/null 2>&1 || exit 3
cut -d, -f1,8,9 gpurun_out/red.csv
