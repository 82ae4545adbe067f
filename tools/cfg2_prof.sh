cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
export TMPDIR=/tmp
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2prof -o c2 -- $B --config 2 --no-dense --no-validate --warmup 10 --reps 30 > gpurun_out/c2prof.log 2>&1 || exit 3
python3 tools/prof_summary.py "$(find gpurun_out/c2prof -name "*kernel_trace.csv" | head -1)" 20 > gpurun_out/c2sum.txt 2>&1 || true
timeout -k 10 200 bash tools/slices_sweep.sh > gpurun_out/ss.txt 2>&1
