cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for g in hipblaslt rocblas hipblaslt rocblas; do
  TCSC_MFMA_GEMM=$g timeout -k 10 120 $B --config 5 --no-dense --no-validate --warmup 10 --reps 40 --csv gpurun_out/ab.csv > /dev/null 2>&1 || exit 3
  python3 -c "import csv;r=[x for x in csv.DictReader(open('gpurun_out/ab.csv'))];print('$g', ' '.join(x['algorithm'][:8]+'='+x['ms_median'][:6] for x in r))"
done
