cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for rnd in 1 2; do
for s in 0 2 3 4 5 6; do
  if [ $s = 0 ]; then unset TCSC_SLICES; else export TCSC_SLICES=$s; fi
  timeout -k 10 120 $B --config 2 --no-dense --no-validate --warmup 10 --reps 50 --csv gpurun_out/ss.csv > /dev/null 2>&1 || exit 3
  python3 -c "import csv;r=[x for x in csv.DictReader(open('gpurun_out/ss.csv'))];print('round $rnd cfg2 slices=$s', ' '.join(x['algorithm'][:10]+'='+x['ms_median'][:6] for x in r))"
done; done
