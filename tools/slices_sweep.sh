cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for cfg in 2 4; do
for s in 0 1 2 3 4 6 8; do
  if [ $s = 0 ]; then unset TCSC_SLICES; else export TCSC_SLICES=$s; fi
  timeout -k 10 120 $B --config $cfg --no-dense --no-validate --warmup 5 --reps 30 --csv gpurun_out/ss.csv > /dev/null 2>&1 || exit 3
  python3 -c "import csv;r=[x for x in csv.DictReader(open('gpurun_out/ss.csv'))];print('cfg$cfg slices=$s', ' '.join(x['algorithm'][:6]+'='+x['ms_median'][:6] for x in r))"
done; done
