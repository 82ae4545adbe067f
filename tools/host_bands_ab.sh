# The host API's banded copy/compute pipeline against one unbanded launch:
# tcsc_bench --api host (reference timing protocol) at cfg 4 and cfg 2.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for cfg in 4 2; do
for bands in 1 0 1 0; do
  if [ $bands = 0 ]; then unset TCSC_HOST_BANDS; else export TCSC_HOST_BANDS=$bands; fi
  timeout -k 10 300 $B --config $cfg --api host --no-dense --no-validate --csv gpurun_out/hb.csv > /dev/null 2>&1 || exit 3
  python3 -c "import csv;r=[x for x in csv.DictReader(open('gpurun_out/hb.csv'))];print('cfg$cfg bands=${bands:-auto}', ' '.join(x['algorithm'][:8]+'='+x['ms_median'][:6] for x in r))"
done; done
