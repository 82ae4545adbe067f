# MFMA path vs gather on small near-dense problems (the reference harness's M=256 cases) and cfg 5
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for p in auto gather auto gather; do
  E=""; [ $p = gather ] && E="TCSC_PATH=gather"
  env $E timeout -k 10 300 $B --shape 256,512,2048,2 --shape 256,1024,4096,2 --shape 64,2048,2048,2 --shape 512,4096,4096,2 --shape 1024,4096,4096,4 --no-dense --no-validate --warmup 5 --reps 30 --csv gpurun_out/ms.csv > /dev/null 2>&1 || exit 3
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('gpurun_out/ms.csv')) if x['algorithm']=='optimized']
print('$p', ' | '.join(f\"{x['M']}x{x['K']}x{x['N']}/{x['nnz']}: {float(x['ms_median'])*1e3:.1f}us\" for x in r))"
done
