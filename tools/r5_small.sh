#!/bin/bash
# Round-5: per-call times of the small-M path (TCSC_SMALL_M=16) against the
# gather (0) on tools/small_m.sh's shapes, prelu_basic, through the native driver.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for r in 1 2; do
for sm in 4 0; do
  TCSC_SMALL_M=$sm timeout -k 10 300 $B --shape 1,512,2048,2 --shape 1,1024,4096,2 --shape 1,2048,8192,2 --shape 1,16384,16384,50 --shape 4,16384,16384,50 --shape 2,4096,4096,20 --shape 4,4096,4096,20 --no-dense --no-validate --warmup 5 --reps 30 --csv gpurun_out/sm.csv > /dev/null 2>&1 || exit 3
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('gpurun_out/sm.csv')) if x['algorithm']=='prelu_basic']
print('small_m=$sm', ' | '.join(f\"{x['M']}x{x['K']}x{x['N']}: {float(x['ms_median'])*1e3:.1f}us\" for x in r))"
done
done
