# Small-M path: GPU parity, then per-call times with the path on (TCSC_SMALL_M=16) and off (0)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/small_tests.log 2>&1; rc=$?
tail -3 gpurun_out/small_tests.log; [ $rc -ne 0 ] && exit $rc
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
for sm in 16 0; do
  TCSC_SMALL_M=$sm timeout -k 10 300 $B --shape 1,512,2048,2 --shape 1,2048,8192,2 --shape 1,16384,16384,50 --shape 4,16384,16384,50 --shape 16,16384,16384,50 --shape 16,4096,4096,20 --no-dense --no-validate --warmup 5 --reps 30 --csv gpurun_out/sm.csv > /dev/null 2>&1 || exit 3
  python3 -c "
import csv
r=[x for x in csv.DictReader(open('gpurun_out/sm.csv')) if x['algorithm']=='prelu_basic']
print('small_m=$sm', ' | '.join(f\"{x['M']}x{x['K']}x{x['N']}: {float(x['ms_median'])*1e3:.1f}us\" for x in r))"
done
