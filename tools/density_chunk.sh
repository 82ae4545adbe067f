# k_stream cost per nonzero-row against the entries per wave and chunk
# (16 columns x 48 rows x density): M=1024 K=N=4096, split-K fixed at 4.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B=sparse-matrix-multiplication-benchmark_amd/bin/tcsc_bench
export TCSC_SLICES=4
for nz in 100 50 33 25 20 14 10; do
  rm -rf gpurun_out/dc
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dc -o t -- $B --shape 1024,4096,4096,$nz --no-dense --no-validate --warmup 10 --reps 30 --json gpurun_out/dc.json > /dev/null 2>&1 || exit 3
  python3 - $nz <<'PY'
import csv, glob, json, sys
nz = int(sys.argv[1])
f = glob.glob('gpurun_out/dc/**/*kernel_trace.csv', recursive=True)[0]
d = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in csv.DictReader(open(f)) if 'k_stream<false, true, 1, 0>' in r['Kernel_Name']]
d = d[-20:]
us = sum(d) / len(d) / 1e3
nnz = 4096 * 4096 / nz
ent = 1024 * nnz / 256 / 1024  # 256-row entries per SIMD
print(f"nz={nz} density={1/nz:.3f} entries/wave/chunk={16*48/nz:.1f} k_stream={us:.1f} us  cycles/entry/SIMD@2.4GHz={us*2400/ent:.1f}")
PY
done
