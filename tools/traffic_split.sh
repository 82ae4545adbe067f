# Where k_stream's fetched bytes come from: FETCH_SIZE (raw KiB) of the full
# kernel against the no-DMA ablation (entry streams + bias only, no X^T).
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
A="--steps 3 --warmup 1 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-validate"
for lib in $P/libtcsc_amd.so $P/abl/libtcsc_amd_abl0_nd.so; do
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    rm -rf gpurun_out/ts
    TCSC_AMD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/ts -o run -- python bench.py $A > gpurun_out/ts.log 2>&1 || exit 3
    python3 - "$lib" "$set" <<'PY'
import collections, csv, glob, sys
vals = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob('gpurun_out/ts/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'k_stream<false, true, 0, 0>' in r['Kernel_Name']:
            vals[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
print(sys.argv[1].split('/')[-1], {k: round(sum(v.values()) / len(v), 1) for k, v in vals.items()})
PY
  done
done
