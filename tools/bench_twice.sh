cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_full.json 2>gpurun_out/bench_full.err || exit 3
for v in "" "--no-validate" "" "--no-validate"; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-bcsr --no-reference-order --no-dense-baseline $v > gpurun_out/bq.json 2>>gpurun_out/bench_full.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/bq.json'));print('$v', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['transpose_ms'],4), d.get('validation'))"
done
