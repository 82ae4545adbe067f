cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for w in 5 20 80 300 5; do
  timeout -k 10 200 python bench.py --steps 20 --warmup $w --no-cpu-baseline --no-bcsr --no-reference-order --no-dense-baseline > gpurun_out/wexp_$w.json 2>gpurun_out/wexp.err || exit 3
  python -c "import json;d=json.load(open('gpurun_out/wexp_$w.json'));print($w, round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), round(d['roofline']['transpose_ms'],4))"
done
