#!/bin/bash
# Round-4 A/B: k_transpose tile shape (64m x 128k vs 256m x 32k, TCSC_XT_WIDE=1): parity, then
# the transpose's own time (bench two_kernel_path.k_transpose_ms) on cfg 4, cfg 2 and the 8-way block.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
TCSC_XT_WIDE=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py 2>&1 | tail -2 || exit 1
for r in 1 2; do
for args in "--config 4" "--config 2" "--shard-of 8"; do
  for w in 0 1; do
    TCSC_XT_WIDE=$w timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/x.json 2>gpurun_out/x.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/x.json'));r=d['roofline'];t=r.get('two_kernel_path') or {};print('$args wide=$w',round(d['ms_per_step'],4),'T',round(t.get('k_transpose_ms') or 0,4))"
  done
done
done
