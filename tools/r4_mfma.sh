#!/bin/bash
# Round-4: the MFMA path's fused split (k_gemm3x) -- tests, then cfg 5 step and kernel times both ways.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
TCSC_MFMA_FUSED=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py 2>&1 | tail -4 || exit 1
for f in 0 1; do
  TCSC_MFMA_FUSED=$f timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --config 5 $Q > gpurun_out/m.json 2>gpurun_out/m.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/m.json'));r=d['roofline'];print('cfg5 mfma_fused=$f',round(d['ms_per_step'],4),r.get('kernel'),round(r.get('kernel_ms') or 0,4),r.get('frac'))"
done
