#!/bin/bash
# Round-4: split-K slice count sweep on the 8-way column block and cfg 2 (TCSC_SLICES forces it).
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
for args in "--shard-of 8" "--config 2"; do
  for z in 1 2 3 4 6; do
    TCSC_SLICES=$z timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/z.json 2>gpurun_out/z.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/z.json'));r=d['roofline'];print('$args Z=$z',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('k_slices'))"
  done
done
