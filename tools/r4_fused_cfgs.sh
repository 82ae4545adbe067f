#!/bin/bash
# Round-4: two-kernel vs fused step time on cfg 2, cfg 3, cfg 4 and cfg 4's 8-way column block.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
for args in "--config 2" "--config 3" "--shard-of 8" "--config 4"; do
  for f in 0 1; do
    TCSC_FUSED=$f timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args fused=$f',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'),r.get('k_slices'))"
  done
done
