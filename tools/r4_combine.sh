#!/bin/bash
# Round-4 A/B: the in-launch split-K combine (the default policy, k_stream OUT 2) against
# k_stream + k_reduce4 (TCSC_COMBINE=0): parity tests first, then cfg 2, cfg 3 and the
# 8-way block, alternating twice.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_combine.py 2>&1 | tail -3 || exit 1
for r in 1 2; do
for args in "--config 1" "--config 2" "--config 3" "--shard-of 8"; do
  for c in 0 auto; do
    unset TCSC_COMBINE; [ $c = 0 ] && export TCSC_COMBINE=0
    timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args combine=$c',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'),r.get('k_slices'),r.get('combine_in_launch'))"
  done
done
done
