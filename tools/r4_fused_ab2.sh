#!/bin/bash
# Round-4 A/B: placement / priority of the fused kernel's producer steps (cfg 4 and the 8-way block).
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
for args in "--config 4" "--shard-of 8"; do
  for v in product late prio lp; do
    if [ $v = product ]; then unset TCSC_AMD_LIB; else export TCSC_AMD_LIB=$D/libtcsc_amd_f$v.so; fi
    TCSC_FUSED=1 timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args $v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
  done
done
