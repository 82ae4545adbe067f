#!/bin/bash
# Round-4 A/B: k_fused producer steps of one stage each (1a), three producer waves (3w), both (3w1a):
# the fused parity tests per build, then cfg 4 and the 8-way column block.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
for v in 1a 3w 3w1a; do
  TCSC_AMD_LIB=$D/libtcsc_amd_f$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py 2>&1 | tail -1 || exit 1
done
for args in "--config 4" "--shard-of 8"; do
  for v in product 1a 3w 3w1a; do
    if [ $v = product ]; then unset TCSC_AMD_LIB; else export TCSC_AMD_LIB=$D/libtcsc_amd_f$v.so; fi
    TCSC_FUSED=1 timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args $v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
  done
done
