#!/bin/bash
# Round-4 A/B: k_fused (big units) with and without the stream-prefetch skip ahead of signal steps
# (lib/diag fskip), against the two-kernel step, cfg 4 and the 8-way block, alternating twice.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py 2>&1 | tail -1 || exit 1
for r in 1 2; do
for args in "--config 4" "--shard-of 8"; do
  for v in two fused skip; do
    f=1; unset TCSC_AMD_LIB
    case $v in two) f=0;; skip) export TCSC_AMD_LIB=$D/libtcsc_amd_fskip.so;; esac
    TCSC_FUSED=$f timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args $v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
  done
done
done
