#!/bin/bash
# Round-4 generic A/B: the default build against lib/diag/libtcsc_amd_<v>.so for each v given
# (staged copies of tools/ab.mk builds), cfg 4, cfg 2 and the 8-way block, alternating twice.
# The parity tests run on the first variant first.  Usage: bash tools/r4_ab_libs.sh b6 [...]
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
TCSC_AMD_LIB=$D/libtcsc_amd_$1.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "not full_size" 2>&1 | tail -1 || exit 1
for r in 1 2; do
for args in "--config 4" "--config 2" "--shard-of 8"; do
  for v in base "$@"; do
    unset TCSC_AMD_LIB
    [ $v != base ] && export TCSC_AMD_LIB=$D/libtcsc_amd_$v.so
    timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args $v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
  done
done
done
