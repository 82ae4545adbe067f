#!/bin/bash
# Round-4 A/B: k_fused with small units (1 k x 64 m, 12 producer waves: lib/diag fsmall, and fsm0
# with several stages per step) against the default big units (4 k x 256 m) and the two-kernel
# step, on cfg 4, the 8-way column block and cfg 2.  (Run when small units were the default build:
# "small" = the product library then, "big" = fbig.)
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py 2>&1 | tail -1 || exit 1
timeout -k 10 100 python -u tools/fused_debug.py probe 2>&1 | grep "wrong X" | head -6
TCSC_AMD_LIB=$D/libtcsc_amd_fsm0.so timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py 2>&1 | tail -1 || exit 1
for args in "--config 4" "--shard-of 8" "--config 2"; do
  for v in two small sm0 big; do
    f=1; unset TCSC_AMD_LIB
    case $v in two) f=0;; sm0|big) export TCSC_AMD_LIB=$D/libtcsc_amd_f$v.so;; esac
    TCSC_FUSED=$f timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args $v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
  done
done
