#!/bin/bash
# Round-4 A/B of the fused path on the GPU box (cfg 4): the fused tests, then
# bench.py's kernel time for the product build and the diagnostic builds in
# lib/diag (frr: round-robin item order; fpu: k_transpose + fused gather
# without production), then the stamps build.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
D=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused.py 2>&1 | tail -2 || exit 1
for v in product frr fpu; do
  if [ $v = product ]; then unset TCSC_AMD_LIB; else export TCSC_AMD_LIB=$D/libtcsc_amd_$v.so; fi
  TCSC_FUSED=1 timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $Q > gpurun_out/b_$v.json 2>gpurun_out/b_$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/b_$v.json'));r=d['roofline'];print('$v',round(d['ms_per_step'],4),round(r.get('kernel_ms'),4),r.get('path'))"
done
unset TCSC_AMD_LIB
TCSC_AMD_LIB=$D/libtcsc_amd_fst.so timeout -k 10 150 python -u tools/fused_stamps.py > gpurun_out/st.log 2>&1 || exit 1
tail -12 gpurun_out/st.log
