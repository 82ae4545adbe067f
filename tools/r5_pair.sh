#!/bin/bash
# Round-5 A/B: the pairwise in-launch combine at 2 K slices (k_stream OUT 3, the
# default) against k_stream + k_reduce4 (TCSC_COMBINE=0), on cfg 4's 8-way column
# and row blocks, alternating twice; the combine tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-graph"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_combine.py tests/test_gpu_dense_order.py tests/test_bcsr_gpu.py 2>&1 | tail -3 || exit 1
for r in 1 2; do
for args in "--shard-of 8 --shard cols" "--shard-of 8 --shard rows"; do
  for c in 0 auto; do
    unset TCSC_COMBINE; [ $c = 0 ] && export TCSC_COMBINE=0
    timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || { tail gpurun_out/c.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args combine=$c step',round(d['ms_per_step'],4),'gather',round(r.get('kernel_ms'),4),r.get('kernel'),r.get('combine_in_launch'))"
  done
done
done
