#!/bin/bash
# Round-5 A/B of the split-K combine forms at 2 slices (cfg 4's 8-way blocks) and
# 4 slices (cfg 2/3): k_reduce4 (TCSC_COMBINE=0), pairwise (default at 2), row
# bands (TCSC_COMBINE=2 at 2 slices; default at 4), alternating twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-graph --no-validate"
for r in 1 2; do
for args in "--shard-of 8 --shard cols" "--shard-of 8 --shard rows" "--config 2" "--config 3"; do
  for c in 0 auto 2; do
    unset TCSC_COMBINE; [ $c != auto ] && export TCSC_COMBINE=$c
    timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 $args $Q > gpurun_out/c.json 2>gpurun_out/c.err || { tail gpurun_out/c.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/c.json'));r=d['roofline'];print('$args combine=$c step',round(d['ms_per_step'],4),'gather',round(r.get('kernel_ms'),4),r.get('combine_in_launch'))"
  done
done
done
