#!/bin/bash
# Per-GPU view of the 8-way strong splits of cfg 4 on one MI355X (rank 0's
# block, bench.py --shard-of 8): the column split (the north star's layout)
# and the row split beside it.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
F="--steps 20 --warmup 5 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-host-api --no-graph --no-other-configs --no-reference-order"
for s in ${SHARDS:-8}; do
  for ax in cols rows; do
    timeout -k 10 300 python bench.py --shard-of $s --shard $ax $F > gpurun_out/shard${s}_$ax.json 2> gpurun_out/shard${s}_$ax.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/shard${s}_$ax.json')); r=d['roofline']; print('shard-of $s $ax: step', round(d['ms_per_step'],4), 'ms, gather', round(r['kernel_ms'],4), 'transpose', round(r['transpose_ms'],4))"
  done
done
