#!/bin/bash
# Round-5 GPU session, part 2: the north star's per-rank block (cfg 4, 8-way
# column split) and the 2/4-way views, the stamps build's breakdown of
# k_stream (cfg 4, its 8-way block, cfg 2), and a rocprofv3 kernel trace of
# the 8-way block's bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
F="--steps 20 --warmup 5 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-host-api --no-graph --no-other-configs --no-reference-order"
for s in ${SHARDS:-2 4 8}; do
  for ax in cols rows; do
    timeout -k 10 300 python bench.py --shard-of $s --shard $ax $F > $OUT/shard${s}_$ax.json 2> $OUT/shard${s}_$ax.err || { echo "shard $s $ax failed"; tail $OUT/shard${s}_$ax.err; exit 1; }
    python -c "import json; d=json.load(open('$OUT/shard${s}_$ax.json')); r=d['roofline']; print('shard-of $s $ax: step', round(d['ms_per_step'],4), 'ms, gather', round(r['kernel_ms'],4), 'transpose', round(r['step_parts_ms']['k_transpose'],4), 'step_frac', round(r['step_frac'],4))"
  done
done
if [ "${STAMPS:-1}" = 1 ]; then
  L=sparse-matrix-multiplication-benchmark_amd/lib/diag/libtcsc_amd_stamps.so
  timeout -k 10 200 python tools/stamps.py --cfg 4 --shard-of 8 --lib $L > $OUT/stamps_8way.txt 2>&1 || { cat $OUT/stamps_8way.txt; exit 1; }
  timeout -k 10 200 python tools/stamps.py --cfg 2 --lib $L > $OUT/stamps_cfg2.txt 2>&1 || { cat $OUT/stamps_cfg2.txt; exit 1; }
  timeout -k 10 300 python tools/stamps.py --cfg 4 --lib $L > $OUT/stamps_cfg4.txt 2>&1 || { cat $OUT/stamps_cfg4.txt; exit 1; }
  tail -n 8 $OUT/stamps_*.txt
fi
if [ "${PROF:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof8 -o run -- python bench.py --shard-of 8 --shard cols --steps 10 --warmup 2 $F > $OUT/prof8.log 2>&1 || { tail $OUT/prof8.log; exit 1; }
  python tools/prof_summary.py $OUT/prof8/run_kernel_trace.csv 10 > $OUT/prof8_summary.json 2>&1; head -c 1500 $OUT/prof8_summary.json
fi
if [ "${PMC:-1}" = 1 ]; then
  # HBM traffic (FETCH_SIZE, WRITE_SIZE, TCC hit/miss, FETCH_SIZE of the no-DMA build) and
  # one SQ pass, each its own rocprofv3 run, of the 8-way block's k_stream (2 K slices: the
  # slab-writing instantiation OUT 1) -> TRAFFIC_KEY cfg4:prelu_basic:2048 (tools/traffic_json.py)
  BENCH_ARGS="--shard-of 8 --no-other-configs --no-reference-order --no-bcsr --no-dense-baseline" \
    TRAFFIC_DIR=gpurun_out/tr8_ ABL_LIB=$PWD/sparse-matrix-multiplication-benchmark_amd/lib/diag/libtcsc_amd_abl0_nd.so \
    bash tools/traffic.sh || exit 1
  BENCH_ARGS="--shard-of 8" SQ_DIR=gpurun_out/sq8 bash tools/sq_pass.sh || exit 1
fi
echo ALL_DONE
