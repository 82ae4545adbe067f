#!/bin/bash
# Gather cost alone: ablations built without X staging (make ablation-nodma).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { # name lib args...
  local n=$1 lib=$2; shift 2
  TCSC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -3 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', round(d['roofline']['kernel_ms'],3), 'ms')"
}
for a in 0 1 2 3 4 5; do run abl${a}_nd $P/abl/libtcsc_amd_abl${a}_nd.so ${BENCH_ARGS:-}; done
