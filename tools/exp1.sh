#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { # name lib args...
  local n=$1 lib=$2; shift 2
  TCSC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -3 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['workload'][-40:])"
}
run full_k16384 $P/libtcsc_amd.so
run abl5_k16384 $P/abl/libtcsc_amd_abl5.so
run abl5_k16448 $P/abl/libtcsc_amd_abl5.so --override K=16448
run full_k16448 $P/libtcsc_amd.so --override K=16448
run abl5_n4096 $P/abl/libtcsc_amd_abl5.so --override N=4096
