#!/bin/bash
# main vs DMA-only (abl5) vs gather-only (abl6) vs skeleton (abl5_nd).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { # name lib args...
  local n=$1 lib=$2; shift 2
  TCSC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -3 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', round(d['roofline']['kernel_ms'],3), 'ms')"
}
run main $P/libtcsc_amd.so ${BENCH_ARGS:-}
run abl5 $P/abl/libtcsc_amd_abl5.so ${BENCH_ARGS:-}
run abl6 $P/abl/libtcsc_amd_abl6.so ${BENCH_ARGS:-}
run abl4_nd $P/abl/libtcsc_amd_abl4_nd.so ${BENCH_ARGS:-}
run abl5_nd $P/abl/libtcsc_amd_abl5_nd.so ${BENCH_ARGS:-}
