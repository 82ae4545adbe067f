#!/bin/bash
# timing-only ablations of the current kernel (results wrong by design)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { TCSC_AMD_LIB=$2 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/$1.json 2> gpurun_out/$1.err || { echo "$1 failed"; tail -3 gpurun_out/$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$1.json')); print('$1', round(d['roofline']['kernel_ms'],4), 'ms')"; }
run main $P/libtcsc_amd.so
for a in 1 3 4 5 6; do run abl$a $P/abl/libtcsc_amd_abl$a.so; done
for a in 0 1 3 4 5; do run abl${a}_nd $P/abl/libtcsc_amd_abl${a}_nd.so; done
