#!/bin/bash
# Ablation + ring-geometry timing of the gather kernel (kernel_ms includes the
# X transpose).  make -C sparse-matrix-multiplication-benchmark_amd all ablation geometry
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { # name lib args...
  local n=$1 lib=$2; shift 2
  TCSC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -3 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', round(d['roofline']['kernel_ms'],3), 'ms', d['config']['workload'][-40:])"
}
run main $P/libtcsc_amd.so
for a in 1 2 3 4 5 6; do run abl$a $P/abl/libtcsc_amd_abl$a.so; done
for g in tk32_nb3 tk40_nb3 tk24_nb3; do run $g $P/geo/libtcsc_amd_$g.so; done
