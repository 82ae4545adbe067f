#!/bin/bash
# Time the gather kernel with each timing-only ablation build (make ablation).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=sparse-matrix-multiplication-benchmark_amd/lib
for a in 0 1 2 3 4 5; do
  lib=$P/libtcsc_amd.so; [ $a -ne 0 ] && lib=$P/abl/libtcsc_amd_abl$a.so
  TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/abl$a.json 2> gpurun_out/abl$a.err
  rc=$?; [ $rc -ne 0 ] && { echo "abl $a rc=$rc"; tail -3 gpurun_out/abl$a.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/abl$a.json')); print('abl $a', round(d['roofline']['kernel_ms'],3), 'ms')"
done
