#!/bin/bash
# Time breakdown of the gather kernel: full, each ablation, with and without DMA.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
run() { # name lib
  TCSC_AMD_LIB=$2 timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/$1.json 2> gpurun_out/$1.err || { echo "$1 failed"; tail -3 gpurun_out/$1.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$1.json')); print('$1', round(d['roofline']['kernel_ms'],3), 'ms')"
}
run main $P/libtcsc_amd.so
for a in 1 3 4 5 6; do run abl$a $P/abl/libtcsc_amd_abl$a.so; done
for a in 0 1 3 4 5; do run abl${a}_nd $P/abl/libtcsc_amd_abl${a}_nd.so; done
for g in ${GEOS:-w16_cw16_b4_c16_tk48_nb3 w16_cw16_b4_c32_tk48_nb3 w12_cw24_b4_c32_tk48_nb3 w16_cw16_b4_c24_tk64_nb2}; do
  TCSC_AMD_LIB=$P/geo/libtcsc_amd_$g.so timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t_$g.log 2>&1
  rc=$?; echo "$g tests rc=$rc $(tail -1 gpurun_out/t_$g.log)"; [ $rc -ge 2 ] && exit $rc
  run $g $P/geo/libtcsc_amd_$g.so
done
