#!/bin/bash
# Gather-geometry sweep: GPU parity tests + cfg4 timing per variant
# (make -C sparse-matrix-multiplication-benchmark_amd geometry).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
P=$PWD/sparse-matrix-multiplication-benchmark_amd/lib
for g in main ${GEOS:-w8_cw32_b8_n2_tk64_nb2 w16_cw16_b4_n2_tk48_nb3 w16_cw16_b4_n2_tk64_nb2 w16_cw16_b8_n1_tk48_nb3 w8_cw32_b4_n2_tk48_nb3 w12_cw24_b4_n2_tk48_nb3}; do
  lib=$P/geo/libtcsc_amd_$g.so; [ $g = main ] && lib=$P/libtcsc_amd.so
  TCSC_AMD_LIB=$lib timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t_$g.log 2>&1
  rc=$?; echo "$g tests rc=$rc $(tail -1 gpurun_out/t_$g.log)"; [ $rc -ge 2 ] && exit $rc
  TCSC_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/b_$g.json 2> gpurun_out/b_$g.err
  rc=$?; [ $rc -ne 0 ] && { echo "$g bench rc=$rc"; tail -3 gpurun_out/b_$g.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/b_$g.json')); print('$g', round(d['roofline']['kernel_ms'],3), 'ms', round(d['value']), 'Gop/s')"
done
