#!/bin/bash
# HBM traffic of k_stream per launch (MI355X_MICROARCH.md "HBM"): FETCH_SIZE
# and WRITE_SIZE in separate --pmc passes (they cannot share one), kernel
# trace only, plus a FETCH_SIZE pass of the no-DMA ablation build (make -C
# sparse-matrix-multiplication-benchmark_amd lib/abl/libtcsc_amd_abl0_nd.so:
# the entry-stream scalar loads without the X^T staging), so that
# tools/traffic_json.py applies the gfx950 x2 FETCH_SIZE correction to the
# 16-B/lane X^T reads only; it writes profiles/traffic.json for bench.py.
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-host-api --no-graph ${BENCH_ARGS:-}"
T=${TRAFFIC_DIR:-gpurun_out/traffic}
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf $T$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $T$i -o run -- $B > $T$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
ABL=${ABL_LIB:-$PWD/sparse-matrix-multiplication-benchmark_amd/lib/abl/libtcsc_amd_abl0_nd.so}
rm -rf ${T}4
TCSC_ALLOW_DIAG=1 TCSC_AMD_LIB=$ABL timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d ${T}4 -o run -- $B --no-validate > ${T}4.log 2>&1
rc=$?; echo "pass 4 (FETCH_SIZE, no-DMA ablation) rc=$rc"; [ $rc -ne 0 ] && exit $rc
# profiles/traffic.json: run `python tools/traffic_json.py` after gpurun merged gpurun_out/ back
exit 0
