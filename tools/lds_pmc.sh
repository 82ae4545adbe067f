#!/bin/bash
# LDS / issue counters of k_stream at cfg4 (one --pmc pass per line, kernel
# trace only).  Summarise with tools/pmc_summary.py after gpurun merged
# gpurun_out/ back.
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-}"
timeout -k 10 120 rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || exit 1
i=0
while read -r set; do
  i=$((i+1))
  rm -rf gpurun_out/lds$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/lds$i -o run -- $B > gpurun_out/lds$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -ne 0 ] && exit $rc
done <<'SETS'
SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM
SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_LDS
SETS
exit 0
