#!/bin/bash
# Latency / issue counters of k_stream at cfg4: the counter list, then one
# --pmc pass per line (kernel trace only).  Summarise: tools/pmc_summary.py k_stream gpurun_out/p3
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out/p3
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dense-baseline --no-bcsr"
timeout -k 10 120 rocprofv3 -L > gpurun_out/p3/avail.txt 2>&1 || true
i=0
while read -r set; do
  [ -z "$set" ] && continue
  i=$((i+1)); rm -rf gpurun_out/p3/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/p3/pmc$i -o run -- $B > gpurun_out/p3/pmc$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/p3/pmc$i.log; exit $rc; }
done <<'SETS'
SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE
SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH
SETS
exit 0
