#!/bin/bash
# Round-2 GPU session: GPU tests, then one SQ issue/stall PMC pass on the bench.
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dense-baseline --no-bcsr"
i=0
for set in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1)); rm -rf gpurun_out/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc$i -o run -- $B > gpurun_out/pmc$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
exit 0
