#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a short bench run (kernel trace
# only, no sys/runtime trace): where k_stream's wave-cycles go (issuing,
# waiting on s_waitcnt / barrier, issue stalls) and how busy the LDS is.
cd "${GRAFT_REPO_ROOT:-.}"; export TMPDIR=/tmp; mkdir -p gpurun_out
D=${SQ_DIR:-gpurun_out/sq}
rm -rf $D
# SQ_PMC overrides the counter list (at most 8 SQ_ + 2 GRBM_ counters in one pass)
PMC=${SQ_PMC:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES}
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $D -o run -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-host-api --no-graph \
    --no-other-configs --no-reference-order ${BENCH_ARGS:-} > $D.log 2>&1
echo "sq pass rc=$?"
