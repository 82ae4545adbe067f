#!/bin/bash
# A/B timing + GPU parity of library variants: abt.sh name=lib ... (tests once, then 3 alternating timing rounds)
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
for spec in "$@"; do
  n=${spec%%=*}; lib=${spec#*=}
  TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/t_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -1 gpurun_out/t_$n.log)"; [ $rc -ge 2 ] && exit $rc
done
for r in 1 2 3; do
  for spec in "$@"; do
    n=${spec%%=*}; lib=${spec#*=}
    TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "$n failed"; tail -3 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); print('round $r $n', round(d['roofline']['kernel_ms'],4), 'ms')"
  done
done
