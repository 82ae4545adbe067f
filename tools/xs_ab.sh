#!/bin/bash
# X-staging A/B: GPU parity of the direct-staging build, then alternating
# bench runs (kernel_ms = k_stream alone, ms_per_step = the whole step).
# usage: xs_ab.sh <lib under test for parity> name=lib ...
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
set -o pipefail
TLIB=$1; shift
TCSC_AMD_LIB=$PWD/$TLIB timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/xs_pytest.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/xs_pytest.log; exit 1; }
tail -3 gpurun_out/xs_pytest.log
for r in 1 2; do
  for spec in "$@"; do
    n=${spec%%=*}; lib=${spec#*=}
    TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dense-baseline --no-bcsr --no-host-api --no-graph ${BENCH_ARGS:-} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "$n failed"; tail -5 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); r=d['roofline']; print('round $r $n k_stream', round(r['kernel_ms'],4), 'ms; step', round(d['ms_per_step'],4), 'ms;', {k: round(v['ms'],4) for k, v in d.get('other_configs',{}).items()}, 'ref', {k: round(v['ms'],3) for k, v in d.get('reference_order',{}).items() if isinstance(v, dict)})"
  done
done
