#!/bin/bash
# A/B timing of library builds in one session, alternating (ROUNDS, default 2):
#   ab.sh name=lib[@VAR=v,VAR2=w] ...   [PARITY=lib: the GPU suite on that build first]
# Prints k_stream (kernel_ms), the whole step and the other configs' steps.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
set -o pipefail
if [ -n "$PARITY" ]; then
  TCSC_AMD_LIB=$PWD/$PARITY timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/ab_pytest.log 2>&1 || { echo "parity FAILED"; tail -30 gpurun_out/ab_pytest.log; exit 1; }
  tail -1 gpurun_out/ab_pytest.log
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in "$@"; do
    n=${spec%%=*}; lib=${spec#*=}; envs=""
    case "$lib" in *@*) envs=${lib#*@}; lib=${lib%%@*};; esac
    env ${envs//,/ } TCSC_ALLOW_DIAG=1 TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-dense-baseline \
        --no-bcsr --no-host-api --no-graph ${BENCH_ARGS:-} > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err \
        || { echo "$n failed"; tail -5 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); r=d['roofline']; print('round $r $n', r['kernel'].split(' ')[0], round(r['kernel_ms'],4), 'step', round(d['ms_per_step'],4), 'T', round(next(iter(r.get('step_parts_ms',{0:0}).values())),4), {k: round(v['ms'],4) for k, v in d.get('other_configs',{}).items()}, 'ref', {k: round(v['ms'],3) for k, v in d.get('reference_order',{}).items() if isinstance(v, dict)})"
  done
done
