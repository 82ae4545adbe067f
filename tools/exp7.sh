#!/bin/bash
# Gather-loop A/B: GPU parity of the libraries named in TEST (default: the
# first one), then alternating timing rounds of all libraries given
# (name=lib ...), k_stream at cfg4.  BENCH_ARGS defaults to skipping the
# dense and BCSR side lines.
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out
BA=${BENCH_ARGS:---no-dense-baseline --no-bcsr}
first=${1%%=*}
for spec in "$@"; do
  n=${spec%%=*}; lib=${spec#*=}
  case " ${TEST:-$first} " in *" $n "*) ;; *) continue;; esac
  TCSC_AMD_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_$n.log 2>&1
  rc=$?; echo "$n tests rc=$rc $(tail -1 gpurun_out/t_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/t_$n.log; exit $rc; }
done
for r in 1 2 3; do
  for spec in "$@"; do
    n=${spec%%=*}; lib=${spec#*=}
    TCSC_AMD_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline $BA > gpurun_out/ab_$n.json 2> gpurun_out/ab_$n.err || { echo "$n failed"; tail -3 gpurun_out/ab_$n.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/ab_$n.json')); x=d['roofline']; print('round $r $n', round(x['kernel_ms'],4), 'ms  transpose', round(x['transpose_ms'],4))"
  done
done
