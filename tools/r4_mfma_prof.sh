#!/bin/bash
# Round-4: kernel times of cfg 5's MFMA path, split + GEMM vs fused split (rocprofv3 kernel trace).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate --no-graph"
for f in 0 1; do
  TCSC_MFMA_FUSED=$f timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/mp$f -o mp -- python3 -u bench.py --steps 10 --warmup 3 --config 5 $Q > gpurun_out/mp$f.json 2>gpurun_out/mp$f.err || exit 1
done
