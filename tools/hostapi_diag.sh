#!/bin/bash
# The bench's host_api line against tools/host_pipe_sweep.py on one box, then
# the profiled bench run without the host API (profiles/r02_*).
cd "${GRAFT_REPO_ROOT:-.}"; mkdir -p gpurun_out; export TMPDIR=/tmp
B="python bench.py --steps 5 --warmup 2 --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-cpu-baseline --no-validate"
for i in 1 2; do
  timeout -k 10 300 $B > gpurun_out/hb.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/hb.json')); print('bench host_api', d['host_api']['ms'])"
done
TCSC_HOST_BANDS=1 timeout -k 10 300 $B > gpurun_out/hb.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/hb.json')); print('bench host_api unbanded', d['host_api']['ms'])"
timeout -k 10 200 python tools/host_pipe_sweep.py 8 || exit 1
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-host-api --no-graph > gpurun_out/rocprof.log 2>&1 || exit 1
echo rocprof ok
