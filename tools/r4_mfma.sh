#!/bin/bash
# Round-4: the MFMA path (k-major X3/W3T block layout): its tests, cfg 5's step, and the
# reference harness (main.cpp, the reference's dense.c validation) whose M = 256 case runs it.
set -o pipefail
Q="--no-cpu-baseline --no-dense-baseline --no-bcsr --no-reference-order --no-other-configs --no-host-api --no-validate"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_mfma.py 2>&1 | tail -3 || exit 1
timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --config 5 $Q > gpurun_out/m.json 2>gpurun_out/m.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/m.json'));print('cfg5',round(d['ms_per_step'],4))"
timeout -k 10 400 python -u -m pytest -x -q --timeout 380 --timeout-method thread tests/test_reference_main_gpu.py 2>&1 | tail -3
grep -n 'validated at\|harness_wrap\|rc=\|Error at' gpurun_out/main_amd_out.txt | tail -8
