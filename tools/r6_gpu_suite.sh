#!/bin/bash
# The full GPU suite (one process), its log under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu --maxfail=25 -q --timeout 120 --timeout-method thread ${PYTEST_EXTRA} \
    > gpurun_out/suite.log 2>&1
rc=$?
tail -25 gpurun_out/suite.log
exit $rc
