#!/bin/bash
# GPU tests only: bash tools/gpu_test.sh <tag> [pytest selectors...]
cd $GRAFT_REPO_ROOT
TAG=${1:-t}; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread "${@:-tests}" > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/$TAG/gpu_tests.log | tail -40
[ $rc -ne 0 ] && grep -E "^E " gpurun_out/$TAG/gpu_tests.log | head -30
exit $rc
