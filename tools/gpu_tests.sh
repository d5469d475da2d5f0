#!/bin/bash
# GPU test step: the named test files (default: all -m gpu tests), one pytest process, per-test timeout
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r3}; mkdir -p gpurun_out/$TAG
FILES=${*:-tests}
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $FILES > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
tail -60 gpurun_out/$TAG/gpu_tests.log
exit $rc
