#!/bin/bash
# GPU round step: the -m gpu suite (one pytest process, per-test timeout), then the default bench
# line. TAG names the output directory under gpurun_out/.
#   gpurun -- 'TAG=r6x bash tools/gpu_suite_bench.sh [test files]'
cd $GRAFT_REPO_ROOT
TAG=${TAG:-r6}; mkdir -p gpurun_out/$TAG
FILES=${*:-tests}
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread $FILES > gpurun_out/$TAG/gpu_tests.log 2>&1
rc=$?
tail -30 gpurun_out/$TAG/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err
rc=$?
tail -c 3000 gpurun_out/$TAG/bench.json; tail -5 gpurun_out/$TAG/bench.err
exit $rc
