#!/bin/bash
# Large-document path: the GPU text tests, then C3 at full size (tools/bench_text.py).
cd $GRAFT_REPO_ROOT
TAG=${1:-c3}; mkdir -p gpurun_out/$TAG
timeout -k 10 500 python -u -m pytest -m gpu -x -q --timeout 400 --timeout-method thread tests/test_gpu_text.py tests/test_gpu_parity.py > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
timeout -k 10 500 python -u tools/bench_text.py --steps 3 > gpurun_out/$TAG/bench_text.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_text.log; exit 1; }
tail -1 gpurun_out/$TAG/bench_text.log | cut -c1-700
