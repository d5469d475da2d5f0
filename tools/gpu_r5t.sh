#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_pipe.py > $O/tests_pipe.log 2>&1 || exit 1
