#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pipe.py > $O/pipe2.log 2>&1 || exit 1
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/gpu_all.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 1 > $O/bench3.json 2> $O/bench3.err || exit 1
