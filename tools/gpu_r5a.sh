#!/bin/bash
# round-5 check: host-link copy probe, pipeline tests, the bench line (pipe value + resident beside it)
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 120 ./tools/bin/copy_probe 1024 > $O/copy.json 2> $O/copy.err || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipe.py > $O/pipe_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 1 > $O/bench.json 2> $O/bench.err || exit 1
