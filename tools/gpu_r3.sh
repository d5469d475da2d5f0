#!/bin/bash
# round-3 GPU step: pipeline tests, then a short pipelined bench and the default bench
cd $GRAFT_REPO_ROOT
TAG=${1:-r3}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest -m gpu -x -v --timeout 120 --timeout-method thread tests/test_gpu_pipe.py > gpurun_out/$TAG/pipe_tests.log 2>&1 || { tail -40 gpurun_out/$TAG/pipe_tests.log; exit 1; }
tail -5 gpurun_out/$TAG/pipe_tests.log
timeout -k 10 300 python bench.py --docs 131072 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/$TAG/bench_131k.json 2> gpurun_out/$TAG/bench_131k.err || { tail -30 gpurun_out/$TAG/bench_131k.err; exit 1; }
cat gpurun_out/$TAG/bench_131k.json
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json
