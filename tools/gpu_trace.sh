#!/bin/bash
# kernel + memory-copy trace of one pipelined bench step (timeline of H2D / kernels / D2H)
cd $GRAFT_REPO_ROOT
TAG=${1:-trace}; shift
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --check 4 "$@" > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -20 gpurun_out/$TAG/bench.err; exit 1; }
cat gpurun_out/$TAG/bench.json | cut -c1-400
find gpurun_out/$TAG/prof -name "*.csv" | head -20
