#!/bin/bash
# One GPU call: all -m gpu tests, smoke, the default bench line, and a rocprofv3 kernel-trace summary of it.
cd $GRAFT_REPO_ROOT
TAG=${1:-r3}; mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -m gpu -x -v --timeout 300 --timeout-method thread tests > gpurun_out/$TAG/gpu_tests.log 2>&1 || { tail -60 gpurun_out/$TAG/gpu_tests.log; exit 1; }
tail -3 gpurun_out/$TAG/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -30 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/$TAG/bench.json 2> gpurun_out/$TAG/bench.err || { tail -30 gpurun_out/$TAG/bench.err; exit 1; }
cut -c1-1500 gpurun_out/$TAG/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --no-cpu-baseline --check 4 > gpurun_out/$TAG/bench_prof.json 2> gpurun_out/$TAG/bench_prof.err || { tail -20 gpurun_out/$TAG/bench_prof.err; exit 1; }
find gpurun_out/$TAG/prof -name "*stats*.csv"
timeout -k 10 300 python tools/bench_history.py > gpurun_out/$TAG/history_bench.json 2>&1 || { tail -20 gpurun_out/$TAG/history_bench.json; exit 1; }
cat gpurun_out/$TAG/history_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$TAG/hprof -o run -- python3 tools/bench_history.py --reps 2 > gpurun_out/$TAG/history_prof.json 2>&1 || { tail -20 gpurun_out/$TAG/history_prof.json; exit 1; }
find gpurun_out/$TAG/hprof -name "*stats*.csv"
