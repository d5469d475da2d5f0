#!/bin/bash
# Round profile on the GPU box: gpu tests, the default bench (with CPU baseline), rocprofv3
# kernel-trace stats of the same bench, and the FETCH_SIZE / WRITE_SIZE passes that give
# roofline.traffic. Usage: bash tools/gpu_prof.sh <tag>   (outputs under gpurun_out/<tag>)
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo "bench failed"; tail -5 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- \
  python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --check 0 > $OUT/stats.log 2>&1 || { echo "rocprof failed"; tail -5 $OUT/stats.log; exit 1; }
tail -1 $OUT/stats.log
for pass in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $OUT/$pass -o $pass -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --check 0 > $OUT/$pass.log 2>&1 || { echo "pmc $pass failed"; tail -5 $OUT/$pass.log; exit 1; }
done
echo "prof done"
