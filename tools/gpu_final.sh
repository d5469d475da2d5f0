#!/bin/bash
# Round-end capture in one GPU call: all -m gpu tests, smoke, the default bench line and its
# rocprofv3 kernel stats, the history bench, the k_doc traffic passes and the C3 bench.
cd $GRAFT_REPO_ROOT
TAG=${1:-final}
bash tools/gpu_full.sh $TAG || exit 1
bash tools/gpu_traffic.sh $TAG/traffic || exit 1
timeout -k 10 600 python -u tools/bench_text.py --steps 3 > gpurun_out/$TAG/bench_text.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_text.log; exit 1; }
tail -1 gpurun_out/$TAG/bench_text.log | cut -c1-600
