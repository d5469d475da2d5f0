#!/bin/bash
# Round-4 capture in one GPU call: tools/gpu_full.sh (all -m gpu tests, smoke, bench line + its
# rocprofv3 kernel stats, history bench), the applyLocalChange latency, the C3 bench and the
# k_doc traffic passes.
cd $GRAFT_REPO_ROOT
TAG=${1:-r4final}
bash tools/gpu_full.sh $TAG || exit 1
timeout -k 10 300 python -u tools/bench_local.py > gpurun_out/$TAG/local.txt 2>&1 || { tail -20 gpurun_out/$TAG/local.txt; exit 1; }
tail -1 gpurun_out/$TAG/local.txt | cut -c1-600
timeout -k 10 600 python -u tools/bench_text.py --steps 3 > gpurun_out/$TAG/bench_text.log 2>&1 || { tail -20 gpurun_out/$TAG/bench_text.log; exit 1; }
tail -1 gpurun_out/$TAG/bench_text.log | cut -c1-800
bash tools/gpu_traffic.sh $TAG/traffic || exit 1
