#!/bin/bash
set -o pipefail
bash tools/gpu_r5final.sh || exit 1
timeout -k 10 600 python -u tools/bench_local.py --calls 10 > gpurun_out/r5final/local.json 2> gpurun_out/r5final/local.err || exit 1
timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 --steps 2 --check 8 --flags diff > gpurun_out/r5final/mid_diff.json 2> gpurun_out/r5final/mid_diff.err || exit 1
timeout -k 10 300 python -u tools/patch_probe.py --runs 2 > gpurun_out/r5final/patch_probe.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/c5_merge_probe.py > gpurun_out/r5final/c5_merge.json 2>&1 || exit 1
AM_SYNC_PROFILE=1 timeout -k 10 500 python -u tools/bench_sync.py --pairs 100000 --e2e > gpurun_out/r5final/c5_e2e.json 2> gpurun_out/r5final/c5_e2e_stages.txt || exit 1
echo "extra ok"
