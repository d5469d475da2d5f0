#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
AM_LDS_BUDGET_KB=40 AM_SYNC_PROFILE=1 timeout -k 10 500 python -u tools/bench_sync.py --pairs 100000 --e2e > $O/c5_e2e_40.json 2> $O/c5_e2e_40_stages.txt || exit 1
AM_LDS_BUDGET_KB=40 timeout -k 10 300 python -u tools/c5_merge_probe.py > $O/c5_merge_40.json 2>&1 || exit 1
