#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python -u tools/bench_handles.py --docs 200000 --reps 3 > $O/handles.json 2> $O/handles.err || exit 1
AM_SYNC_PROFILE=1 timeout -k 10 500 python -u tools/bench_sync.py --pairs 100000 --e2e > $O/c5_e2e.json 2> $O/c5_e2e_stages.txt || exit 1
