#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_all.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_handles.py --docs 200000 --reps 3 > $O/handles2.json 2> $O/handles2.err || exit 1
AM_SYNC_PROFILE=1 timeout -k 10 500 python -u tools/bench_sync.py --pairs 100000 --e2e > $O/c5_e2e3.json 2> $O/c5_e2e3_stages.txt || exit 1
timeout -k 10 600 python -u bench.py > $O/bench4.json 2> $O/bench4.err || exit 1
