#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_l.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_local.py --calls 10 > $O/local2.json 2> $O/local2.err || exit 1
timeout -k 10 400 python -u tools/bench_handles.py --docs 200000 --reps 3 > $O/handles3.json 2> $O/handles3.err || exit 1
