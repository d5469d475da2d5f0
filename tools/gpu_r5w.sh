#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_w.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/c5_merge_probe.py > $O/c5_merge_lds.json 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 --steps 2 --check 8 --flags diff > $O/mid_lds.json 2>&1 || exit 1
