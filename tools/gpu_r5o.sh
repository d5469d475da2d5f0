#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
for f in none patch diff; do
timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 --steps 2 --check 2 --flags $f > $O/mid_$f.json 2> $O/mid_$f.err || exit 1
done
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/ -m gpu > $O/gpu_all.log 2>&1 || exit 1
