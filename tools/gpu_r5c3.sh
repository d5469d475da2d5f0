#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 1000 python -u tools/bench_text.py --docs 1000 --steps 3 > $O/c3_text.log 2>&1 || exit 1
