#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 400 python -u bench.py --workload c2 --no-cpu-baseline > $O/c2_bench.json 2> $O/c2_bench.err || exit 1
timeout -k 10 300 python -u tools/bench_getpatch.py > $O/getpatch.json 2> $O/getpatch.err || exit 1
