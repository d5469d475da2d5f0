#!/bin/bash
# round-5 check: mid tests, the bench line, the mid bench, copy probe
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_mid.py > $O/tests_d.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --steps 6 --warmup 1 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 > $O/mid.json 2> $O/mid.err || exit 1
timeout -k 10 120 ./tools/bin/copy_probe 1024 > $O/copy2.json 2> $O/copy2.err || exit 1
