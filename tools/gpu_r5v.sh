#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_apply_patch.py tests/test_gpu_mid.py tests/test_gpu_text.py tests/test_gpu_backend_batch.py > $O/tests_v.log 2>&1 || exit 1
AM_DIFF_MODE=wide timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_apply_patch.py tests/test_gpu_backend_batch.py > $O/tests_v_wide.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 --steps 2 --check 8 --flags diff > $O/mid_diff_lane0.json 2> $O/mid_diff3.err || exit 1
AM_DIFF_MODE=wide timeout -k 10 300 python -u tools/bench_mid.py --docs 512 --steps 2 --check 8 --flags diff > $O/mid_diff_wide512.json 2> $O/mid_diff3.err || exit 1
AM_DIFF_MODE=lane0 timeout -k 10 300 python -u tools/bench_mid.py --docs 512 --steps 2 --check 8 --flags diff > $O/mid_diff_lane0_512.json 2> $O/mid_diff3.err || exit 1
timeout -k 10 300 python -u tools/patch_probe.py --runs 2 > $O/pprobe0.log 2>&1 || exit 1
