#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
AM_DEBUG_WS_CANARY=64 AM_LIB_PATH=tools/dcheck/libam_dcheck.so timeout -k 10 300 python -u tools/patch_probe.py --runs 1 > $O/pprobe.log 2>&1
AM_DEBUG_WS_CANARY=64 AM_LIB_PATH=tools/dcheck/libam_dcheck.so timeout -k 10 300 python -u tools/mid_probe.py --docs 2048 --flags diff > $O/mprobe.log 2>&1 || exit 1
