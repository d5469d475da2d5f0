#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
AM_LIB_PATH=$PWD/tools/dcheck/libam_dcheck.so timeout -k 10 200 python -u tools/mid_probe.py --docs 512 --flags diff > $O/p8prof.log 2>&1 || exit 1
