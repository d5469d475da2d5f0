#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
AM_LIB_PATH=$PWD/tools/dcheck/libam_dcheck.so AM_DEBUG_WS_CANARY=4194304 timeout -k 10 200 python -u tools/mid_canary.py --docs 2048,2055,2141,2147,2237,2344,0,1 --flags diff > $O/dcheck.log 2>&1 || exit 1
