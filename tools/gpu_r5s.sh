#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u tools/pipe_vs_oracle.py > $O/pvo.log 2>&1 || exit 1
AM_PIPE_ENGINES=0 timeout -k 10 300 python -u tools/pipe_vs_oracle.py > $O/pvo_noeng.log 2>&1 || exit 1
