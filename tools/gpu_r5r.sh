#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 300 python -u tools/batch_vs_oracle.py > $O/bvo.log 2>&1 || exit 1
AM_FAST=0 timeout -k 10 300 python -u tools/batch_vs_oracle.py --reps 2 > $O/bvo_general.log 2>&1 || exit 1
