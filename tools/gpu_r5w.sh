#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
for lib in tools/clock/libam_w4.so tools/clock/libam_w3.so tools/clock/libam_w2.so; do
  if [ $lib = default ]; then unset AM_LIB_PATH; else export AM_LIB_PATH=$lib; fi
  timeout -k 10 300 python -u tools/c5_merge_probe.py >> $O/c5_waves.log 2>&1 || exit 1
  timeout -k 10 300 python -u tools/bench_mid.py --docs 8192 --steps 2 --check 0 --flags diff >> $O/mid_waves.log 2>&1 || exit 1
done
