#!/bin/bash
# A/B of the global-mode k_doc occupancy on C3: default library vs tools/clock/libam_glb4.so
cd $GRAFT_REPO_ROOT
TAG=${1:-c3ab}; mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u tools/bench_text.py --steps 2 > gpurun_out/$TAG/w2.log 2>&1 || { tail -20 gpurun_out/$TAG/w2.log; exit 1; }
tail -1 gpurun_out/$TAG/w2.log | cut -c1-420
AM_LIB_PATH=$GRAFT_REPO_ROOT/tools/clock/libam_glb4.so timeout -k 10 300 python -u tools/bench_text.py --steps 2 > gpurun_out/$TAG/w4.log 2>&1 || { tail -20 gpurun_out/$TAG/w4.log; exit 1; }
tail -1 gpurun_out/$TAG/w4.log | cut -c1-420
