#!/bin/bash
# Sequential GPU steps, each under its own time limit, stopping at the first failure.
# Usage: bash tools/gpu_seq.sh <tag> "<step 1>" "<step 2>" ...   (outputs under gpurun_out/<tag>)
cd $GRAFT_REPO_ROOT
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
i=0
for step in "$@"; do
  i=$((i+1))
  echo "== step $i: $step"
  timeout -k 10 280 bash -c "$step" > $OUT/step$i.log 2>&1
  rc=$?
  tail -15 $OUT/step$i.log
  if [ $rc -ne 0 ]; then echo "step $i failed rc=$rc"; exit $rc; fi
done
