#!/bin/bash
# A/B of k_doc builds (tools/ab/libam_<name>.so, tools/build_variants.sh) on C5 pairs (LDS mode, with
# and without the applyChanges patch) after the variants' parity runs. Usage: bash tools/gpu_ab_kdoc.sh tag name...
cd $GRAFT_REPO_ROOT
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for n in "$@"; do
  lib=$GRAFT_REPO_ROOT/tools/ab/libam_$n.so
  AM_LIB_PATH=$lib timeout -k 10 600 python -u -m pytest -m gpu -x -q --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_gpu_apply_patch.py tests/test_gpu_backend_batch.py > $O/tests_$n.log 2>&1 || { echo "$n tests failed"; tail -20 $O/tests_$n.log; exit 1; }
  echo "$n tests: $(tail -1 $O/tests_$n.log)"
done
for n in base "$@"; do
  lib=""; [ $n = base ] || lib=$GRAFT_REPO_ROOT/tools/ab/libam_$n.so
  for p in --no-patch ""; do
    AM_LIB_PATH=$lib timeout -k 10 200 python -u tools/c5_merge_probe.py $p > $O/c5_${n}_${p:-patch}.json 2>&1 || { echo "$n c5 failed"; tail -5 $O/c5_${n}_${p:-patch}.json; exit 1; }
    echo "$n $p $(tail -1 $O/c5_${n}_${p:-patch}.json)"
  done
done
