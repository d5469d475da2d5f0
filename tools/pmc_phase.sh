#!/bin/bash
# Per-phase instruction counts of k_doc_fast: SQ_INSTS_VALU / SALU / LDS of the FD_STOP variants
# (tools/build_stop.sh) and of the full kernel. Usage on the GPU box: bash tools/pmc_phase.sh <tag>
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-phase}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for k in ${KS:-0 1 2 3 4 5 6 7 8 9 10 11 12 13 14 full}; do
  lib=$R/tools/stop/libam_stop$k.so
  [ "$k" = full ] && lib=$R/automerge_amd/libautomerge_amd.so
  AM_LIB_PATH=$lib timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv \
    -d $OUT/s$k -o s$k -- python3 $R/tools/pmc_phase.py 32768 > $OUT/s$k.log 2>&1 || { echo "stop $k failed"; exit 1; }
  echo "stop $k ok"
done
python3 $R/tools/pmc_summary_phase.py $OUT
