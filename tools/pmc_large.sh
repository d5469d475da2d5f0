#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / SQ passes of the general kernels (glb_mode::k_doc, k_diff) on large and
# mid-size documents (tools/large_doc_probe.py), one rocprofv3 --pmc run per group, never combined
# with tracing. Usage on the GPU box: bash tools/pmc_large.sh <tag>
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmc_large}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1 wl=$2; shift 2
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 $R/tools/large_doc_probe.py $wl --diff > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
run text_fetch "--text 1000 --docs 64" FETCH_SIZE && run text_write "--text 1000 --docs 64" WRITE_SIZE && \
run text_sq "--text 1000 --docs 64" $SQ && \
run mid_fetch "--mid --docs 2048" FETCH_SIZE && run mid_write "--mid --docs 2048" WRITE_SIZE && run mid_sq "--mid --docs 2048" $SQ
