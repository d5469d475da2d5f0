#!/bin/bash
# PMC passes over the 1-GPU bench (one rocprofv3 --pmc run per counter group; never combined with
# tracing). Usage on the GPU box: bash tools/pmc.sh <tag> [docs]
R=$GRAFT_REPO_ROOT
TAG=${1:-pmc}
DOCS=${2:-131072}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 $R/bench.py --docs $DOCS --steps 2 --warmup 1 --no-cpu-baseline --check 0 > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run fetch FETCH_SIZE && run write WRITE_SIZE && \
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS && \
run sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE
