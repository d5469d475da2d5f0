#!/bin/bash
# instruction-fetch counters of k_doc_fast on one C4 batch with patches (tools/pmc_phase.py): one
# rocprofv3 pass for the SQ fetch counters, one for the SQC instruction-cache counters.
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-icache}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_IFETCH_LEVEL SQ_WAVE_CYCLES \
  --output-format csv -d $OUT/c -o c -- python3 $R/tools/pmc_phase.py 131072 > $OUT/c.log 2>&1 || { echo "pass c failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
  --output-format csv -d $OUT/d -o d -- python3 $R/tools/pmc_phase.py 131072 > $OUT/d.log 2>&1 || { echo "pass d failed"; exit 1; }
python3 $R/tools/pmc_summary.py $OUT k_doc_fast
