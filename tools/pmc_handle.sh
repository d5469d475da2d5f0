#!/bin/bash
# SQ and instruction-cache counters of k_doc on the per-handle shape (one saved 100k-op text + one
# change, tools/phase_clock.py --handle 1000 --docs 1 on the phase-clock probe build): one rocprofv3
# --pmc run per group, never with tracing. Usage on the GPU box: bash tools/pmc_handle.sh <tag>
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-pmc_handle}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export AM_LIB_PATH=$R/${AM_PROBE_LIB:-phaseclock/libam_clock.so}
run() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o $name -- \
    python3 $R/tools/phase_clock.py --handle 1000 --docs 1 > $OUT/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc"
  return $rc
}
run sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS && \
run ic SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_VMEM
for f in $(find $OUT -name "*counter_collection.csv"); do
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(float)
for r in csv.DictReader(open(sys.argv[1])):
    if "k_doc" in r["Kernel_Name"] and "fast" not in r["Kernel_Name"]:
        acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(sys.argv[1].split("/")[-1], dict(acc))
PY
done
