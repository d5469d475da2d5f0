#!/bin/bash
# SQ issue / wait counters of k_doc_fast on one C4 batch with patches (tools/pmc_phase.py).
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-sq}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS \
  --output-format csv -d $OUT/a -o a -- python3 $R/tools/pmc_phase.py 131072 > $OUT/a.log 2>&1 || { echo "pass a failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM \
  --output-format csv -d $OUT/b -o b -- python3 $R/tools/pmc_phase.py 131072 > $OUT/b.log 2>&1 || { echo "pass b failed"; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
tot = {}
for p in ("a", "b"):
    f = glob.glob(os.path.join(out, p, "**", "*counter_collection.csv"), recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "k_doc_fast" in r.get("Kernel_Name", ""):
            tot[(p, r["Counter_Name"])] = tot.get((p, r["Counter_Name"]), 0.0) + float(r["Counter_Value"])
for (p, k), v in sorted(tot.items()):
    w = tot.get((p, "SQ_WAVES"), 1)
    print("%s %-22s total %14.0f  per wave %10.1f" % (p, k, v, v / w))
PY
