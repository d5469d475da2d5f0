#!/bin/bash
# roofline.traffic of the headline command: one rocprofv3 --pmc pass per counter (FETCH_SIZE, then
# WRITE_SIZE) over bench.py's default (HBM-resident) C4 job; tools/traffic.py turns them into
# profiles/traffic_k_doc.json (per launch, gfx950 FETCH_SIZE correction, kernel-source digest).
R=$GRAFT_REPO_ROOT
TAG=${1:-traffic}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d $OUT/$c -o $c -- \
    python3 $R/bench.py --steps 2 --warmup 1 --mode resident --no-cpu-baseline --check 0 > $OUT/$c.log 2>&1 || { echo "$c pass failed"; tail -5 $OUT/$c.log; exit 1; }
  echo "$c ok"
done
cd $R && python3 tools/traffic.py $OUT $OUT/traffic_k_doc.json
