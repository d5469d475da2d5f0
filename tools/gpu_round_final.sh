#!/bin/bash
# Round-end measurements on the GPU box: the default bench, its rocprofv3 kernel-trace stats,
# the PMC passes behind roofline.traffic (then the bench again, which reports them), the SQ
# instruction counters of k_doc_fast, and the host-link copy probe. Outputs under gpurun_out/<tag>.
#   gpurun -- bash tools/gpu_round_final.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
echo "tests ok"
timeout -k 10 400 python3 -u bench.py > $O/bench_a.json 2> $O/bench_a.err || { echo "bench failed"; exit 1; }
echo "bench a ok"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -o bench -- \
  python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --check 0 > $O/stats.log 2>&1 || { echo "rocprof stats failed"; exit 1; }
echo "stats ok"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/$c -o $c -- \
    python3 $R/bench.py --mode resident --steps 2 --warmup 1 --no-cpu-baseline --check 0 > $O/$c.log 2>&1 || { echo "$c pass failed"; exit 1; }
  echo "$c ok"
done
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
  --output-format csv -d $O/sq -o sq -- python3 $R/bench.py --mode resident --steps 2 --warmup 1 --no-cpu-baseline --check 0 > $O/sq.log 2>&1 || { echo "sq pass failed"; exit 1; }
echo "sq ok"
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "gpu tests failed"; exit 1; }
echo "tests ok"
python3 tools/traffic.py $O profiles/traffic_k_doc.json > $O/traffic.log 2>&1 || { echo "traffic.py failed"; exit 1; }
cp profiles/traffic_k_doc.json $O/traffic_k_doc.json
timeout -k 10 400 python3 -u bench.py > $O/bench_b.json 2> $O/bench_b.err || { echo "bench b failed"; exit 1; }
echo "bench b ok"
timeout -k 10 120 tools/bin/copy_probe 1024 > $O/copy_probe.json 2> $O/copy_probe.err || { echo "copy probe failed"; exit 1; }
echo "all ok"
