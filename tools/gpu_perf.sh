#!/bin/bash
# k_doc_fast iteration: GPU parity tests of the fast path, total instructions per wave (PMC), a
# resident-mode C4 bench (kernel stage times). Usage: bash tools/gpu_perf.sh <tag>
cd $GRAFT_REPO_ROOT
TAG=${1:-perf}; mkdir -p gpurun_out/$TAG
timeout -k 10 400 python -u -m pytest -m gpu -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_apply_patch.py tests/test_gpu_pipe.py tests/test_gpu_newbackend.py > gpurun_out/$TAG/tests.log 2>&1 || { tail -30 gpurun_out/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/$TAG/tests.log
KS=full bash tools/pmc_phase.sh $TAG/pmc > gpurun_out/$TAG/pmc.txt 2>&1 || { cat gpurun_out/$TAG/pmc.txt; exit 1; }
cat gpurun_out/$TAG/pmc.txt | tail -2
timeout -k 10 300 python bench.py --mode resident --docs 131072 --steps 10 --warmup 2 --no-cpu-baseline --check 8 > gpurun_out/$TAG/resident.json 2> gpurun_out/$TAG/resident.err || { tail -20 gpurun_out/$TAG/resident.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/$TAG/resident.json')); print('value', d['value'], 'stage_ms', d.get('stage_ms'), 'fast', d.get('fast_docs'))"
