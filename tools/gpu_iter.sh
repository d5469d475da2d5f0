#!/bin/bash
# One GPU iteration: wave + parity tests, phase clock of the probe build, bench (no CPU baseline).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/it
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/it/gpu_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/it/gpu_tests.log; exit 1; }
tail -2 gpurun_out/it/gpu_tests.log
if [ -f tools/probe/libam_clock.so ]; then
  AM_LIB_PATH=tools/probe/libam_clock.so timeout -k 10 200 python tools/phase_clock.py --docs 131072 > gpurun_out/it/phase.log 2>&1 || { echo "phase failed"; tail -5 gpurun_out/it/phase.log; exit 1; }
  tail -16 gpurun_out/it/phase.log
fi
timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/it/bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/it/bench.log; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/it/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['stage_ms'])"
