#!/bin/bash
# A/B of the pipeline's compute streams: AM_PIPE_STREAMS=1 (one stream) vs the default (two, alternating)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sab
for k in 1 2 3; do
  for ns in 1 2; do
    AM_PIPE_STREAMS=$ns timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --check 8 > gpurun_out/sab/${k}_$ns.log 2>&1 || { echo "streams=$ns failed"; tail -5 gpurun_out/sab/${k}_$ns.log; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/sab/${k}_$ns.log').read().strip().splitlines()[-1]); print('streams=$ns', round(d['value']/1e6,1), 'Mops/s', 'ms/step %.2f' % d['ms_per_step'], 'k_doc %.3f ms' % d['roofline']['avg_ms'], 'verified', d['verified_docs'], 'errors', d['errors'], 'digest', d['digest'])"
  done
done
