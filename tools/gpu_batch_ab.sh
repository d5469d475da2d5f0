#!/bin/bash
# pipeline batch size sweep of the default C4 bench (fill / drain of the H2D-bound pipeline)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bab
for bs in 131072 65536 32768 16384; do
  timeout -k 10 150 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --check 8 --batch $bs > gpurun_out/bab/$bs.log 2>&1 || { echo "batch=$bs failed"; tail -5 gpurun_out/bab/$bs.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bab/$bs.log').read().strip().splitlines()[-1]); print('batch=$bs', round(d['value']/1e6,1), 'Mops/s', 'ms/step %.2f' % d['ms_per_step'], 'k_doc %.3f ms' % d['roofline']['avg_ms'], 'kernel ms/step %.2f' % d['kernel_ms_per_step'], 'verified', d['verified_docs'], 'errors', d['errors'])"
done
