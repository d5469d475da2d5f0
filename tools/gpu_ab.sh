#!/bin/bash
# A/B bench of probe variants: bash tools/gpu_ab.sh name1 name2 ...  ("base" = the in-tree library)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for n in "$@"; do
  if [ "$n" = base ]; then lib=""; else lib=$GRAFT_REPO_ROOT/tools/probe/libam_$n.so; fi
  AM_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --check 8 > gpurun_out/ab/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab/$n.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab/$n.log').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,1), 'Mops/s', {k: round(v,3) for k,v in d['stage_ms'].items()}, d.get('kernel_info'))"
done
