#!/bin/bash
# A/B bench of probe variants: bash tools/gpu_ab.sh name1 name2 ...  ("base" = the in-tree library,
# "env:VAR=value" = the in-tree library with that environment variable)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
i=0
for n in "$@"; do
  i=$((i+1))
  ev=""
  if [ "$n" = base ]; then lib=""; elif [ "${n#env:}" != "$n" ]; then lib=""; ev="${n#env:}"; else lib=$GRAFT_REPO_ROOT/tools/probe/libam_$n.so; fi
  env $ev AM_LIB_PATH=$lib timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-pcie --check 8 > gpurun_out/ab/${i}.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab/${i}.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ab/${i}.log').read().strip().splitlines()[-1]); print('$n', round(d['value']/1e6,1), 'Mops/s', 'k_doc %.3f ms' % d['roofline']['avg_ms'], 'verified', d['verified_docs'], 'errors', d['errors'])"
done
