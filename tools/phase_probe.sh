cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for n in 1 2 3 4 5; do
  AM_LIB_PATH=$GRAFT_REPO_ROOT/tools/probe/libam_stop$n.so timeout -k 10 120 python bench.py --docs 65536 --steps 3 --warmup 1 --no-cpu-baseline --check 0 > gpurun_out/probe$n.log 2>&1 || { echo "probe $n failed"; tail -3 gpurun_out/probe$n.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/probe$n.log').read().strip().splitlines()[-1]); print($n, d['stage_ms'])"
done
