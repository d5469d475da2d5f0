cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -25 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --docs 262144 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
