cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --docs 65536 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_small.log 2>&1
rc=$?; echo "bench_small rc=$rc"; tail -3 gpurun_out/bench_small.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --docs 262144 --steps 10 --warmup 2 > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.log
[ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1 -o c4 -- python3 $R/bench.py --docs 262144 --steps 5 --warmup 1 --no-cpu-baseline --check 0 > $R/gpurun_out/prof_r1.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -3 $R/gpurun_out/prof_r1.log; find $R/gpurun_out/prof_r1 -name "*.csv" | head
