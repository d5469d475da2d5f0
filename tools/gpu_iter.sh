# GPU iteration: parity tests, phase-clock profile, 1-GPU bench (each step time-limited)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/gpu_tests.log
[ $rc -ne 0 ] && exit $rc
AM_LIB_PATH=tools/probe/libam_clock.so timeout -k 10 300 python tools/phase_clock.py --docs 65536 > gpurun_out/phase.log 2>&1
rc=$?; cat gpurun_out/phase.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --docs 262144 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
exit $rc
