cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/gpu_tests.log
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  echo "smoke rc=$?"; tail -5 gpurun_out/smoke.log
fi
