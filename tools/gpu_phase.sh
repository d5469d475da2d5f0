cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
AM_LIB_PATH=tools/clock/libam_clock.so timeout -k 10 300 python tools/phase_clock.py --docs ${1:-65536} --patch > gpurun_out/phase.log 2>&1
rc=$?; cat gpurun_out/phase.log; exit $rc
