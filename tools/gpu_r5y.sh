#!/bin/bash
set -o pipefail
O=gpurun_out/r5
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/c5prof -o c5 -- python3 -u tools/bench_sync.py --pairs 100000 --e2e > $O/c5_e2e_prof.json 2> $O/c5_e2e_prof.err || exit 1
