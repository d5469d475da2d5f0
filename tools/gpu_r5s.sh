#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5/smoke.log 2>&1 || exit 1
