#!/bin/bash
# Probe variants of libautomerge_amd.so (never shipped): k_doc_fast returns after phase k
# (-DFD_STOP=k), for per-phase instruction counts (tools/pmc_phase.sh).
set -e
cd "$(dirname "$0")/../automerge_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics"
mkdir -p ../../tools/stop
make -s
for k in ${*:-0 1 2 3 4 5 6 7 8 9 10 11 12 13 14}; do
  ( /opt/rocm/bin/hipcc $F -DFD_STOP=$k -c am_kernels.hip -o /tmp/am_kernels_stop$k.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o ../../tools/stop/libam_stop$k.so /tmp/am_kernels_stop$k.o \
      am_capi.o am_sync.o am_inflate.o am_hist.o am_graph.o am_local.o am_sync_proto.o -lz -lpthread -lhsa-runtime64 ) &
  while [ $(jobs -r | wc -l) -ge 8 ]; do sleep 1; done
done
wait
ls ../../tools/stop/
