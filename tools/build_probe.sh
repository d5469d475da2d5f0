#!/bin/bash
# Probe variant of libautomerge_amd.so (never shipped): the phase clock build (-DAM_PHASE_CLOCK).
set -e
cd "$(dirname "$0")/../automerge_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics"
OUT=${1:-../../tools/clock}  # a directory gpurun does not skip when the build must travel (e.g. ../../phaseclock)
mkdir -p $OUT
make -s
/opt/rocm/bin/hipcc $F -DAM_PHASE_CLOCK -c am_kernels.hip -o /tmp/am_kernels_clock.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o $OUT/libam_clock.so /tmp/am_kernels_clock.o \
  am_capi.o am_sync.o am_inflate.o am_hist.o am_graph.o am_local.o am_sync_proto.o -lz -lpthread -lhsa-runtime64
echo built $OUT/libam_clock.so
