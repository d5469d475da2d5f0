#!/bin/bash
# Probe variants of libautomerge_amd.so (never shipped): phase clock, and early-exit builds.
set -e
cd "$(dirname "$0")/../automerge_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics"
mkdir -p ../../tools/probe
make -s am_capi.o am_workload.o am_sync.o am_inflate.o
/opt/rocm/bin/hipcc $F -DAM_PHASE_CLOCK -c am_kernels.hip -o /tmp/am_kernels_clock.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o ../../tools/probe/libam_clock.so /tmp/am_kernels_clock.o am_capi.o am_sync.o am_inflate.o am_workload.o -lz -lpthread
echo built tools/probe/libam_clock.so
