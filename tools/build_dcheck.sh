#!/bin/bash
# Diagnostics variant of libautomerge_amd.so (never shipped): the applyChanges-patch replay checks every
# index of its unchecked pools (-DAM_DIFF_CHECK) and reports an overrun as a patch status instead.
set -e
cd "$(dirname "$0")/../automerge_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics"
mkdir -p ../../tools/dcheck
make -s
/opt/rocm/bin/hipcc $F -DAM_DIFF_CHECK -c am_kernels.hip -o /tmp/am_kernels_dcheck.o
/opt/rocm/bin/hipcc $F -DAM_DIFF_CHECK -c am_capi.hip -o /tmp/am_capi_dcheck.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o ../../tools/dcheck/libam_dcheck.so /tmp/am_kernels_dcheck.o \
  /tmp/am_capi_dcheck.o am_sync.o am_inflate.o am_hist.o am_graph.o am_local.o am_sync_proto.o -lz -lpthread -lhsa-runtime64
echo built tools/dcheck/libam_dcheck.so
