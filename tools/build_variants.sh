#!/bin/bash
# Probe variants of libautomerge_amd.so for A/B runs on the GPU (never shipped):
#   tools/probe/libam_<name>.so built with extra flags. Usage: tools/build_variants.sh name "-DFOO=1" [...]
set -e
cd "$(dirname "$0")/../automerge_amd/csrc"
F="-O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics"
OUT=${OUTDIR:-../../tools/probe}  # a directory gpurun does not skip when the build must travel
mkdir -p $OUT
make -s am_capi.o am_sync.o am_inflate.o am_hist.o am_graph.o am_local.o am_sync_proto.o
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc $F $flags -c am_kernels.hip -o /tmp/am_kernels_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -fPIC -shared -o $OUT/libam_$name.so /tmp/am_kernels_$name.o am_capi.o am_sync.o am_inflate.o am_hist.o am_graph.o am_local.o am_sync_proto.o -lz -lpthread -lhsa-runtime64
  echo built $OUT/libam_$name.so
done
