#!/bin/bash
# Build diagnostic / A-B variants of libvrhip into build_ab/libvrhip_NAME.so (select on the GPU
# box with VR_LIB_PATH=build_ab/libvrhip_NAME.so).  Only the fast-shading march objects (the
# default kernels) are rebuilt with the extra flags; the host, general-kernel and exact-variant
# objects are the in-tree build's (make -C volume_renderer_amd/csrc first).  Diagnostic
# -DVR_ABLATE builds give WRONG images.
# usage: tools/ablate_build.sh NAME "-DFLAG=.. -DFLAG2=.."
set -e
cd "$(dirname "$0")/../volume_renderer_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize $2"
mkdir -p ../../build_ab/$1
for k in 1 2 4; do
  hipcc $F -DVR_MARCH_FAST=1 -DVR_MARCH_K=$k -c vr_march.hip -o ../../build_ab/$1/vr_march_fast_k$k.o &
done
wait
hipcc --offload-arch=gfx950 -shared -o ../../build_ab/libvrhip_$1.so ../../build_ab/$1/*.o \
  vr_capi.o vr_kernels.o vr_volume_ops.o vr_march_exact_k*.o
