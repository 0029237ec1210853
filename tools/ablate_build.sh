#!/bin/bash
# Build diagnostic / A-B variants of libvrhip into build_ab/libvrhip_NAME.so (select on the GPU
# box with VR_LIB_PATH=build_ab/libvrhip_NAME.so).  Diagnostic -DVR_ABLATE builds give WRONG images.
# usage: tools/ablate_build.sh NAME "-DFLAG=.. -DFLAG2=.."
set -e
cd "$(dirname "$0")/../volume_renderer_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize $2"
mkdir -p ../../build_ab/$1
for f in vr_capi vr_kernels; do hipcc $F -c $f.hip -o ../../build_ab/$1/$f.o & done
for v in 1:fast 0:exact; do for k in 1 2 4 8; do
  hipcc $F -DVR_MARCH_FAST=${v%:*} -DVR_MARCH_K=$k -c vr_march.hip -o ../../build_ab/$1/vr_march_${v#*:}_k$k.o &
done; done
wait
hipcc --offload-arch=gfx950 -shared -o ../../build_ab/libvrhip_$1.so ../../build_ab/$1/*.o
