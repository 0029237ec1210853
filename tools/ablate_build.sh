#!/bin/bash
# Build diagnostic variants of libvrhip into build_ab/ (timing only; outputs are WRONG).
# usage: tools/ablate_build.sh NAME "-DFLAG=.. -DFLAG2=.."
set -e
cd "$(dirname "$0")/../volume_renderer_amd/csrc"
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fno-slp-vectorize $2"
mkdir -p ../../build_ab/$1
for f in vr_capi vr_kernels; do hipcc $F -c $f.hip -o ../../build_ab/$1/$f.o & done
hipcc $F -DVR_MARCH_FAST=1 -c vr_march.hip -o ../../build_ab/$1/vr_march_fast.o &
hipcc $F -DVR_MARCH_FAST=0 -c vr_march.hip -o ../../build_ab/$1/vr_march_exact.o &
wait
hipcc --offload-arch=gfx950 -shared -o ../../build_ab/libvrhip_$1.so ../../build_ab/$1/*.o
